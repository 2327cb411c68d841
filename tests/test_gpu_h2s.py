"""The in-kernel half-pair GEMMs (gnnmp.h GNN_MATH_HALF_PAIR, ABI 23; gemm_x3.hip NPL = 2 / H2S):
f32 operands split into f16 hi / lo while staging, with per-row (NT) and per-block (TN) power-of-two
scales, 3 products.  SAGE-ResBN's hidden layers run on them (conv._SAGEAggregateFirst).  Checked
against float64 at relL2 <= 1e-6 (the split-bf16 form's own error is ~2e-7) over rows whose
magnitudes span 1e-7 .. 1e4, zero rows, and M with a short last row block."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def _rows(M, K, gen, spread=True):
    a = torch.randn(M, K, generator=gen, dtype=torch.float64)
    if spread:  # per-row magnitudes 1e-7 .. 1e4, a few zero rows
        mag = 10.0 ** torch.empty(M, 1, dtype=torch.float64).uniform_(-7, 4, generator=gen)
        a = a * mag
        a[::97] = 0.0
    return a


@pytest.mark.parametrize("M,k1,k2,N", [(5000, 64, 64, 64), (203, 64, 0, 128), (4097, 32, 48, 96), (128, 16, 16, 128)])
def test_h2s_nt_vs_f64(device, M, k1, k2, N):
    from elliptic_gnn_project_amd.fused import gemm_nt, h2s_nt_ok

    assert h2s_nt_ok(N, k1, k2)
    g = torch.Generator().manual_seed(M + N)
    a1 = _rows(M, k1, g)
    a2 = _rows(M, k2, g) if k2 else None
    w1 = torch.randn(N, k1, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(N, k2, generator=g, dtype=torch.float64) * 0.1 if k2 else None
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    ref = a1 @ w1.t() + bias
    if k2:
        ref = ref + a2 @ w2.t()
    dv = lambda t: t.float().to(device) if t is not None else None  # noqa: E731
    rexp = torch.empty(M, dtype=torch.int32, device=device)
    y = gemm_nt(dv(a1), None, N, a2=dv(a2), bias=dv(bias), w1=dv(w1), w2=dv(w2), math="half_pair", row_exp=rexp)
    torch.cuda.synchronize()
    # row-relative accuracy: every row against its own scale (rows span 11 decades)
    A = torch.cat([a1.float().double()] + ([a2.float().double()] if k2 else []), 1)
    W = torch.cat([w1.float().double()] + ([w2.float().double()] if k2 else []), 1)
    ref32 = A @ W.t() + bias.float().double()  # the f32 inputs exactly
    err = (y.double().cpu() - ref32).abs()
    scale = (A.abs() @ W.abs().t()).amax(1, keepdim=True) + bias.abs().float().double().max()
    assert float((err / scale).max()) < 2e-6
    assert _rel(y, ref32) < 1e-6
    # the row exponents: max |A[r, :]| < 2^E_r (numpy frexp), 0 for zero rows
    mx = A.abs().amax(1).numpy()
    _, e = np.frexp(mx)
    np.testing.assert_array_equal(rexp.cpu().numpy(), np.where(mx > 0, e, 0).astype(np.int32))
    # the split-bf16 form of the same call agrees to its own accuracy
    y3 = gemm_nt(dv(a1), None, N, a2=dv(a2), bias=dv(bias), w1=dv(w1), w2=dv(w2))
    assert _rel(y3, ref32) < 1e-6


def test_h2s_nt_epilogue_matches_split(device):
    """ReLU + dropout + projection epilogue after the row / column unscale: the same keep bits as the
    split-bf16 kernel (the shared epilogue), values within fp32 rounding."""
    from elliptic_gnn_project_amd.fused import gemm_nt

    g = torch.Generator().manual_seed(3)
    M, K, N = 3001, 64, 128
    a = torch.randn(M, K, generator=g).to(device)
    w = (torch.randn(N, K, generator=g) * 0.1).to(device)
    b = torch.randn(N, generator=g).to(device)
    proj = torch.randn(4, N, generator=g).to(device)
    z1 = torch.empty(M, 4, device=device)
    z2 = torch.empty(M, 4, device=device)
    kw = dict(bias=b, relu=True, dropout_p=0.5, seed=77, w1=w, proj=proj)
    y1 = gemm_nt(a, None, N, math="half_pair", z=z1, **kw)
    y2 = gemm_nt(a, None, N, z=z2, **kw)
    assert torch.equal(y1 == 0, y2 == 0) or float(((y1 == 0) != (y2 == 0)).float().mean()) < 1e-5
    assert _rel(y1, y2) < 1e-6
    assert _rel(z1, z2) < 1e-6


@pytest.mark.parametrize("M,k1,k2,Nr", [(5000, 64, 64, 64), (70001, 64, 64, 64), (1000, 96, 0, 128), (17, 32, 32, 64)])
def test_h2s_tn_vs_f64(device, M, k1, k2, Nr):
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_tn

    g = torch.Generator().manual_seed(M + Nr)
    a1 = _rows(M, k1, g)
    a2 = _rows(M, k2, g) if k2 else None
    gg = _rows(M, Nr, g)  # G rows spread too (the per-block G bound)
    dv = lambda t: t.float().to(device) if t is not None else None  # noqa: E731
    # the row exponents of [a1 | a2] from the forward NT, as the conv saves them
    rexp = torch.empty(M, dtype=torch.int32, device=device)
    w1 = torch.randn(8 * 2, k1, generator=g).to(device)
    w2 = torch.randn(16, k2, generator=g).to(device) if k2 else None
    gemm_nt(dv(a1), None, 16, a2=dv(a2), w1=w1, w2=w2, math="half_pair", row_exp=rexp)
    (d1, d2), db, _, _ = gemm_tn(Nr, dv(a1), dv(a2), g=dv(gg), math="half_pair", row_exp=rexp)
    torch.cuda.synchronize()
    G = gg.float().double()
    r1 = G.t() @ a1.float().double()
    assert _rel(d1, r1) < 1e-6
    if k2:
        assert _rel(d2, G.t() @ a2.float().double()) < 1e-6
    assert _rel(db, G.sum(0)) < 1e-6
    # and the split-bf16 TN of the same call
    (e1, _), _, _, _ = gemm_tn(Nr, dv(a1), dv(a2), g=dv(gg))
    assert _rel(e1, r1) < 1e-6


def test_h2s_row_exp_needs_the_half_pair_form(device):
    """A caller asking for row_exp gets it or an error — never a silently unwritten buffer."""
    from elliptic_gnn_project_amd.fused import gemm_nt

    a = torch.randn(100, 20, device=device)  # k1 = 20: not a multiple of 16
    w = torch.randn(64, 20, device=device)
    rexp = torch.empty(100, dtype=torch.int32, device=device)
    with pytest.raises(NotImplementedError):
        gemm_nt(a, None, 64, w1=w, math="half_pair", row_exp=rexp)
    with pytest.raises(NotImplementedError):
        gemm_nt(torch.randn(100, 32, device=device), None, 64, w1=torch.randn(64, 32, device=device),
                row_exp=rexp)  # split-bf16 math


def test_sage_resbn_step_h2s_vs_split(device):
    """SAGE-ResBN (configs[3] shape, 5,000 nodes): the train step's logits and gradients with the hidden
    layers on the half-pair GEMMs equal the split-bf16 step's to fp32 accuracy."""
    from elliptic_gnn_project_amd import conv
    from elliptic_gnn_project_amd.train_gnn import build_model
    from elliptic_gnn_project_amd.fused import gemm_nt  # noqa: F401  (library loaded)

    N, E, F = 5000, 12000, 165
    g = torch.Generator().manual_seed(9)
    x = torch.randn(N, F, generator=g).to(device)
    ei = torch.randint(0, N, (2, E), generator=g).to(device)
    ei = torch.cat([ei, ei.flip(0)], 1)
    t_idx = torch.randint(0, 49, (N,), generator=g).to(device)
    cfg = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.0, time_embed_dim=2,
               time_embed_type="sin", max_timestep=49)
    out = {}
    for h2 in (True, False):
        conv._H2S = h2
        torch.manual_seed(1)
        m = build_model("sage_resbn", F, cfg).to(device).train()
        logits = m(x, ei, t_idx)
        (logits.square().sum()).backward()
        out[h2] = (logits.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    conv._H2S = True
    assert _rel(out[True][0], out[False][0]) < 1e-6
    for k in out[False][1]:
        ref = out[False][1][k]
        if k.startswith("convs.") and k.endswith("lin_l.bias") and not k.startswith("convs.2."):
            # a hidden conv's bias feeds BatchNorm: its true gradient is exactly zero, both steps hold
            # rounding noise (~1e-5 absolute here)
            assert float(out[True][1][k].abs().max()) < 1e-3 and float(ref.abs().max()) < 1e-3, k
            continue
        assert _rel(out[True][1][k], ref) < 1e-5, k
