"""GPU parity of the fp32 MFMA GEMM kernels (K7) and the fused SAGENet path.

GEMMs are floating-point kernels: compared with a plain torch fp32 reference on the CPU
(rtol=atol=1e-5 at these magnitudes), in both arithmetic modes: "split_bf16" (the default:
hi+mid+lo bf16 terms on the bf16 matrix cores) and "f32" (exact f32 MFMA).  The fused network is compared with the CPU oracle
in eval mode and in train mode with dropout, using oracle/dropout_hash.py's bit-exact mask.
"""
import numpy as np
import pytest
import torch

from oracle import pyg_ref
from oracle.dropout_hash import keep_mask

pytestmark = pytest.mark.gpu


def rel_l2(a, b, floor=1e-7):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), floor / 1e-5))


@pytest.mark.parametrize("M,k1,k2,n", [(1000, 166, 166, 128), (257, 5, 0, 3), (4097, 128, 128, 128),
                                       (300, 64, 64, 256), (129, 33, 17, 130), (64, 1, 0, 1)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "dropout", "proj"])
@pytest.mark.parametrize("wform", [False, True])
def test_gemm_nt(device, M, k1, k2, n, epi, wform):
    from elliptic_gnn_project_amd.fused import gemm_nt

    if epi == "proj" and n > 128:
        pytest.skip("projection needs N <= 128")
    g = torch.Generator().manual_seed(M + k1 + n)
    a1 = torch.randn(M, k1, generator=g)
    a2 = torch.randn(M, k2, generator=g) if k2 else None
    bt = torch.randn(k1 + k2, n, generator=g) / (k1 + k2) ** 0.5
    bias = torch.randn(n, generator=g)
    proj = torch.randn(4, n, generator=g)
    A = torch.cat([a1, a2], 1) if k2 else a1
    ref = A @ bt
    kw = {}
    p = 0.0
    if epi != "plain":
        ref = torch.relu(ref + bias)
        kw = dict(bias=bias.to(device), relu=True)
    if epi == "dropout":
        p = 0.3
        m = torch.from_numpy(keep_mask(1234, M, n, p))
        ref = ref * m / (1 - np.float32(p))
        kw.update(dropout_p=p, seed=1234)
    z = None
    if epi == "proj":
        z = torch.empty(M, 4, device=device)
        kw.update(proj=proj.to(device), z=z)
    if wform:  # B read in place from Linear weights W [n, k] (the split-bf16 path when n <= 128)
        kw.update(w1=bt[:k1].t().contiguous().to(device), w2=bt[k1:].t().contiguous().to(device) if k2 else None)
        if n > 128:
            pytest.skip("w1/w2 form needs N <= 128")
    c = gemm_nt(a1.to(device), None if wform else bt.to(device), n,
                a2=a2.to(device) if a2 is not None else None, **kw)
    torch.testing.assert_close(c.cpu(), ref, rtol=1e-5, atol=1e-5)
    if epi == "proj":
        torch.testing.assert_close(z.cpu(), ref @ proj.t(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,k1,k2,n", [(1000, 166, 166, 128), (300, 7, 9, 33), (4097, 128, 0, 64)])
@pytest.mark.parametrize("math", ["split_bf16", "f32"])
def test_gemm_nt_weight_layout(device, M, k1, k2, n, math):
    """B read in place from PyTorch Linear weights (w1/w2) vs B from the transposed copy."""
    from elliptic_gnn_project_amd.fused import gemm_nt

    g = torch.Generator().manual_seed(M + n)
    a1 = torch.randn(M, k1, generator=g)
    a2 = torch.randn(M, k2, generator=g) if k2 else None
    w1 = torch.randn(n, k1, generator=g) / (k1 + k2) ** 0.5
    w2 = torch.randn(n, k2, generator=g) / (k1 + k2) ** 0.5 if k2 else None
    A = torch.cat([a1, a2], 1) if k2 else a1
    W = torch.cat([w1, w2], 1) if k2 else w1
    c = gemm_nt(a1.to(device), None, n, a2=a2.to(device) if k2 else None, w1=w1.to(device),
                w2=w2.to(device) if k2 else None, math=math)
    c2 = gemm_nt(a1.to(device), W.t().contiguous().to(device), n, a2=a2.to(device) if k2 else None, math=math)
    if math == "f32":
        assert torch.equal(c, c2)  # the same k-ordered fmaf chain
    torch.testing.assert_close(c.cpu(), A @ W.t(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c2.cpu(), A @ W.t(), rtol=1e-5, atol=1e-5)


def test_gemm_split_bf16_accuracy_vs_f64(device):
    """The split-bf16 product keeps fp32 accuracy: error vs a float64 reference is no larger than
    the exact-f32 MFMA's (Elliptic layer-1 shape, both K segments)."""
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_tn

    g = torch.Generator().manual_seed(7)
    M, F, n = 20000, 166, 128
    a1, a2 = torch.randn(M, F, generator=g), torch.randn(M, F, generator=g)
    w1, w2 = torch.randn(n, F, generator=g) * 0.08, torch.randn(n, F, generator=g) * 0.08
    ref = (torch.cat([a1, a2], 1).double() @ torch.cat([w1, w2], 1).double().t())
    errs = {}
    for math in ("split_bf16", "f32"):
        c = gemm_nt(a1.to(device), None, n, a2=a2.to(device), w1=w1.to(device), w2=w2.to(device), math=math)
        errs[math] = rel_l2(c, ref)
    assert errs["split_bf16"] < 1e-6 and errs["split_bf16"] < 2 * errs["f32"], errs
    G = torch.randn(M, n, generator=g) * 1e-3
    refw = G.double().t() @ torch.cat([a1, a2], 1).double()
    for math in ("split_bf16", "f32"):
        dW, _, _, _ = gemm_tn(n, a1.to(device), a2.to(device), g=G.to(device), math=math)
        errs["tn_" + math] = rel_l2(torch.cat([dW[0], dW[1]], 1), refw)
    assert errs["tn_split_bf16"] < 1e-6 and errs["tn_split_bf16"] < 2 * errs["tn_f32"], errs


@pytest.mark.parametrize("M,nr,k1,k2", [(5000, 128, 166, 166), (777, 3, 20, 0), (64, 128, 128, 128),
                                        (20000, 64, 167, 167), (33, 1, 1, 0)])
@pytest.mark.parametrize("form", ["g", "g_mask", "dz_mask"])
@pytest.mark.parametrize("math", ["split_bf16", "f32"])
def test_gemm_tn(device, M, nr, k1, k2, form, math):
    from elliptic_gnn_project_amd.fused import gemm_tn

    g_ = torch.Generator().manual_seed(M + nr)
    a1 = torch.randn(M, k1, generator=g_)
    a2 = torch.randn(M, k2, generator=g_) if k2 else None
    A = torch.cat([a1, a2], 1) if k2 else a1
    h = torch.relu(torch.randn(M, nr, generator=g_))
    dz = torch.randn(M, 4, generator=g_)
    proj = torch.randn(4, nr, generator=g_)
    G = torch.randn(M, nr, generator=g_)
    kw = {}
    if form == "dz_mask":
        G = dz @ proj
        kw = dict(dz=dz.to(device), proj=proj.to(device))
    else:
        kw = dict(g=G.to(device))
    if form != "g":
        G = torch.where(h > 0, G * 2.0, torch.zeros_like(G))
        kw.update(h=h.to(device), hscale=2.0)
    gout = torch.empty(M, nr, device=device)
    dW, db, dW2, dzs = gemm_tn(nr, a1.to(device), a2.to(device) if a2 is not None else None, gout=gout,
                               math=math, **kw)
    torch.testing.assert_close(gout.cpu(), G, rtol=1e-5, atol=1e-5)
    dWfull = torch.cat([dW[0], dW[1]], 1) if dW[1] is not None else dW[0]
    assert dW[0].is_contiguous()
    assert rel_l2(dWfull, G.t() @ A) < 1e-5
    assert rel_l2(db, G.sum(0)) < 1e-5
    if form == "dz_mask":
        assert rel_l2(dW2, dz.t() @ h) < 1e-5
        assert rel_l2(dzs, dz.sum(0)) < 1e-5


@pytest.mark.parametrize("M,k1,k2,n", [(50000, 64, 0, 2), (3001, 166, 166, 2), (1000, 7, 9, 5), (777, 384, 0, 8),
                                       (4097, 2, 0, 64), (1000, 3, 0, 33), (513, 8, 0, 256), (100, 1, 0, 1),
                                       # fewer K chunks than output columns (lanes per row >= N)
                                       (1000, 12, 0, 6), (999, 8, 0, 8), (640, 4, 4, 5)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "dropout"])
@pytest.mark.parametrize("wform", [False, True])
def test_gemm_nt_skinny(device, M, k1, k2, n, epi, wform):
    """Narrow output-layer shapes (N <= 8, or K <= 8) on the VALU kernels (gemm_skinny.hip):
    full f32 arithmetic, the NT epilogue (bias, ReLU, counter-hash dropout) unchanged."""
    from elliptic_gnn_project_amd.fused import gemm_nt

    if wform and n > 128:
        pytest.skip("w1/w2 form needs N <= 128")
    g = torch.Generator().manual_seed(M + k1 + 3 * n)
    a1 = torch.randn(M, k1, generator=g)
    a2 = torch.randn(M, k2, generator=g) if k2 else None
    bt = torch.randn(k1 + k2, n, generator=g) / (k1 + k2) ** 0.5
    bias = torch.randn(n, generator=g)
    A = torch.cat([a1, a2], 1) if k2 else a1
    ref = (A.double() @ bt.double()).float()
    kw = {}
    if epi != "plain":
        ref = torch.relu(ref + bias)
        kw = dict(bias=bias.to(device), relu=True)
    if epi == "dropout":
        p = 0.4
        m = torch.from_numpy(keep_mask(99, M, n, p))
        ref = ref * m / (1 - np.float32(p))
        kw.update(dropout_p=p, seed=99)
    if wform:
        kw.update(w1=bt[:k1].t().contiguous().to(device), w2=bt[k1:].t().contiguous().to(device) if k2 else None)
    for math in ("split_bf16", "f32"):
        c = gemm_nt(a1.to(device), None if wform else bt.to(device), n,
                    a2=a2.to(device) if a2 is not None else None, math=math, **kw)
        torch.testing.assert_close(c.cpu(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,nr,k1,k2", [(50000, 2, 64, 0), (3001, 2, 166, 166), (1000, 5, 7, 9), (777, 8, 384, 0),
                                        (1000, 1, 3, 0), (203769, 2, 64, 0)])
def test_gemm_tn_skinny(device, M, nr, k1, k2):
    """dW = Gᵀ·A and db = Σ G for Nr <= 8 (plain g form) on the VALU kernel; deterministic."""
    from elliptic_gnn_project_amd.fused import gemm_tn

    g_ = torch.Generator().manual_seed(M + 7 * nr)
    a1 = torch.randn(M, k1, generator=g_)
    a2 = torch.randn(M, k2, generator=g_) if k2 else None
    A = torch.cat([a1, a2], 1) if k2 else a1
    G = torch.randn(M, nr, generator=g_)
    a1d, a2d = a1.to(device), a2.to(device) if a2 is not None else None
    dW, db, _, _ = gemm_tn(nr, a1d, a2d, g=G.to(device))
    dWfull = torch.cat([dW[0], dW[1]], 1) if dW[1] is not None else dW[0]
    assert rel_l2(dWfull, G.double().t() @ A.double()) < 1e-6
    assert rel_l2(db, G.double().sum(0)) < 1e-6
    dW2, db2, _, _ = gemm_tn(nr, a1d, a2d, g=G.to(device))
    assert torch.equal(dW2[0], dW[0]) and torch.equal(db2, db)


def _graph(n, e, seed):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    return prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))


@pytest.mark.parametrize("layers,hidden", [(2, 128), (3, 128), (3, 64), (4, 32)])
@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_fused_sage_train_step(device, layers, hidden, dropout):
    """Fused SAGENet vs the oracle: logits and every parameter gradient, same dropout masks."""
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = _graph(5000, 6000, seed=21)
    N = data.x.size(0)
    torch.manual_seed(5)
    model = SAGENet(data.x.size(1), hidden, layers=layers, dropout=dropout).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    torch.manual_seed(77)
    logits = model(data.x.to(device), data.edge_index.to(device))
    torch.manual_seed(77)
    seeds = torch.randint(0, 2 ** 62, (layers,), dtype=torch.int64).tolist()
    masks = [torch.from_numpy(keep_mask(seeds[l], N, hidden, dropout)) for l in range(layers - 1)] \
        if dropout > 0 else None
    mask = data.train_mask
    cw = pyg_ref.class_weight(data.y[mask])
    loss = pyg_ref.ce_loss(logits[mask.to(device)], data.y[mask].to(device), cw.to(device))
    loss.backward()
    kw = dict(layers=layers, dropout=dropout, training=True, dropout_masks=masks)
    ref = pyg_ref.model_forward("sage", params, data.x, data.edge_index, **kw)
    torch.testing.assert_close(logits.detach().cpu(), ref, rtol=1e-5, atol=1e-5)
    _, grads = pyg_ref.train_step_grads("sage", params, data.x, data.edge_index, data.y, mask, cw, **kw)
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 1e-5, k


def test_fused_matches_unfused_and_input_grad(device):
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = _graph(3000, 4000, seed=3)
    torch.manual_seed(1)
    model = SAGENet(data.x.size(1), 64, layers=3, dropout=0.0).to(device)
    x = data.x.to(device).requires_grad_(True)
    ei = data.edge_index.to(device)
    out_f = model(x, ei)
    out_f.square().sum().backward()
    gx_f = x.grad.clone()
    gp_f = {k: v.grad.clone() for k, v in model.named_parameters()}
    model.zero_grad()
    x.grad = None
    model.fused = False
    out_u = model(x, ei)
    out_u.square().sum().backward()
    torch.testing.assert_close(out_f, out_u, rtol=1e-5, atol=1e-5)
    assert rel_l2(gx_f, x.grad) < 1e-5
    for k, v in model.named_parameters():
        assert rel_l2(gp_f[k], v.grad) < 1e-5, k


def test_fused_full_elliptic_eval_and_determinism(device):
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = _graph(203_769, 234_355, seed=42)
    torch.manual_seed(4)
    model = SAGENet(166, 128, layers=2, dropout=0.5).to(device)
    p = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.eval()
    x, ei = data.x.to(device), data.edge_index.to(device)
    with torch.no_grad():
        a = model(x, ei)
        b = model(x, ei)
    assert torch.equal(a, b)
    ref = pyg_ref.model_forward("sage", p, data.x, data.edge_index, layers=2)
    torch.testing.assert_close(a.cpu(), ref, rtol=1e-5, atol=1e-5)


def _train_setup(device, dropout):
    from elliptic_gnn_project_amd.gnn import SAGENet
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn

    data = _graph(4000, 5000, seed=9).to(device)
    torch.manual_seed(11)
    model = SAGENet(data.x.size(1), 64, layers=2, dropout=dropout).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=0.01, weight_decay=1e-4, capturable=True)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    loss_fn = _make_loss_fn({}, cw, model, 1, 34)

    def step():
        model.train()
        opt.zero_grad(set_to_none=True)
        out = model(data.x, data.edge_index)
        loss = loss_fn(out.index_select(0, data.train_idx), data.y.index_select(0, data.train_idx))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss

    return model, step


def test_captured_step_matches_eager(device):
    """HIP-graph replay of the whole train step == the same number of eager steps (bitwise)."""
    from elliptic_gnn_project_amd.train_gnn import CapturedStep

    m_e, step_e = _train_setup(device, 0.0)
    for _ in range(5):
        step_e()
    m_g, step_g = _train_setup(device, 0.0)
    cs = CapturedStep(step_g, warmup=3)  # 3 eager warm-up steps, then capture (not executed)
    cs()
    cs()
    torch.cuda.synchronize()
    for (k, a), b in zip(m_e.state_dict().items(), m_g.state_dict().values()):
        assert torch.equal(a, b), k


def test_captured_step_redraws_dropout(device):
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.train_gnn import CapturedStep

    model, step = _train_setup(device, 0.5)
    cs = CapturedStep(step, warmup=1)
    ctr = fused._SEED_CTR[device]
    c0 = int(ctr.item())
    l1 = float(cs().item())
    l2 = float(cs().item())
    assert int(ctr.item()) == c0 + 2
    assert l1 != l2


@pytest.mark.parametrize("layers,hidden", [(2, 64), (3, 64), (3, 32)])
@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_fused_gcn_train_step(device, layers, hidden, dropout):
    """Fused GCNNet (bias/ReLU/dropout in the aggregation store, their backward in the skinny
    GEMM's mask epilogue) vs the oracle: logits and every parameter gradient, same masks."""
    from elliptic_gnn_project_amd.gnn import GCNNet

    data = _graph(5000, 6000, seed=23)
    N = data.x.size(0)
    torch.manual_seed(6)
    model = GCNNet(data.x.size(1), hidden, layers=layers, dropout=dropout).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    torch.manual_seed(78)
    logits = model(data.x.to(device), data.edge_index.to(device))
    torch.manual_seed(78)
    seeds = torch.randint(0, 2 ** 62, (layers,), dtype=torch.int64).tolist()
    masks = [torch.from_numpy(keep_mask(seeds[l], N, hidden, dropout)) for l in range(layers - 1)] \
        if dropout > 0 else None
    mask = data.train_mask
    cw = pyg_ref.class_weight(data.y[mask])
    loss = pyg_ref.ce_loss(logits[mask.to(device)], data.y[mask].to(device), cw.to(device))
    loss.backward()
    kw = dict(layers=layers, dropout=dropout, training=True, dropout_masks=masks)
    ref = pyg_ref.model_forward("gcn", params, data.x, data.edge_index, **kw)
    torch.testing.assert_close(logits.detach().cpu(), ref, rtol=1e-5, atol=1e-5)
    _, grads = pyg_ref.train_step_grads("gcn", params, data.x, data.edge_index, data.y, mask, cw, **kw)
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 1e-5, k


def test_fused_gcn_matches_unfused(device):
    """Eval mode: the fused node and the per-conv path (same kernels, torch glue) agree, incl. dx."""
    from elliptic_gnn_project_amd.gnn import GCNNet

    data = _graph(3000, 4000, seed=4)
    torch.manual_seed(2)
    model = GCNNet(data.x.size(1), 64, layers=3, dropout=0.3).to(device).eval()
    outs = []
    for fused in (True, False):
        model.fused = fused
        x = data.x.to(device).requires_grad_(True)
        out = model(x, data.edge_index.to(device))
        out.square().sum().backward()
        outs.append((out.detach(), x.grad.detach(), [p.grad.detach().clone() for p in model.parameters()]))
        model.zero_grad()
    (o1, dx1, g1), (o2, dx2, g2) = outs
    torch.testing.assert_close(o1, o2, rtol=1e-5, atol=1e-5)
    assert rel_l2(dx1, dx2) < 1e-5
    for a, b in zip(g1, g2):
        assert rel_l2(a, b) < 1e-5


def test_fused_gcn_graph_capture(device):
    """The fused GCN step replays as a HIP graph with a fresh dropout mask per replay."""
    from elliptic_gnn_project_amd.gnn import GCNNet

    data = _graph(3000, 4000, seed=5)
    torch.manual_seed(3)
    model = GCNNet(data.x.size(1), 64, layers=2, dropout=0.5).to(device).train()
    x, ei = data.x.to(device), data.edge_index.to(device)
    model(x, ei)  # plan + seed counter outside the capture
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        model(x, ei)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = model(x, ei)
    g.replay()
    a = out.clone()
    g.replay()
    b = out.clone()
    assert torch.isfinite(a).all() and not torch.equal(a, b)  # new mask per replay
