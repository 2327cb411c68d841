"""GPU: split images ("planes") of the SAGE layer-1 operand and the GEMMs that read them.

* gnn_split_planes_f32 and K1's split-image store (gnn_sage_mean_fwd_planes) are integer /
  rounding work: bit-exact against a numpy restatement of the split (RNE f32 -> bf16 by the
  integer rule, remainders in f32), and hi + mid + lo == v exactly.  K1's planes are the split
  of the f32 K1 output bit for bit (same kernel loop, same summation order).
* The NT / TN kernels on planes are floating point: within the split's error of a float64
  reference (relL2 < 1e-6, the bound test_gpu_fused.py holds the in-kernel split to), and the
  fused SAGE step with planes on and off within 1e-5.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _bf16_rne(v):
    u = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def _widen(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def split3(v):
    """hi / mid / lo bf16 words of float32 v (finite, normal-range values)."""
    v = np.asarray(v, dtype=np.float32)
    hi = _bf16_rne(v)
    r1 = (v - _widen(hi)).astype(np.float32)
    mid = _bf16_rne(r1)
    r2 = (r1 - _widen(mid)).astype(np.float32)
    lo = _bf16_rne(r2)
    return hi, mid, lo


def _planes_np(im):
    return im.img.view(torch.int16).cpu().numpy().view(np.uint16)


def _features(n, f, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, f, generator=g) * torch.exp(torch.randn(n, 1, generator=g) * 3)
    x[0, :8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38, -2.5e-30, 1.0 + 2 ** -23, 65504.0])
    return x


def test_split_planes_bit_exact(device):
    from elliptic_gnn_project_amd.planes import SplitImage

    N, F = 1003, 166
    x = _features(N, F, 1)
    im = SplitImage(N, F, F, device)
    assert (im.col2, im.ld) == (168, 336)
    im.img.fill_(1.0)  # every column of the x half must be written
    im.fill_x(x.to(device))
    got = _planes_np(im)
    for p, want in enumerate(split3(x.numpy())):
        assert np.array_equal(got[p][:, 168:334], want), p
        assert not got[p][:, 334:].any()
    hi, mid, lo = (_widen(got[p][:, 168:334]).astype(np.float64) for p in range(3))
    assert np.array_equal(hi + mid + lo, x.numpy().astype(np.float64))


def _plan_and_x(n, e, seed, device):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.graph import get_plan

    data = prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    from elliptic_gnn_project_amd.planes import register_input

    ei = data.edge_index.to(device)
    # a registered constant input (as train_gnn.main / bench.py register x): the SAGE layer-1 [agg | x] image
    return data, get_plan(ei, data.x.size(0)), register_input(data.x.to(device))


@pytest.mark.parametrize("n,e", [(5000, 6000), (203_769, 234_355)])
def test_mean_planes_equal_split_of_k1(device, n, e):
    """K1's split-image store == the numpy split of the f32 K1 output, bit for bit (incl. hub
    rows and in-degree-0 rows of the full Elliptic-shape graph)."""
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.planes import SplitImage

    data, plan, x = _plan_and_x(n, e, 31, device)
    agg = aggregate(plan, x, _lib.AGG_MEAN, nodew=plan.deg).cpu().numpy()
    im = SplitImage(x.size(0), x.size(1), x.size(1), device)
    im.img.fill_(1.0)
    gen = im.fill_mean(plan, x)
    assert gen == 1
    got = _planes_np(im)
    for p, want in enumerate(split3(agg)):
        assert np.array_equal(got[p][:, :166], want), p
        assert not got[p][:, 166:168].any()


def _sage_layer_operands(M, F, n, seed):
    g = torch.Generator().manual_seed(seed)
    agg = torch.randn(M, F, generator=g)
    x = torch.randn(M, F, generator=g)
    w1 = torch.randn(n, F, generator=g) * 0.08
    w2 = torch.randn(n, F, generator=g) * 0.08
    return agg, x, w1, w2


def _image(agg, x, device):
    from elliptic_gnn_project_amd.planes import SplitImage

    im = SplitImage(agg.size(0), agg.size(1), x.size(1), device)
    im.fill_x(x.to(device))
    # the agg half through the same split kernel (its bit-exactness is tested above)
    from elliptic_gnn_project_amd import _lib
    _lib.call("gnn_split_planes_f32", agg.to(device).data_ptr(), agg.size(1), im.n, im.k1, im.ptr, im.ld, im.ps, 0,
              im.col2, _lib.stream_handle(device))
    return im


@pytest.mark.parametrize("M", [20000, 32, 1000, 4097, 203_769])
@pytest.mark.parametrize("epi", ["plain", "relu_drop_proj"])
def test_nt_planes_vs_f64(device, M, epi):
    from oracle.dropout_hash import keep_mask
    from elliptic_gnn_project_amd.fused import gemm_nt

    F, n = 166, 128
    agg, x, w1, w2 = _sage_layer_operands(M, F, n, M)
    bias = torch.randn(n) * 0.1
    proj = torch.randn(4, n)
    ref = torch.cat([agg, x], 1).double() @ torch.cat([w1, w2], 1).double().t()
    kw = dict(w1=w1.to(device), w2=w2.to(device))
    z = None
    if epi != "plain":
        p = 0.5
        m = torch.from_numpy(keep_mask(99, M, n, p)).double()
        ref = torch.relu(ref + bias.double()) * m * 2.0
        z = torch.empty(M, 4, device=device)
        kw.update(bias=bias.to(device), relu=True, dropout_p=p, seed=99, proj=proj.to(device), z=z)
    im = _image(agg, x, device)
    assert gemm_nt(None, None, n, planes=im, check_planes=True, **kw)
    c = gemm_nt(None, None, n, planes=im, **kw)
    assert rel_l2(c, ref) < 1e-6
    if z is not None:
        assert rel_l2(z, c.double().cpu() @ proj.double().t()) < 1e-6
        z.fill_(float("nan"))
    c0 = gemm_nt(agg.to(device), None, n, a2=x.to(device), **kw)  # the in-kernel split form
    torch.testing.assert_close(c.cpu(), c0.cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M", [20001, 16, 1000, 203_769])
@pytest.mark.parametrize("form", ["dz_mask", "g_mask", "g", "g_mask_gout"])
def test_tn_planes_vs_f64(device, M, form):
    from elliptic_gnn_project_amd.fused import gemm_tn

    F, nr = 166, 128
    agg, x, _, _ = _sage_layer_operands(M, F, 1, M + 1)
    g_ = torch.Generator().manual_seed(M)
    h = torch.relu(torch.randn(M, nr, generator=g_))
    dz = torch.randn(M, 4, generator=g_) * 1e-3
    proj = torch.randn(4, nr, generator=g_)
    G = torch.randn(M, nr, generator=g_) * 1e-3
    if form == "dz_mask":
        G = dz @ proj
        kw = dict(dz=dz.to(device), proj=proj.to(device))
    else:
        kw = dict(g=G.to(device))
    if form != "g":
        G = torch.where(h > 0, G * 2.0, torch.zeros_like(G))
        kw.update(h=h.to(device), hscale=2.0)
    gout = torch.empty(M, nr, device=device) if form == "g_mask_gout" else None
    im = _image(agg, x, device)
    assert gemm_tn(nr, None, None, planes=im, check_planes=True, **kw)
    dW, db, dW2, dzs = gemm_tn(nr, None, None, planes=im, gout=gout, **kw)
    A = torch.cat([agg, x], 1).double()
    refw = G.double().t() @ A
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), refw) < 1e-6
    assert rel_l2(db, G.double().sum(0)) < 1e-6
    if form == "dz_mask":
        assert rel_l2(dW2, dz.double().t() @ h.double()) < 1e-6
        assert rel_l2(dzs, dz.double().sum(0)) < 1e-6
    if gout is not None:
        torch.testing.assert_close(gout.cpu(), G, rtol=1e-6, atol=1e-9)
    # the same gradient through the in-kernel split form
    dWf, dbf, _, _ = gemm_tn(nr, agg.to(device), x.to(device), **kw)
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), torch.cat([dWf[0], dWf[1]], 1)) < 1e-6


def _sage_step(model, x, ei, seed):
    torch.manual_seed(seed)
    out = model(x, ei)
    loss = out.square().mean()
    return out, loss


@pytest.mark.parametrize("n,e", [(5000, 6000), (203_769, 234_355)])
def test_fused_sage_planes_on_off(device, n, e):
    """The fused SAGE train step (dropout 0.5) with the layer-1 operand as a split image vs the
    in-kernel split: logits and every gradient within 1e-5 (same dropout masks)."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(n, e, 5, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(3)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.5).to(device).train()
    res = []
    fused._H2 = False  # the split-bf16 image (the half-pair one: tests/test_gpu_h2.py)
    for on in (True, False):
        fused._PLANES = on
        try:
            model.zero_grad()
            out, loss = _sage_step(model, x, ei, 123)
            loss.backward()
            res.append((out.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._PLANES = True
            fused._H2 = True
    (o1, g1), (o2, g2) = res
    torch.testing.assert_close(o1, o2, rtol=1e-5, atol=1e-5)
    for k in g1:
        assert rel_l2(g1[k], g2[k]) < 1e-5, k
    assert any(getattr(x, a, None) is not None  # the planes path ran (half-pair or split-bf16 image)
               for a in ("_gnnmp_split_image", "_gnnmp_split_image_h2"))


def test_two_forwards_then_backward(device):
    """A second grad-enabled forward over the same x rewrites the image's agg half; the first
    forward's backward notices (generation stamp), refreshes it and gets the same gradients."""
    from elliptic_gnn_project_amd.gnn import SAGENet
    from elliptic_gnn_project_amd.planes import register_input

    data, plan, x = _plan_and_x(3000, 4000, 8, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(4)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.0).to(device).train()
    out, loss = _sage_step(model, x, ei, 1)
    loss.backward()
    ref = {k: p.grad.clone() for k, p in model.named_parameters()}
    model.zero_grad()
    x2 = register_input(x * 2.0)  # another x: its own image
    out_a, loss_a = _sage_step(model, x, ei, 1)
    out_b, loss_b = _sage_step(model, x, ei, 1)  # same x: rewrites the agg half
    _ = model(x2, ei)
    loss_a.backward()
    for k, p in model.named_parameters():
        assert torch.equal(p.grad, ref[k]), k
    assert any(getattr(x, a, None) is not None  # the planes path ran (half-pair or split-bf16 image)
               for a in ("_gnnmp_split_image", "_gnnmp_split_image_h2"))


def test_unregistered_input_builds_no_image(device):
    """A per-batch / per-step input (not registered) takes the in-kernel split: no [3, N, ld]
    image is allocated for it, and the result equals the registered input's within 1e-5."""
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(3000, 4000, 9, device)
    ei = data.edge_index.to(device)
    xu = x.clone()  # same values, not registered
    torch.manual_seed(5)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.0).to(device).train()
    outs = []
    for inp in (x, xu):
        model.zero_grad()
        out, loss = _sage_step(model, inp, ei, 2)
        loss.backward()
        outs.append((out.detach(), {k: p.grad.clone() for k, p in model.named_parameters()}))
    assert any(getattr(x, a, None) is not None for a in ("_gnnmp_split_image", "_gnnmp_split_image_h2"))
    assert all(getattr(xu, a, None) is None for a in ("_gnnmp_split_image", "_gnnmp_split_image_h2"))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-5)
    for k in outs[0][1]:
        assert rel_l2(outs[0][1][k], outs[1][1][k]) < 1e-5, k


def test_x_image_follows_in_place_edit(device):
    from elliptic_gnn_project_amd.planes import x_image

    x = torch.randn(500, 166, device=device)
    im = x_image(x)
    assert x_image(x) is im
    x.mul_(3.0)
    im2 = x_image(x)
    hi = _planes_np(im2)[0][:, 168:334]
    assert np.array_equal(hi, split3(x.cpu().numpy())[0])


@pytest.mark.parametrize("F,nr", [(166, 64), (166, 128), (40, 16)])
def test_input_tn_on_x_only_image(device, F, nr):
    """dW = Gᵀ·x for a model input x (GCN / GAT layer 1): the split-image TN over x's cached planes
    (x in columns [0, F), k2 = 0) and the f32-operand TN both within the split's error of float64;
    the planes are x's split bit for bit and follow an in-place edit of x."""
    from elliptic_gnn_project_amd.fused import gemm_tn_input
    from elliptic_gnn_project_amd.planes import register_input, x_only_image

    N = 5000
    g0 = torch.Generator().manual_seed(F + nr)
    x = torch.randn(N, F, generator=g0).to(device)
    assert x_only_image(x) is None  # unregistered inputs keep the f32 operand
    register_input(x)
    G = torch.randn(N, nr, generator=g0).to(device)
    ref = (G.double().t() @ x.double()).cpu()
    from elliptic_gnn_project_amd.fused import gemm_tn

    (dW1, _), db1, _, _ = gemm_tn(nr, x, g=G)  # the f32-operand TN
    (dW2, _), db2, _, _ = gemm_tn_input(nr, x, G)  # x's cached planes
    im = x_only_image(x)
    assert getattr(x, "_gnnmp_split_image_x", None) is im
    assert im is not None and im.k2 == 0 and im.ld == 176  # planes.X_ONLY_LD: every x-only image
    hi, mid, lo = split3(x.cpu().numpy())
    P = _planes_np(im)
    assert np.array_equal(P[0, :, :F], hi) and np.array_equal(P[1, :, :F], mid) and np.array_equal(P[2, :, :F], lo)
    assert not P[:, :, F:].any()
    for dW, db in ((dW1, db1), (dW2, db2)):
        assert rel_l2(dW, ref) < 1e-6
        assert rel_l2(db, G.double().sum(0).cpu()) < 1e-6
    x.add_(0.0)  # in-place edit: the planes are rebuilt from the new version
    (dW3, _), _, _, _ = gemm_tn_input(nr, x, G)
    assert rel_l2(dW3, ref) < 1e-6


@pytest.mark.parametrize("F,n,bias", [(166, 64, False), (166, 128, True), (166, 2, True)])
def test_input_nt_on_x_only_image(device, F, n, bias):
    """y = x·Wᵀ (+ b) for a model input x (GCN / GAT layer 1): the split-image NT over x's cached
    176-wide planes (N <= 128, N % 4 == 0) against float64, as the f32-operand NT is."""
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_nt_input
    from elliptic_gnn_project_amd.planes import register_input, x_only_image

    N = 4099  # a ragged last row tile
    g0 = torch.Generator().manual_seed(F + n)
    x = register_input(torch.randn(N, F, generator=g0).to(device))
    W = (torch.randn(n, F, generator=g0) * 0.1).to(device)
    b = torch.randn(n, generator=g0).to(device) if bias else None
    ref = x.double() @ W.double().t() + (b.double() if bias else 0)
    y0 = gemm_nt(x, None, n, bias=b, w1=W)
    im = x_only_image(x)
    assert im is not None and x_only_image(x) is im  # cached on x
    takes = gemm_nt(None, None, n, planes=im, check_planes=True, bias=b, w1=W)
    assert takes == (n % 4 == 0)  # (N = 2 stays on the skinny VALU NT: 16-byte C row stores)
    y1 = gemm_nt_input(x, n, bias=b, w1=W)
    assert rel_l2(y0, ref) < 1e-6 and rel_l2(y1, ref) < 1e-6
