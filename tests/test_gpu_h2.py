"""GPU: half-pair images (include/gnnmp.h gnn_split_h2_f32: u = v·2^e, f16 hi = RNE(u),
lo = RNE((u - hi)·2^11), e the per-image pre-scale putting max|u| in [2^13, 2^14)) and the
3-product f16 GEMMs that read them — the 2-layer SAGE's layer-1 [agg | x] operand.

* gnn_split_h2_f32 and K1's half-pair store (gnn_sage_mean_fwd_h2) are rounding work: bit-exact
  against a numpy restatement (numpy's float32 -> float16 cast is RNE), and K1's planes are the
  split of the f32 K1 output bit for bit.
* The NT / TN kernels are floating point: within relL2 1e-6 of a float64 reference (the bound the
  split-bf16 image kernels are held to; the dropped lo·lo term is 2^-22 relative), also for
  weights / gradients far outside [1/16, 16] (the per-column / per-block power-of-two scales)
  and for inputs of any magnitude (1e-7 .. 3e4: the image's pre-scale; ABI 18's unscaled image
  lost 9e-5 relL2 at 1e-7), and the fused SAGE step with half-pair planes within 1e-5 of the
  split-bf16 planes and of the float64 oracle.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_l2(a, b, floor=1e-30):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), floor))


def split_h2(v, e=0):
    """hi / lo f16 words of float32 v · 2^e (|v · 2^e| < 2^15)."""
    v = np.asarray(v, dtype=np.float32) * np.float32(2.0 ** e)  # exact: a power of two
    hi = v.astype(np.float16)
    r = ((v - hi.astype(np.float32)) * np.float32(2048.0)).astype(np.float32)
    lo = r.astype(np.float16)
    return hi.view(np.uint16), lo.view(np.uint16)


def _planes_np(im):
    return im.img.view(torch.int16).cpu().numpy().view(np.uint16)


def _plan_and_x(n, e, seed, device):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.graph import get_plan
    from elliptic_gnn_project_amd.planes import register_input

    data = prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    ei = data.edge_index.to(device)
    return data, get_plan(ei, data.x.size(0)), register_input(data.x.to(device))


def test_split_h2_bit_exact(device):
    from elliptic_gnn_project_amd.planes import HalfPairImage

    g = torch.Generator().manual_seed(3)
    x = torch.randn(777, 166, generator=g) * torch.exp(torch.randn(777, 1, generator=g) * 3)
    x[0, :8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 16383.0, -2.5e-30, 1.0 + 2 ** -23, 6.0e-8])
    x = x.clamp(-16383.0, 16383.0)
    for scale, e in ((1.0, 0), (2.0 ** -30, 30), (2.0 ** 40, -40), (3e-7, 21)):  # max|x| = 16383
        xs = x * scale
        im = HalfPairImage(777, 166, 166, device)
        im.img.fill_(1.0)
        im.fill_x(xs.to(device))
        assert im.exp == e, (scale, im.exp)
        got = _planes_np(im)
        hi, lo = split_h2(xs.numpy(), e)
        assert np.array_equal(got[0][:, 168:334], hi)
        assert np.array_equal(got[1][:, 168:334], lo)
        assert not got[0][:, 334:].any() and not got[1][:, 334:].any()
        # (hi + 2^-11 lo) · 2^-e reproduces v to 2^-22 relative, or 2^-36 of the image's top
        rec = (got[0][:, 168:334].view(np.float16).astype(np.float64)
               + got[1][:, 168:334].view(np.float16).astype(np.float64) / 2048.0) * 2.0 ** -e
        xd = xs.double().numpy()
        assert np.all(np.abs(rec - xd) <= 2.0 ** -22 * np.abs(xd) + 2.0 ** -36 * 2.0 ** -e)


@pytest.mark.parametrize("n,e", [(5000, 6000), (203_769, 234_355)])
def test_mean_h2_equals_split_of_k1(device, n, e):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.planes import HalfPairImage

    data, plan, x = _plan_and_x(n, e, 31, device)
    agg = aggregate(plan, x, _lib.AGG_MEAN, nodew=plan.deg).cpu().numpy()
    im = HalfPairImage(x.size(0), x.size(1), x.size(1), device)
    im.img.fill_(1.0)
    for gen, ex in enumerate((0, 9, -3), start=1):  # K1 stores mean · 2^exp (the image's pre-scale)
        im.exp = ex
        assert im.fill_mean(plan, x, hub=False) == gen
        got = _planes_np(im)
        for p, want in enumerate(split_h2(agg, ex)):
            assert np.array_equal(got[p][:, :166], want), (p, ex)
            assert not got[p][:, 166:168].any()


def _mean_hub_np(plan, x, T):
    """Restatement of K1's hub form (gnn_sage_mean_fwd_h2 hub): a row with deg > T summed by 4
    waves, wave w over the row's 8-slot groups w, w + 4, ... in slot order, the waves' sums then
    added in wave order; every other row in slot order (float32 throughout); PyG's mean."""
    rowptr, col, _ = (t.cpu().numpy() for t in plan.csr())
    xs = x.cpu().numpy()
    deg = plan.deg.cpu().numpy()[: x.size(0)]
    out = np.zeros_like(xs)
    for r in range(x.size(0)):
        b, e = int(rowptr[r]), int(rowptr[r + 1])
        if deg[r] > T:
            acc = [np.zeros(xs.shape[1], np.float32) for _ in range(4)]
            for s in range(b, e):
                w = ((s - b) // 8) % 4
                acc[w] = acc[w] + xs[col[s]]
            tot = ((acc[0] + acc[1]) + acc[2]) + acc[3]
        else:
            tot = np.zeros(xs.shape[1], np.float32)
            for s in range(b, e):
                tot = tot + xs[col[s]]
        out[r] = tot
    return out / np.maximum(deg, np.float32(1.0))[:, None]


@pytest.mark.parametrize("shape", ["ring_isolated", "star", "tiny", "many_hubs"])
def test_mean_h2_hub_form_edge_graphs(device, shape):
    """The hub form on edge-case graphs — no hub rows (balanced waves only: bit-identical to the
    16-row waves), one degree-300 star centre, 3 nodes, every row a hub — vs the restatement."""
    from elliptic_gnn_project_amd.graph import get_plan
    from elliptic_gnn_project_amd.planes import HalfPairImage

    g = torch.Generator().manual_seed(5)
    if shape == "ring_isolated":  # 3000 ring nodes, 500 isolated ones
        n = 3500
        src = torch.arange(3000)
        ei = torch.stack([torch.cat([src, (src + 1) % 3000]), torch.cat([(src + 1) % 3000, src])])
    elif shape == "star":
        n = 1000
        leaves = torch.arange(1, 301)
        ei = torch.stack([torch.cat([leaves, torch.zeros(300, dtype=torch.long)]),
                          torch.cat([torch.zeros(300, dtype=torch.long), leaves])])
    elif shape == "tiny":
        n = 3
        ei = torch.tensor([[0, 1, 2, 2], [1, 2, 0, 1]])
    else:  # 40 nodes, all-to-all: every row has 39 > K1_HUB_DEG slots
        n = 40
        a, b = torch.meshgrid(torch.arange(n), torch.arange(n), indexing="ij")
        m = a != b
        ei = torch.stack([a[m], b[m]])
    plan = get_plan(ei.to(device), n)
    x = (torch.randn(n, 166, generator=g) * 3).to(device)
    im = HalfPairImage(n, 166, 166, device)
    im.fill_x(x)
    im.img.fill_(1.0)
    im.fill_mean(plan, x)
    got = _planes_np(im)
    T = int(plan.hub["c"].seg_len)  # the plan's hub degree (graph.K1_HUB_DEG: 16 / 32 by size)
    for p, w in enumerate(split_h2(_mean_hub_np(plan, x, T), im.exp)):
        assert np.array_equal(got[p][:, :166], w), p
        assert not got[p][:, 166:168].any()
    if shape == "ring_isolated":
        assert plan.hub is not None and int(plan.hub["c"].num_long) == 0 and int(plan.hub["c"].num_pieces) > 1
        im.fill_mean(plan, x, hub=False)
        assert np.array_equal(_planes_np(im), got)


@pytest.mark.parametrize("n,e,padded", [(5000, 6000, False), (20_000, 30_000, True)])
def test_mean_h2_hub_form_vs_restatement(device, n, e, padded):
    """K1's hub form (graph.K1_HUB_MAX_N: rows with deg > K1_HUB_DEG on blocks of their own): bit for
    bit the half-pair split of the numpy restatement of its summation order, padding columns
    zero; the ordinary rows bit-identical to the one-wave-per-16-rows K1, the hub rows within
    1e-5 of it (another f32 summation order of up to ~200 terms); the keep bits and the NT B prep riding along unchanged."""
    from elliptic_gnn_project_amd.fused import _nt_workspace, gemm_nt
    from elliptic_gnn_project_amd.planes import HalfPairImage, x_padded

    data, plan, x = _plan_and_x(n, e, 31, device)
    T = int(plan.hub["c"].seg_len)
    assert plan.hub is not None and int(plan.hub["c"].num_long) == int((plan.deg[: x.size(0)] > T).sum()) > 0
    hubs = plan.hub["hubs"].long().cpu().numpy()
    want = _mean_hub_np(plan, x, T)
    im = HalfPairImage(x.size(0), x.size(1), x.size(1), device)
    im.fill_x(x)
    kw = dict(x_pad=x_padded(x, im.col2)) if padded else {}
    for ex in (0, 7):
        im.img.fill_(1.0)
        im.exp = ex
        im.fill_mean(plan, x, **kw)  # the hub form by default at this size
        got = _planes_np(im)
        for p, w in enumerate(split_h2(want, ex)):
            assert np.array_equal(got[p][:, :166], w), (p, ex)
            assert not got[p][:, 166:168].any()
    hub_img = _planes_np(im)
    im.fill_mean(plan, x, hub=False, **kw)
    one = _planes_np(im)
    rest = np.setdiff1d(np.arange(x.size(0)), hubs)
    assert np.array_equal(hub_img[:, rest], one[:, rest])
    rec = lambda g: g[0][:, :166].view(np.float16).astype(np.float64) + g[1][:, :166].view(np.float16) / 2048.0
    a, b = rec(hub_img)[hubs], rec(one)[hubs]
    assert np.abs(a - b).max() <= 1e-5 * np.abs(b).max()
    # keep bits and the B prep of the consuming NT ride along with the hub blocks
    n_out = 128
    g = torch.Generator().manual_seed(4)
    w1 = (torch.randn(n_out, x.size(1), generator=g) * 0.08).to(device)
    w2 = (torch.randn(n_out, x.size(1), generator=g) * 0.08).to(device)
    kb1, kb2 = (torch.zeros(x.size(0), 4, dtype=torch.int32, device=device) for _ in range(2))
    im.fill_mean(plan, x, (kb1, n_out, 0.5, 3, None), hub=False, **kw)
    nt = dict(w1=w1, w2=w2, bias=torch.randn(n_out, generator=g).to(device), relu=True, dropout_p=0.5, seed=9)
    im.fill_mean(plan, x, **kw)
    img0 = im.img.clone()
    c_one = gemm_nt(None, None, n_out, planes=im, **nt)
    ws = _nt_workspace(device, n_out, im.k1, im.k2)
    prm = gemm_nt(None, None, n_out, planes=im, workspace=ws, b_stage="params", **nt)
    im.fill_mean(plan, x, (kb2, n_out, 0.5, 3, None), prep_b=prm, **kw)
    assert torch.equal(kb1, kb2) and torch.equal(im.img, img0)
    assert torch.equal(gemm_nt(None, None, n_out, planes=im, workspace=ws, b_stage="ready", **nt), c_one)


def _operands(M, F, n, seed, wscale=0.08):
    g = torch.Generator().manual_seed(seed)
    agg = torch.randn(M, F, generator=g) * 0.7
    x = torch.randn(M, F, generator=g)
    w1 = torch.randn(n, F, generator=g) * wscale
    w2 = torch.randn(n, F, generator=g) * wscale
    return agg, x, w1, w2


def _image(agg, x, device):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.planes import HalfPairImage

    im = HalfPairImage(agg.size(0), agg.size(1), x.size(1), device)
    im.fill_x(x.to(device))  # sets im.exp from x; agg must stay within 2x of max|x| (as a mean does)
    _lib.call("gnn_split_h2_f32", agg.to(device).data_ptr(), agg.size(1), im.n, im.k1, im.ptr, im.ld, im.ps, 0,
              im.col2, im.exp, _lib.stream_handle(device))
    return im


@pytest.mark.parametrize("M", [32, 1000, 4097, 20000, 203_769])
@pytest.mark.parametrize("epi", ["plain", "relu_drop_proj"])
def test_nt_h2_vs_f64(device, M, epi):
    from oracle.dropout_hash import keep_mask
    from elliptic_gnn_project_amd.fused import gemm_nt

    F, n = 166, 128
    agg, x, w1, w2 = _operands(M, F, n, M)
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


@pytest.mark.parametrize("fmt", ["h2", "split"])
def test_nt_prep_b_then_ready_equals_one_call(device, fmt):
    """gnn_gemm_nt_prep_b on a side stream, then gnn_gemm_nt_f32 with b_ready over the same
    workspace (the SAGE layer-0 schedule): bit-identical to the one-call form, for the half-pair
    and the split-bf16 image."""
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.fused import _nt_workspace, gemm_nt
    from elliptic_gnn_project_amd.planes import SplitImage

    M, F, n = 5000, 166, 128
    agg, x, w1, w2 = _operands(M, F, n, 7)
    if fmt == "h2":
        im = _image(agg, x, device)
    else:
        im = SplitImage(M, F, F, device)
        im.fill_x(x.to(device))
        _lib.call("gnn_split_planes_f32", agg.to(device).data_ptr(), F, M, F, im.ptr, im.ld, im.ps, 0, im.col2,
                  _lib.stream_handle(device))
    kw = dict(w1=w1.to(device), w2=w2.to(device), bias=torch.randn(n).to(device), relu=True, dropout_p=0.5, seed=5)
    one = gemm_nt(None, None, n, planes=im, **kw)
    ws = _nt_workspace(device, n, im.k1, im.k2)
    side, cur = torch.cuda.Stream(device=device), torch.cuda.current_stream(device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        assert gemm_nt(None, None, n, planes=im, workspace=ws, b_stage="prep", **kw) is None
    cur.wait_stream(side)
    two = gemm_nt(None, None, n, planes=im, workspace=ws, b_stage="ready", **kw)
    assert torch.equal(one, two)


def test_k1_prep_b_then_ready_equals_one_call(device):
    """The half-pair NT's B prep carried by K1's launch (gnn_sage_mean_fwd_h2 prep_b), then the NT
    with b_ready: the image and C bit-identical to K1 alone + the one-call NT."""
    from elliptic_gnn_project_amd.fused import _nt_workspace, gemm_nt

    data, plan, x = _plan_and_x(20_000, 30_000, 5, device)
    n = 128
    g = torch.Generator().manual_seed(11)
    w1 = (torch.randn(n, x.size(1), generator=g) * 0.08).to(device)
    w2 = (torch.randn(n, x.size(1), generator=g) * 0.08).to(device)
    kw = dict(w1=w1, w2=w2, bias=torch.randn(n, generator=g).to(device), relu=True, dropout_p=0.5, seed=9)
    from elliptic_gnn_project_amd.planes import HalfPairImage

    im = HalfPairImage(x.size(0), x.size(1), x.size(1), device)
    im.fill_x(x)
    im.fill_mean(plan, x)
    img0 = im.img.clone()
    one = gemm_nt(None, None, n, planes=im, **kw)
    ws = _nt_workspace(device, n, im.k1, im.k2)
    p = gemm_nt(None, None, n, planes=im, workspace=ws, b_stage="params", **kw)
    im.fill_mean(plan, x, prep_b=p)
    assert torch.equal(im.img, img0)
    two = gemm_nt(None, None, n, planes=im, workspace=ws, b_stage="ready", **kw)
    assert torch.equal(one, two)


@pytest.mark.parametrize("cls", ["h2", "split"])
def test_k1_padded_x_equals_x(device, cls):
    """K1 over x padded with zero columns to the image's col2 (16-byte pieces, one pass per row)
    writes the image bit for bit as K1 over x itself."""
    from elliptic_gnn_project_amd.planes import HalfPairImage, SplitImage, x_padded

    data, plan, x = _plan_and_x(20_000, 30_000, 5, device)
    C = HalfPairImage if cls == "h2" else SplitImage
    im = C(x.size(0), x.size(1), x.size(1), device)
    im.fill_x(x)
    im.fill_mean(plan, x)
    img0 = im.img.clone()
    im.img.fill_(7)
    im.fill_x(x)
    xp = x_padded(x, im.col2)
    assert xp.shape == (x.size(0), im.col2) and x_padded(x, im.col2) is xp  # cached
    im.fill_mean(plan, x, x_pad=xp)
    assert torch.equal(im.img, img0)


def test_fused_sage_k1_prep_equals_nt_prep(device):
    """The SAGE train step with the layer-0 B prep inside K1's launch (default) and inside the NT
    call (GNNMP_K1_PREP=0): bit-identical logits and gradients."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(20_000, 30_000, 5, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(3)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.5).to(device).train()
    res = []
    saved, saved_pad = fused._K1_PREP, fused._K1_PAD
    for on in (True, False):
        fused._K1_PREP = on
        fused._K1_PAD = on  # (also: K1 over the padded x vs x itself)
        try:
            model.zero_grad()
            out, loss = _sage_step(model, x, ei, 79)
            loss.backward()
            res.append((out.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._K1_PREP, fused._K1_PAD = saved, saved_pad
    (o1, g1), (o2, g2) = res
    assert torch.equal(o1, o2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_fused_sage_side_prep_equals_inline(device):
    """The SAGE train step with the layer-0 B prep on the side stream (default) and in line
    (GNNMP_SIDE_PREP=0): bit-identical logits and gradients."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(20_000, 30_000, 5, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(3)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.5).to(device).train()
    res = []
    saved, saved_k1 = fused._SIDE_PREP, fused._K1_PREP
    fused._K1_PREP = False
    for on in (True, False):
        fused._SIDE_PREP = on
        try:
            model.zero_grad()
            out, loss = _sage_step(model, x, ei, 78)
            loss.backward()
            res.append((out.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._SIDE_PREP = saved
    fused._K1_PREP = saved_k1
    (o1, g1), (o2, g2) = res
    assert torch.equal(o1, o2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


@pytest.mark.parametrize("wscale", [3e4, 1e-6, 0.5])
def test_nt_h2_column_scales(device, wscale):
    """Weights far outside f16's comfortable range: every output column is scaled by its own
    power of two (largest weight into [8, 16)), so big and tiny columns stay accurate."""
    from elliptic_gnn_project_amd.fused import gemm_nt

    M, F, n = 4097, 166, 96
    agg, x, w1, w2 = _operands(M, F, n, 7, wscale)
    w1[3] *= 1e4  # one column much larger than the rest
    w2[5] *= 1e-4  # and one much smaller
    ref = torch.cat([agg, x], 1).double() @ torch.cat([w1, w2], 1).double().t()
    im = _image(agg, x, device)
    c = gemm_nt(None, None, n, planes=im, w1=w1.to(device), w2=w2.to(device))
    for j in range(n):
        assert rel_l2(c[:, j], ref[:, j]) < 1e-6, j


@pytest.mark.parametrize("M", [16, 1000, 20001, 203_769])
@pytest.mark.parametrize("dzscale,gout", [(1e-3, False), (1e-3, True), (1e-9, False), (1e4, False)])
def test_tn_h2_vs_f64(device, M, dzscale, gout):
    """dW = Gᵀ·[agg | x] with G = (dz·P) ⊙ [h > 0]·2: the dz form of the SAGE hidden layer, with
    tiny and large gradients (each row block's power-of-two G scale)."""
    from elliptic_gnn_project_amd.fused import gemm_tn

    F, nr = 166, 128
    agg, x, _, _ = _operands(M, F, 1, M + 1)
    g_ = torch.Generator().manual_seed(M)
    h = torch.relu(torch.randn(M, nr, generator=g_))
    dz = torch.randn(M, 4, generator=g_) * dzscale
    proj = torch.randn(4, nr, generator=g_)
    G = torch.where(h > 0, (dz @ proj) * 2.0, torch.zeros(M, nr))
    kw = dict(dz=dz.to(device), proj=proj.to(device), h=h.to(device), hscale=2.0)
    go = torch.empty(M, nr, device=device) if gout else None
    im = _image(agg, x, device)
    assert gemm_tn(nr, None, None, planes=im, check_planes=True, **kw)
    dW, db, dW2, dzs = gemm_tn(nr, None, None, planes=im, gout=go, **kw)
    A = torch.cat([agg, x], 1).double()
    Gd = torch.where(h > 0, (dz.double() @ proj.double()) * 2.0, torch.zeros(M, nr, dtype=torch.float64))
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), Gd.t() @ A) < 1e-6
    assert rel_l2(db, Gd.sum(0)) < 1e-6
    assert rel_l2(dW2, dz.double().t() @ h.double()) < 1e-6
    assert rel_l2(dzs, dz.double().sum(0)) < 1e-6
    if go is not None:
        torch.testing.assert_close(go.cpu(), G, rtol=1e-6, atol=1e-30)


def _sage_step(model, x, ei, seed):
    torch.manual_seed(seed)
    out = model(x, ei)
    loss = out.square().mean()
    return out, loss


@pytest.mark.parametrize("n,e", [(5000, 6000), (203_769, 234_355)])
def test_fused_sage_h2_vs_split_bf16(device, n, e):
    """The fused SAGE train step (dropout 0.5) on the half-pair image vs the split-bf16 image:
    logits and every gradient within 1e-5 (same dropout masks)."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(n, e, 5, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(3)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.5).to(device).train()
    res = []
    for on in (True, False):
        fused._H2 = on
        try:
            model.zero_grad()
            out, loss = _sage_step(model, x, ei, 123)
            loss.backward()
            res.append((out.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._H2 = True
    assert getattr(x, "_gnnmp_split_image_h2", None) is not None  # the half-pair path ran
    (o1, g1), (o2, g2) = res
    torch.testing.assert_close(o1, o2, rtol=1e-5, atol=1e-5)
    for k in g1:
        assert rel_l2(g1[k], g2[k]) < 1e-5, k


def test_fused_sage_keep_bits_equal_hash(device):
    """GNNMP_KEEP_MASK=1 (K1 writes the NT's keep bits, the NT reads them) against the default
    (the NT hashes): the same masks, so logits and gradients are bit-identical."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.gnn import SAGENet

    data, plan, x = _plan_and_x(20_000, 30_000, 5, device)
    ei = data.edge_index.to(device)
    torch.manual_seed(3)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.5).to(device).train()
    res = []
    saved = fused._KEEP_MASK
    for on in (True, False):
        fused._KEEP_MASK = on
        try:
            model.zero_grad()
            out, loss = _sage_step(model, x, ei, 77)
            loss.backward()
            res.append((out.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._KEEP_MASK = saved
    (o1, g1), (o2, g2) = res
    assert torch.equal(o1, o2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_nonfinite_input_keeps_split_bf16(device):
    """A non-finite x has no half-pair pre-scale (h2_exp None): the layer takes the split-bf16
    image.  Any finite magnitude takes the half-pair image (the scaled-input tests below)."""
    from elliptic_gnn_project_amd.gnn import SAGENet
    from elliptic_gnn_project_amd.planes import h2_exp, register_input

    data, plan, x = _plan_and_x(3000, 4000, 6, device)
    x = x.clone()
    x[0, 0] = float("inf")
    register_input(x)
    assert h2_exp(x) is None
    torch.manual_seed(4)
    model = SAGENet(x.size(1), 128, layers=2, dropout=0.0).to(device).train()
    with torch.no_grad():
        model(x, data.edge_index.to(device))
    assert getattr(x, "_gnnmp_split_image_h2", None) is None
    assert getattr(x, "_gnnmp_split_image", None) is not None


SCALES = [1e-7, 1e-5, 1e-3, 3e4]


@pytest.mark.parametrize("scale", SCALES)
def test_h2_scaled_inputs_nt_tn_vs_f64(device, scale):
    """The headline NT and TN on a half-pair image of inputs of any magnitude: [agg | x] scaled by
    1e-7 .. 3e4 (ABI 18 kept no pre-scale: 9e-5 relL2 at 1e-7, split-bf16 above 2^14) within relL2
    1e-6 of float64 — the image's power-of-two pre-scale keeps every value's f16 planes normal."""
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_tn

    M, F, n = 20001, 166, 128
    agg, x, w1, w2 = _operands(M, F, n, 17)
    agg, x = agg * scale, x * scale
    im = _image(agg, x, device)
    A = torch.cat([agg, x], 1).double()
    ref = A @ torch.cat([w1, w2], 1).double().t()
    c = gemm_nt(None, None, n, planes=im, w1=w1.to(device), w2=w2.to(device))
    assert rel_l2(c, ref) < 1e-6, rel_l2(c, ref)
    g_ = torch.Generator().manual_seed(3)
    h = torch.relu(torch.randn(M, n, generator=g_))
    dz = torch.randn(M, 4, generator=g_) * 1e-3
    proj = torch.randn(4, n, generator=g_)
    kw = dict(dz=dz.to(device), proj=proj.to(device), h=h.to(device), hscale=2.0)
    assert gemm_tn(n, None, None, planes=im, check_planes=True, **kw)
    dW, db, dW2, dzs = gemm_tn(n, None, None, planes=im, **kw)
    Gd = torch.where(h > 0, (dz.double() @ proj.double()) * 2.0, torch.zeros(M, n, dtype=torch.float64))
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), Gd.t() @ A) < 1e-6
    assert rel_l2(db, Gd.sum(0)) < 1e-6


def test_h2_power_of_two_scaling_is_exact(device):
    """x · 2^-24 and x give bitwise the same GEMM results up to the factor: the pre-scale is an
    exact power of two on both sides (image split and epilogue), so no input magnitude changes
    the rounding."""
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_tn

    M, F, n = 5000, 166, 128
    agg, x, w1, w2 = _operands(M, F, n, 23)
    g_ = torch.Generator().manual_seed(4)
    h = torch.relu(torch.randn(M, n, generator=g_))
    dz = torch.randn(M, 4, generator=g_) * 1e-2
    proj = torch.randn(4, n, generator=g_)
    kw = dict(dz=dz.to(device), proj=proj.to(device), h=h.to(device), hscale=2.0)
    out = []
    for s in (1.0, 2.0 ** -24):
        im = _image(agg * s, x * s, device)
        c = gemm_nt(None, None, n, planes=im, w1=w1.to(device), w2=w2.to(device))
        dW, _, _, _ = gemm_tn(n, None, None, planes=im, **kw)
        out.append((c / s, torch.cat([dW[0], dW[1]], 1) / s))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("arch", ["sage", "gcn"])
@pytest.mark.parametrize("scale", [1e-7, 1e-3, 3e4])
def test_fused_step_scaled_input_vs_f64(device, arch, scale):
    """The registered-input train step (SAGE: K1 into the half-pair [agg | x] image, the NT and TN
    over it; GCN: layer 1's NT on x's half-pair image) with the node features scaled by 1e-7 ..
    3e4: logits and every parameter gradient within relL2 1e-5 of the float64 oracle."""
    from oracle import pyg_ref
    from elliptic_gnn_project_amd.planes import register_input
    from elliptic_gnn_project_amd.train_gnn import build_model

    data, plan, _ = _plan_and_x(5000, 6000, 5, device)
    xs = data.x * scale
    x = register_input(xs.to(device))
    ei = data.edge_index if arch == "sage" else data.edge_index
    torch.manual_seed(6)
    model = build_model(arch, x.size(1), dict(hidden_dim=128 if arch == "sage" else 64, layers=2,
                                              dropout=0.0)).to(device).train()
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    logits = model(x, ei.to(device))
    img = "_gnnmp_split_image_h2" if arch == "sage" else "_gnnmp_split_image_x_h2"
    assert getattr(x, img, None) is not None  # the half-pair path ran
    tm = data.train_mask
    cw = pyg_ref.class_weight(data.y[tm])
    loss = pyg_ref.ce_loss(logits[tm.to(device)], data.y[tm].to(device), cw.to(device))
    loss.backward()
    p64 = {k: v.double() if v.is_floating_point() else v for k, v in params.items()}
    ref = pyg_ref.model_forward(arch, p64, xs.double(), ei, layers=2)
    assert rel_l2(logits, ref) < 1e-5
    _, grads = pyg_ref.train_step_grads(arch, p64, xs.double(), ei, data.y, tm, cw.double(), layers=2)
    for k, v in model.named_parameters():
        # at 1e-7 every node's logits are the bias: the class-weighted dlogits cancel in the output
        # bias gradient (true value ~1e-8, fp32 noise ~1e-8), so biases are held to 1e-7 absolute
        e = rel_l2(v.grad, grads[k], floor=1e-2 if k.endswith("bias") else 1e-30)
        assert e < 1e-5, (k, e)


@pytest.mark.parametrize("use_ptr", [False, True])
def test_k1_keep_bits_equal_the_dropout_hash(device, use_ptr):
    """K1 of the half-pair path writes the keep bits of the NT's dropout (bit c of word r·4 + c/32
    = keep_elem(seed, r·128 + c)) — bit for bit the oracle's mask, with a plain seed and with the
    HIP-graph device counter (seed' = counter · golden + salt)."""
    from oracle.dropout_hash import keep_mask
    from elliptic_gnn_project_amd.planes import HalfPairImage

    data, plan, x = _plan_and_x(5000, 6000, 12, device)
    im = HalfPairImage(x.size(0), x.size(1), x.size(1), device)
    kb = im.keep_buffer()
    kb.fill_(-1)
    if use_ptr:
        ctr = torch.tensor([12345], dtype=torch.int64, device=device)
        seed = ((12345 * 0x9E3779B97F4A7C15) + 3) & 0xFFFFFFFFFFFFFFFF
        im.fill_mean(plan, x, (kb, 128, 0.5, 3, ctr))
    else:
        seed = 987654321987
        im.fill_mean(plan, x, (kb, 128, 0.5, seed, None))
    want = keep_mask(seed, x.size(0), 128, 0.5)
    got = kb.cpu().numpy().view(np.uint32)
    bits = (got[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1
    assert np.array_equal(bits.reshape(x.size(0), 128).astype(bool), want)


@pytest.mark.parametrize("F,n,bias", [(166, 64, True), (166, 128, False), (40, 16, True)])
def test_input_nt_h2(device, F, n, bias):
    """y = x·Wᵀ (+ b) for a registered model input (GCN / GAT layer 1) on x's half-pair image
    (176-wide rows): within relL2 1e-6 of float64, and equal to the split-bf16 image's result
    within 1e-5."""
    from elliptic_gnn_project_amd.fused import gemm_nt, gemm_nt_input
    from elliptic_gnn_project_amd.planes import HalfPairImage, register_input, x_only_image

    M = 20000
    g = torch.Generator().manual_seed(F + n)
    x = register_input(torch.randn(M, F, generator=g).to(device))
    w = torch.randn(n, F, generator=g) * 0.1
    b = torch.randn(n, generator=g) if bias else None
    kw = dict(w1=w.to(device), bias=b.to(device) if bias else None)
    y = gemm_nt_input(x, n, **kw)
    assert getattr(x, "_gnnmp_split_image_x_h2", None) is not None
    ref = x.double().cpu() @ w.double().t() + (b.double() if bias else 0.0)
    assert rel_l2(y, ref) < 1e-6
    im = x_only_image(x)
    y2 = gemm_nt(None, None, n, planes=im, **kw)
    torch.testing.assert_close(y.cpu(), y2.cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F,nr", [(166, 64), (166, 128), (167, 64), (40, 16)])
@pytest.mark.parametrize("scale", [1.0, 1e-6, 3e4])
@pytest.mark.parametrize("prof", ["rand", "ramp", "late"])
def test_input_tn_h2_g_form(device, F, nr, scale, prof):
    """dW = Gᵀ·x, db = ΣG for a registered model input (GCN / GAT layer 1, SAGE-ResBN layer 0) on
    x's half-pair image (the plain g form of the half-pair TN, round 5): within relL2 1e-6 of
    float64 for inputs and gradients of any magnitude, and equal to the split-bf16 image's TN
    within 1e-5.  ``prof`` shapes |G| along the rows for the kernel's running block scale: ramp —
    growing 1e-4 -> 1e4 down the rows (the scale drops chunk after chunk, the accumulators are
    rescaled); late — rows zero except the last of every 800 (the scale is set by one chunk)."""
    from elliptic_gnn_project_amd.fused import gemm_tn, gemm_tn_input
    from elliptic_gnn_project_amd.planes import HalfPairImage, register_input, x_only_image

    M = 20011
    g_ = torch.Generator().manual_seed(F + nr)
    x = register_input((torch.randn(M, F, generator=g_) * scale).to(device))
    G = torch.randn(M, nr, generator=g_) * torch.exp(torch.randn(M, 1, generator=g_) * 2) * 1e-3
    if prof == "ramp":
        G = G * torch.logspace(-4, 4, M).view(M, 1)
    elif prof == "late":
        G = G * (torch.arange(M).view(M, 1) % 800 == 799)
    im = x_only_image(x, HalfPairImage)
    assert gemm_tn(nr, None, g=G.to(device), planes=im, check_planes=True)
    (dW, _), db, _, _ = gemm_tn_input(nr, x, G.to(device))
    ref = G.double().t() @ x.double().cpu()
    assert rel_l2(dW, ref) < 1e-6, rel_l2(dW, ref)
    assert rel_l2(db, G.double().sum(0)) < 1e-6
    (dW2, _), _, _, _ = gemm_tn(nr, None, g=G.to(device), planes=x_only_image(x))
    torch.testing.assert_close(dW.cpu(), dW2.cpu(), rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
