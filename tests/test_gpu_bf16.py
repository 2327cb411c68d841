"""bf16-storage path (BASELINE configs[4]: the scaled 2M-node 3-layer SAGE in bf16): node
features, aggregates and hidden activations stored bf16, every GEMM on bf16 operands (weights
rounded to bf16) with f32 accumulation; z, logits and gradients f32.

The reference is the same computation in float64 on the CPU with the same rounding points
(inputs, aggregates and hidden activations rounded to bf16 where the kernels store them).  The
kernels sum in a different order than the reference, so a stored bf16 value may land one bf16
ulp (2^-8 relative) away; tolerances are stated per test in those terms."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF_ULP = 2.0 ** -8


def rb(t):  # round to bf16 (RNE), back to the computing dtype
    return t.to(torch.bfloat16).to(t.dtype)


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("F", [166, 128, 7])
def test_aggregate_bf16_mean(device, F):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.graph import get_plan
    from oracle import pyg_ref

    g = torch.Generator().manual_seed(F)
    N, E = 3000, 9000
    ei = torch.randint(0, N, (2, E), generator=g)
    x = torch.randn(N, F, generator=g).to(torch.bfloat16)
    ref = pyg_ref.scatter(x.double()[ei[0]], ei[1], N, "mean")
    plan = get_plan(ei.to(device), N, _lib.LOOPS_KEEP)
    y = aggregate(plan, x.to(device), _lib.AGG_MEAN, nodew=plan.deg)
    assert y.dtype == torch.bfloat16
    d = (y.double().cpu() - ref).abs()
    assert float((d <= BF_ULP * ref.abs() + 1e-30).double().mean()) == 1.0, float(d.max())


@pytest.mark.parametrize("F", [128, 166])
def test_aggregate_bf16_mean_bwd(device, F):
    """The bf16 transposed mean (meanᵀ of the bf16-storage backward, one reciprocal per slot):
    every output within one bf16 ulp of the float64 meanᵀ, on a graph with hub rows."""
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.graph import get_plan

    g = torch.Generator().manual_seed(F + 1)
    N, E = 4000, 12000
    ei = torch.randint(0, N, (2, E), generator=g)
    ei[1, :600] = 7  # a hub destination (in-degree >= 600)
    x = torch.randn(N, F, generator=g).to(torch.bfloat16)
    deg = torch.bincount(ei[1], minlength=N).double().clamp_min(1.0)
    ref = torch.zeros(N, F, dtype=torch.float64).index_add_(0, ei[0], (x.double() / deg[:, None])[ei[1]])
    plan = get_plan(ei.to(device), N, _lib.LOOPS_KEEP)
    y = aggregate(plan, x.to(device), _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg)
    assert y.dtype == torch.bfloat16
    d = (y.double().cpu() - ref).abs()
    mag = torch.maximum(ref.abs(), y.double().cpu().abs())  # one ulp of the larger: a flip may cross a binade
    # + the f32 sum's own error where the terms cancel (an exact 0 in float64 reads ~1e-8 in f32)
    terms = torch.zeros(N, F, dtype=torch.float64).index_add_(0, ei[0], (x.double().abs() / deg[:, None])[ei[1]])
    assert float((d <= 2 * BF_ULP * mag + 2.0 ** -20 * terms).double().mean()) == 1.0, float(d.max())
    assert float((d <= BF_ULP * ref.abs() + 1e-30).double().mean()) > 0.999  # RNE's half ulp, but for ties


@pytest.mark.parametrize("M,k1,k2,n", [(3000, 166, 166, 128), (777, 128, 128, 64), (129, 30, 0, 2)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu_proj"])
def test_gemm_nt_bf16(device, M, k1, k2, n, epi):
    from elliptic_gnn_project_amd.fused import gemm_nt

    g = torch.Generator().manual_seed(M + n)
    a1 = torch.randn(M, k1, generator=g).to(torch.bfloat16)
    a2 = torch.randn(M, k2, generator=g).to(torch.bfloat16) if k2 else None
    w1 = torch.randn(n, k1, generator=g) * 0.1
    w2 = torch.randn(n, k2, generator=g) * 0.1 if k2 else None
    bias = torch.randn(n, generator=g)
    proj = torch.randn(4, n, generator=g)
    A = torch.cat([a1, a2], 1) if k2 else a1
    W = torch.cat([w1, w2], 1) if k2 else w1
    ref = A.double() @ rb(W).double().t()
    kw = {}
    z = None
    if epi != "plain":
        ref = torch.relu(ref + bias.double())
        z = torch.empty(M, 4, device=device)
        kw = dict(bias=bias.to(device), relu=True, proj=proj.to(device), z=z)
    c = gemm_nt(a1.to(device), None, n, a2=a2.to(device) if k2 else None, w1=w1.to(device),
                w2=w2.to(device) if k2 else None, **kw)
    assert c.dtype == torch.bfloat16
    d = (c.double().cpu() - ref).abs()
    assert float(d.max()) <= float((BF_ULP * ref.abs() + 1e-5).max()), float(d.max())
    assert rel_l2(c, ref) < 3e-3
    if z is not None:  # projection of the stored (bf16-rounded) h
        assert rel_l2(z, c.double().cpu() @ proj.double().t()) < 1e-5


@pytest.mark.parametrize("form", ["dz_mask", "g_mask"])
def test_gemm_tn_bf16(device, form):
    from elliptic_gnn_project_amd.fused import gemm_tn

    g_ = torch.Generator().manual_seed(5)
    M, nr, k1, k2 = 5000, 128, 166, 166
    a1 = torch.randn(M, k1, generator=g_).to(torch.bfloat16)
    a2 = torch.randn(M, k2, generator=g_).to(torch.bfloat16)
    h = torch.relu(torch.randn(M, nr, generator=g_)).to(torch.bfloat16)
    dz = torch.randn(M, 4, generator=g_) * 1e-3
    proj = torch.randn(4, nr, generator=g_)
    G = dz @ proj if form == "dz_mask" else torch.randn(M, nr, generator=g_) * 1e-3
    kw = dict(dz=dz.to(device), proj=proj.to(device)) if form == "dz_mask" else dict(g=G.to(device))
    Gm = torch.where(h.float() > 0, G * 2.0, torch.zeros_like(G))
    gout = torch.empty(M, nr, device=device)
    dW, db, dW2, _ = gemm_tn(nr, a1.to(device), a2.to(device), h=h.to(device), hscale=2.0, gout=gout, **kw)
    torch.testing.assert_close(gout.cpu(), Gm, rtol=1e-5, atol=1e-8)  # G itself stays f32
    A = torch.cat([a1, a2], 1).double()
    ref = rb(Gm).double().t() @ A  # the MFMA operand is G rounded to bf16
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), ref) < 1e-5
    assert rel_l2(db, Gm.sum(0)) < 1e-5
    if form == "dz_mask":
        assert rel_l2(dW2, dz.t().double() @ h.double()) < 1e-5


def _ref_sage_bf16(params, x_bf, ei, N, layers):
    """float64 SAGE forward with the bf16-storage rounding points (x, agg_l, h_l stored bf16; the
    hidden layers' GEMM weights rounded to bf16).  Returns (logits, saved (agg_l, h_l) list)."""
    from oracle import pyg_ref

    P = {k: v.double() for k, v in params.items()}
    h, saved = x_bf.double(), []
    for l in range(layers - 1):
        agg = rb(pyg_ref.scatter(h[ei[0]], ei[1], N, "mean"))
        pre = agg @ rb(P[f"convs.{l}.lin_l.weight"]).t() + P[f"convs.{l}.lin_l.bias"] + \
            h @ rb(P[f"convs.{l}.lin_r.weight"]).t()
        saved.append((agg, h))
        h = rb(torch.relu(pre))
    l = layers - 1
    z_l = h @ P[f"convs.{l}.lin_l.weight"].t()
    z_r = h @ P[f"convs.{l}.lin_r.weight"].t()
    logits = pyg_ref.scatter(z_l[ei[0]], ei[1], N, "mean") + z_r + P[f"convs.{l}.lin_l.bias"]
    saved.append((None, h))
    return logits, saved


def _ref_sage_bf16_grads(params, saved, dlogits, ei, N, layers):
    """Backward of _ref_sage_bf16 in float64 with the kernels' backward rounding points (bf16
    storage keeps the hidden layers' gradients in bf16, as autocast would): the TN's MFMA operand
    G = dL/dpre is rounded to bf16 for the weight gradients and stored so (gout); meanᵀ of the
    stored G is rounded to bf16 (the bf16 aggregation); dh = [meanᵀ(G) | G]·[W_l; W_r] runs with
    bf16-rounded weights and is stored bf16 (the one-product bf16 image NT); db = ΣG sums the
    unrounded G of the top hidden layer (formed in f32 from dz) and the bf16 G below it."""
    P = {k: v.double() for k, v in params.items()}
    deg = torch.bincount(ei[1], minlength=N).double().clamp_min(1.0)

    def mean_t(g):  # meanᵀ: dst-row gradient / in-degree, summed onto the sources
        return torch.zeros(N, g.size(1), dtype=g.dtype, device=g.device).index_add_(0, ei[0], (g / deg[:, None])[ei[1]])

    out = {}
    l = layers - 1
    h = saved[l][1]
    g = dlogits.double()
    mg = mean_t(g)
    out[f"convs.{l}.lin_l.weight"] = mg.t() @ h
    out[f"convs.{l}.lin_r.weight"] = g.t() @ h
    out[f"convs.{l}.lin_l.bias"] = g.sum(0)
    dh = mg @ P[f"convs.{l}.lin_l.weight"] + g @ P[f"convs.{l}.lin_r.weight"]
    for l in range(layers - 2, -1, -1):
        agg, hin = saved[l]
        G = dh * (saved[l + 1][1] > 0).double()
        Gb = rb(G)
        out[f"convs.{l}.lin_l.weight"] = Gb.t() @ agg
        out[f"convs.{l}.lin_r.weight"] = Gb.t() @ hin
        out[f"convs.{l}.lin_l.bias"] = G.sum(0)
        if l > 0:
            dh = rb(rb(mean_t(Gb)) @ rb(P[f"convs.{l}.lin_l.weight"]) + Gb @ rb(P[f"convs.{l}.lin_r.weight"]))
    return out


def test_fused_sage_bf16_train_step(device):
    """3-layer SAGE on bf16 features: logits and every parameter gradient vs the float64 reference
    with the kernels' rounding points in both directions (forward stores, the TN's bf16 G).  What
    remains is f32 summation order, which moves a stored bf16 value by one ulp (2^-8 relative)
    only where the f32 sum falls within f32 rounding of a bf16 rounding boundary (~1e-4 of the
    values): relative L2 well under 1e-3 for the logits and 2e-4 for the gradients."""
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=9000, seed=4),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    N = data.x.size(0)
    torch.manual_seed(3)
    model = SAGENet(data.x.size(1), 128, layers=3, dropout=0.0).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    x_bf = data.x.to(torch.bfloat16)
    logits = model(x_bf.to(device), data.edge_index.to(device))
    assert logits.dtype == torch.float32
    w = torch.randn(N, 2, generator=torch.Generator().manual_seed(1))
    (logits * w.to(device)).sum().backward()
    ref, saved = _ref_sage_bf16(params, x_bf, data.edge_index, N, 3)
    assert rel_l2(logits, ref) < 1e-3, rel_l2(logits, ref)
    grads = _ref_sage_bf16_grads(params, saved, w, data.edge_index, N, 3)
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 2e-4, (k, rel_l2(v.grad, grads[k]))


@pytest.mark.parametrize("M,k1,n,epi", [(3000, 166, 128, "bias_relu_drop_proj"), (777, 128, 128, "plain"),
                                        (4133, 128, 64, "bias_relu_proj"), (64, 166, 8, "bias_relu")])
def test_gemm_nt_bf16_image(device, M, k1, n, epi):
    """The weight-stationary bf16 NT on a one-plane image (gemm_nt_img16_kernel, LDS-DMA ring):
    C = epi([A1 | A2]·RNE([W1 | W2])ᵀ) stored bf16, every element within one bf16 ulp of the f64
    reference, dropout masks bit-identical to the counter hash, z = h·Pᵀ of the stored h."""
    from elliptic_gnn_project_amd.fused import gemm_nt
    from elliptic_gnn_project_amd.planes import BfImage
    from oracle.dropout_hash import keep_mask

    g = torch.Generator().manual_seed(M + n)
    im = BfImage(M, k1, k1, device, zero=True)
    a1 = torch.randn(M, k1, generator=g).to(torch.bfloat16)
    a2 = torch.randn(M, k1, generator=g).to(torch.bfloat16)
    im.a1.copy_(a1.to(device))
    im.a2.copy_(a2.to(device))
    w1 = torch.randn(n, k1, generator=g) * 0.1
    w2 = torch.randn(n, k1, generator=g) * 0.1
    bias = torch.randn(n, generator=g)
    proj = torch.randn(4, n, generator=g)
    ref = torch.cat([a1, a2], 1).double() @ rb(torch.cat([w1, w2], 1)).double().t()
    kw, z, p = {}, None, 0.0
    if epi != "plain":
        ref = torch.relu(ref + bias.double())
        kw = dict(bias=bias.to(device), relu=True)
    if "drop" in epi:
        p = 0.3
        kw.update(dropout_p=p, seed=1234)
        ref = ref * torch.from_numpy(keep_mask(1234, M, n, p)).double() / (1 - p)
    if "proj" in epi:
        z = torch.empty(M, 4, device=device)
        kw.update(proj=proj.to(device), z=z)
    out = torch.empty(M, n, dtype=torch.bfloat16, device=device)
    assert gemm_nt(None, None, n, planes=im, out=out, w1=w1.to(device), w2=w2.to(device), check_planes=True, **kw)
    c = gemm_nt(None, None, n, planes=im, out=out, w1=w1.to(device), w2=w2.to(device), **kw)
    d = (c.double().cpu() - ref).abs()
    assert float(d.max()) <= float((BF_ULP * ref.abs() + 1e-5).max()), float(d.max())
    assert rel_l2(c, ref) < 3e-3
    if z is not None:
        assert rel_l2(z, c.double().cpu() @ proj.double().t()) < 1e-5


def test_fused_sage_bf16_image_equals_tiled(device, monkeypatch):
    """The image path of the bf16-storage SAGE (BfImage operands, the image NT) and the tiled bf16
    NT over separate operands give the same logits and gradients within the bf16 rounding
    points' slack (both round the same products once; only accumulation order differs)."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=9000, seed=14),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    x_bf = data.x.to(torch.bfloat16).to(device)
    ei = data.edge_index.to(device)
    res = []
    for flag in (True, False):
        monkeypatch.setattr(fused, "_BF_IMAGE", flag)
        torch.manual_seed(3)
        model = SAGENet(data.x.size(1), 128, layers=3, dropout=0.0).to(device)
        logits = model(x_bf, ei)
        logits.square().sum().backward()
        res.append((logits.detach().cpu(), [p.grad.detach().cpu() for p in model.parameters()]))
    assert rel_l2(res[0][0], res[1][0]) < 1e-3
    for a, b in zip(res[0][1], res[1][1]):
        assert rel_l2(a, b) < 5e-3


def test_fused_sage_bf16_k1_padded_equals_unpadded(device, monkeypatch):
    """Layer 0 of the bf16-storage SAGE gathers x from the image's zero-padded A2 half at the padded
    width (168 columns, 8-byte pieces) instead of x itself (166, 4-byte): logits and gradients are
    bit for bit the same (same slot order, same f32 sums; the padding columns aggregate to zero)."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=9000, seed=15),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    x_bf = data.x.to(torch.bfloat16).to(device)
    ei = data.edge_index.to(device)
    res = []
    for flag in (True, False):
        monkeypatch.setattr(fused, "_K1_PAD", flag)
        torch.manual_seed(3)
        model = SAGENet(data.x.size(1), 128, layers=3, dropout=0.0).to(device)
        logits = model(x_bf, ei)
        logits.square().sum().backward()
        res.append((logits.detach().cpu(), [p.grad.detach().cpu() for p in model.parameters()]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("form,k1,M,gdt", [("dz_mask", 166, 5000, "f32"), ("g_mask", 166, 4133, "f32"),
                                           ("g_mask", 128, 3001, "f32"), ("dz_mask", 128, 40, "f32"),
                                           ("dz_mask", 128, 200_000, "bf16"), ("g_mask", 128, 200_000, "bf16"),
                                           ("dz_mask", 128, 6000, "bf16"), ("g_mask", 128, 5000, "bf16")])
def test_gemm_tn_bf16_image(device, form, k1, M, gdt):
    """The bf16 image TN (gemm_tn_img16_kernel, register ring D chunks ahead): dW = RNE(G)ᵀ·[A1 | A2]
    from a one-plane image, G = (dz·P or g) ⊙ mask formed in f32 (and written to gout), db, dzᵀh."""
    from elliptic_gnn_project_amd.fused import gemm_tn
    from elliptic_gnn_project_amd.planes import BfImage

    g_ = torch.Generator().manual_seed(M + k1)
    nr = 128
    im = BfImage(M, k1, k1, device, zero=True)
    a1 = torch.randn(M, k1, generator=g_).to(torch.bfloat16)
    a2 = torch.randn(M, k1, generator=g_).to(torch.bfloat16)
    im.a1.copy_(a1.to(device))
    im.a2.copy_(a2.to(device))
    h = torch.relu(torch.randn(M, nr, generator=g_)).to(torch.bfloat16)
    dz = torch.randn(M, 4, generator=g_) * 1e-3
    proj = torch.randn(4, nr, generator=g_)
    G = dz @ proj if form == "dz_mask" else torch.randn(M, nr, generator=g_) * 1e-3
    if gdt == "bf16" and form == "g_mask":
        G = G.to(torch.bfloat16).float()  # the lower layers' g arrives bf16 (the dh NT's output)
    gin = G.to(torch.bfloat16) if gdt == "bf16" else G
    kw = dict(dz=dz.to(device), proj=proj.to(device)) if form == "dz_mask" else dict(g=gin.to(device))
    Gm = torch.where(h.float() > 0, G * 2.0, torch.zeros_like(G))
    odt = torch.bfloat16 if gdt == "bf16" else torch.float32
    gout = torch.empty(M, nr, device=device, dtype=odt)
    assert gemm_tn(nr, None, None, h=h.to(device), hscale=2.0, gout=gout, planes=im, check_planes=True, **kw)
    dW, db, dW2, dzs = gemm_tn(nr, None, None, h=h.to(device), hscale=2.0, gout=gout, planes=im, **kw)
    torch.testing.assert_close(gout.cpu().float(), Gm.to(odt).float(), rtol=1e-5 if gdt == "f32" else 2.0 ** -8,
                               atol=1e-8)
    A = torch.cat([a1, a2], 1).double()
    ref = rb(Gm).double().t() @ A
    assert rel_l2(torch.cat([dW[0], dW[1]], 1), ref) < 1e-5
    assert rel_l2(db, Gm.sum(0)) < 1e-5, rel_l2(db, Gm.sum(0))
    if form == "dz_mask":
        assert rel_l2(dW2, dz.t().double() @ h.double()) < 1e-5
        assert rel_l2(dzs, dz.sum(0)) < 1e-5
