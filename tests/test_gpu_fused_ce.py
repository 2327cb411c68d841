"""GPU: the SAGE output layer's mean and the masked weighted CE in one launch
(include/gnnmp.h gnn_sage_out_mean_ce_f32, train_ops.fused_ce_target) — bit for bit the two
launches it replaces (gnn_aggregate_f32 MEAN + addend + bias, then gnn_masked_ce_f32): logits,
dlogits, the loss partials and the loss; at the model level every gradient of the train step,
eager and replayed from a captured HIP graph (src/train_gnn.py:187-209)."""
import pytest
import torch

from oracle import pyg_ref

pytestmark = pytest.mark.gpu


def _data(n, e, seed, device):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    return prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10)).to(device)


@pytest.mark.parametrize("n,e,C", [(5000, 6000, 2), (203_769, 234_355, 2), (777, 900, 3), (64, 0, 2), (300, 500, 4)])
def test_out_mean_ce_equals_two_launches(device, n, e, C):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.graph import get_plan
    from elliptic_gnn_project_amd.train_ops import _ce_operands, _MaskedCE, sage_out_mean_ce

    data = _data(n, e, 3, device)
    N = data.x.size(0)
    plan = get_plan(data.edge_index, N, _lib.LOOPS_KEEP)
    g = torch.Generator().manual_seed(n + C)
    z = (torch.randn(N, 2 * C, generator=g) * 2).to(device)
    bias = torch.randn(C, generator=g).to(device)
    y = torch.randint(0, C, (N,), generator=g).to(device)
    mask = (torch.rand(N, generator=g) < 0.6).to(device)
    mask[0] = True
    w = (torch.rand(C, generator=g) + 0.5).to(device)
    denom = float(mask.sum())
    ref_logits = aggregate(plan, z[:, :C], _lib.AGG_MEAN, nodew=plan.deg, addend=z[:, C:], bias=bias)
    key, yy, m8, ww, inv = _ce_operands(y, mask, w, denom, device)
    ref_loss = _MaskedCE.apply(ref_logits.requires_grad_(True), yy, m8, ww, inv)
    ref_loss.backward()
    logits, ce = sage_out_mean_ce(plan, z, C, bias, (key, yy, m8, ww, inv))
    assert torch.equal(logits, ref_logits.detach())
    assert torch.equal(ce[1], ref_loss.detach())  # the loss: same partials, same finish
    assert torch.equal(ce[2][:, C:], ref_logits.grad)  # dlogits (unit upstream gradient)
    # u = dlogits / max(deg, 1): its CSC sum is MEAN_BWD's meanᵀ(dlogits), bit for bit
    u = ce[2]._gnnmp_u
    assert torch.equal(u, ref_logits.grad / plan.deg.clamp(min=1.0).view(N, 1))
    assert torch.equal(aggregate(plan, u, _lib.AGG_SUM, transpose=True),
                       aggregate(plan, ref_logits.grad, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg))
    # vs the float64 oracle of the reference's loss (src/train_gnn.py:159-175)
    lo = pyg_ref.ce_loss(ref_logits.detach().double().cpu()[mask.cpu()], y.cpu()[mask.cpu()], w.double().cpu())
    assert abs(float(ce[1]) - float(lo)) <= 1e-5 * max(1.0, abs(float(lo)))


def _setup(device, seed=11, dropout=0.5):
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model
    from elliptic_gnn_project_amd.train_ops import ClipAdam

    data = _data(4000, 5000, 9, device)
    torch.manual_seed(seed)
    model = build_model("sage", data.x.size(1), dict(hidden_dim=128, layers=2, dropout=dropout)).to(device)
    opt = ClipAdam(model.parameters(), lr=0.01, weight_decay=1e-4, max_norm=1.0)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    loss_fn = _make_loss_fn({}, cw, model, 1, 34)
    denom = float(data.train_mask.sum())
    return data, model, opt, loss_fn, denom


@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_train_step_with_fused_ce_equals_separate(device, dropout):
    """The train step with the CE computed in the output layer's launch (loss_fn.target) and
    without: bit-identical logits, loss and gradients."""
    res = []
    for fused in (True, False):
        data, model, opt, loss_fn, denom = _setup(device, dropout=dropout)
        model.train()
        torch.manual_seed(5)
        if fused:
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index)
            assert getattr(logits, "_gnnmp_ce", None) is not None
        else:
            logits = model(data.x, data.edge_index)
            assert getattr(logits, "_gnnmp_ce", None) is None
        loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
        loss.backward()
        res.append((logits.detach().clone(), loss.detach().clone(),
                    {k: p.grad.clone() for k, p in model.named_parameters()}))
    (l1, s1, g1), (l2, s2, g2) = res
    assert torch.equal(l1, l2) and torch.equal(s1, s2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_fused_ce_ignored_for_other_operands(device):
    """A loss over other operands than the target's (here another mask) launches its own CE."""
    data, model, opt, loss_fn, denom = _setup(device, dropout=0.0)
    model.train()
    with loss_fn.target(data.y, data.train_mask, denom):
        logits = model(data.x, data.edge_index)
    other = data.train_mask.clone()
    other[: other.numel() // 2] = False
    d2 = float(other.sum())
    a = loss_fn.full(logits, data.y, other, denom=d2)
    b = loss_fn.full(logits.detach().clone().requires_grad_(True), data.y, other, denom=d2)
    assert torch.equal(a.detach(), b.detach())


@pytest.mark.parametrize("defer_loss", [False, True])
def test_captured_step_with_fused_ce_matches_eager(device, defer_loss):
    """bench.py's step (fused CE, ClipAdam) replayed from a captured graph == the same step eager,
    parameters bitwise after 5 steps, the replayed loss == the eager one."""
    from elliptic_gnn_project_amd.train_gnn import CapturedStep
    from elliptic_gnn_project_amd.train_ops import unit_gradient

    def make():
        data, model, opt, loss_fn, denom = _setup(device, dropout=0.0)

        def step():
            model.train()
            opt.zero_grad(set_to_none=True)
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index)
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
            loss.backward(unit_gradient(loss.device))
            opt.step()
            return loss.detach()
        return model, step

    m_e, step_e = make()
    losses = [float(step_e()) for _ in range(5)]
    m_g, step_g = make()
    cs = CapturedStep(step_g, warmup=3, defer_loss=defer_loss)
    cs()
    out = cs()
    torch.cuda.synchronize()
    assert float(out) == losses[-1]
    for (k, a), b in zip(m_e.state_dict().items(), m_g.state_dict().values()):
        assert torch.equal(a, b), k


@pytest.mark.parametrize("dropout", [0.0, 0.5])
@pytest.mark.parametrize("unit", [False, True])
def test_gcn_step_with_fused_ce_equals_separate(device, dropout, unit):
    """GCN (configs[0] preset): the train step with the CE in the output aggregation's launch
    (gnn_gcn_out_ce_f32 under loss_fn.target) and with the two launches: bit-identical logits,
    loss and every gradient — the output bias gradient from the fused launch's dlogits column
    sums (unit_gradient path) included."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model
    from elliptic_gnn_project_amd.train_ops import unit_gradient

    data = _data(4000, 5000, 9, device)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    denom = float(data.train_mask.sum())
    res = []
    for on in (True, False):
        fused._GCN_CE = on
        try:
            torch.manual_seed(11)
            model = build_model("gcn", data.x.size(1), dict(hidden_dim=64, layers=2, dropout=dropout)).to(device)
            loss_fn = _make_loss_fn({}, cw, model, 1, 34)
            model.train()
            torch.manual_seed(5)
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index)
            assert (getattr(logits, "_gnnmp_ce", None) is not None) == on
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
            loss.backward(unit_gradient(device)) if unit else loss.backward()
            res.append((logits.detach().clone(), loss.detach().clone(),
                        {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._GCN_CE = True
    (l1, s1, g1), (l2, s2, g2) = res
    assert torch.equal(l1, l2) and torch.equal(s1, s2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


@pytest.mark.parametrize("dropout", [0.0, 0.5])
@pytest.mark.parametrize("unit", [False, True])
def test_gat_step_with_fused_ce_equals_separate(device, dropout, unit):
    """GAT (configs[2] preset 2L 4x16): the output conv in the narrow form with the CE in its
    launch (gnn_gat_out_ce_f32 under loss_fn.target) and with the CE in its own launch:
    bit-identical logits, loss and every gradient (the output bias gradient from the fused
    launch's dlogits column sums on the unit_gradient path included)."""
    from elliptic_gnn_project_amd import aggregation
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model
    from elliptic_gnn_project_amd.train_ops import unit_gradient

    data = _data(4000, 5000, 9, device)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    denom = float(data.train_mask.sum())
    res = []
    for on in (True, False):
        aggregation._GAT_CE = on
        try:
            torch.manual_seed(11)
            model = build_model("gat", data.x.size(1), dict(hidden_dim=64, heads=4, layers=2, dropout=dropout)).to(device)
            loss_fn = _make_loss_fn({}, cw, model, 1, 34)
            model.train()
            torch.manual_seed(5)
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index)
            assert (getattr(logits, "_gnnmp_ce", None) is not None) == on
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
            loss.backward(unit_gradient(device)) if unit else loss.backward()
            res.append((logits.detach().clone(), loss.detach().clone(),
                        {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            aggregation._GAT_CE = True
    (l1, s1, g1), (l2, s2, g2) = res
    assert torch.equal(l1, l2) and torch.equal(s1, s2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


@pytest.mark.parametrize("unit", [False, True])
def test_resbn_step_with_fused_out_ce_equals_separate(device, unit):
    """SAGE-ResBN (configs[3]): its transform-first output conv runs the mean and the masked CE in
    one launch under loss_fn.target (gnn_sage_out_mean_ce_f32 with dlogits' column sums; the
    backward's meanᵀ as the CSC sum of u) — bit-identical logits, loss and gradients to the two
    launches (conv._OUT_CE off)."""
    from elliptic_gnn_project_amd import conv
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model
    from elliptic_gnn_project_amd.train_ops import unit_gradient

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=7000, seed=8),
                          dict(use_time_scalar=False, symmetrize_edges=True, train_window_k=8)).to(device)
    cfg = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, time_embed_dim=2, time_embed_type="sin",
               max_timestep=49)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    denom = float(data.train_mask.sum())
    res = []
    for on in (True, False):
        conv._OUT_CE = on
        try:
            torch.manual_seed(3)
            model = build_model("sage_resbn", data.x.size(1), cfg).to(device)
            loss_fn = _make_loss_fn({}, cw, model, 1, 34)
            model.train()
            torch.manual_seed(9)
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index, data.timestep)
            assert (getattr(logits, "_gnnmp_ce", None) is not None) == on
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
            loss.backward(unit_gradient(device)) if unit else loss.backward()
            res.append((logits.detach().clone(), loss.detach().clone(),
                        {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            conv._OUT_CE = True
    (l1, s1, g1), (l2, s2, g2) = res
    assert torch.equal(l1, l2) and torch.equal(s1, s2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_resbn_bn_colsum_bias_gradient(device):
    """SAGE-ResBN: K12's backward writing dz's block column sums (gnn_bn_act_bwd_colsum_f32), which
    become the layer-0 conv's bias gradient (colsum_of): every other gradient bit-identical to the
    separate colsum pass, that bias gradient (a BN-cancelled sum: analytically 0) within 1e-6 of it
    relative to Σ|dz|, and the logits / loss unchanged."""
    from elliptic_gnn_project_amd import fused
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model
    from elliptic_gnn_project_amd.train_ops import unit_gradient

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=7000, seed=8),
                          dict(use_time_scalar=False, symmetrize_edges=True, train_window_k=8)).to(device)
    cfg = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, time_embed_dim=2, time_embed_type="sin",
               max_timestep=49)
    cw = pyg_ref.class_weight(data.y[data.train_mask].cpu())
    denom = float(data.train_mask.sum())
    res = []
    for on in (True, False):
        fused._BN_COLSUM = on
        try:
            torch.manual_seed(3)
            model = build_model("sage_resbn", data.x.size(1), cfg).to(device)
            loss_fn = _make_loss_fn({}, cw, model, 1, 34)
            model.train()
            torch.manual_seed(9)
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index, data.timestep)
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
            loss.backward(unit_gradient(device))
            res.append((logits.detach().clone(), loss.detach().clone(),
                        {k: p.grad.clone() for k, p in model.named_parameters()}))
        finally:
            fused._BN_COLSUM = True
    (l1, s1, g1), (l2, s2, g2) = res
    assert torch.equal(l1, l2) and torch.equal(s1, s2)
    bias0 = "convs.0.lin_l.bias"
    assert bias0 in g1
    for k in g1:
        if k == bias0:
            scale = float(g1["convs.0.lin_l.weight"].abs().max())
            assert float((g1[k] - g2[k]).abs().max()) <= 1e-6 * max(1.0, scale), k
        else:
            assert torch.equal(g1[k], g2[k]), k
