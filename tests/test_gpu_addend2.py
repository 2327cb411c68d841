"""GPU: the aggregation's second addend (gnn_agg_params.addend2, ABI 20) and its one user, the
SAGE-ResBN identity residual whose gradient the hidden conv's transposed aggregation sums in its
own store (conv.SAGEConv.forward_with_residual): bit for bit the separate add autograd made."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("F", [2, 4, 8, 64, 128, 166])
@pytest.mark.parametrize("mode", ["mean", "mean_bwd", "gcn"])
def test_addend2_equals_a_separate_add(device, F, mode):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.dataset_elliptic import synthetic_elliptic
    from elliptic_gnn_project_amd.graph import get_plan

    d = synthetic_elliptic(num_nodes=20000, num_edges=30000, seed=2)
    ei = d.edge_index.to(device)
    N = d.x.size(0)
    m, tr = {"mean": (_lib.AGG_MEAN, False), "mean_bwd": (_lib.AGG_MEAN_BWD, True), "gcn": (_lib.AGG_GCN, False)}[mode]
    plan = get_plan(ei, N, _lib.LOOPS_REPLACE if mode == "gcn" else _lib.LOOPS_KEEP)
    nodew = plan.dinv if mode == "gcn" else plan.deg
    g = torch.Generator().manual_seed(F)
    x, a1, a2 = (torch.randn(N, F, generator=g).to(device) for _ in range(3))
    ref = aggregate(plan, x, m, transpose=tr, nodew=nodew, addend=a1) + a2
    got = aggregate(plan, x, m, transpose=tr, nodew=nodew, addend=a1, addend2=a2)
    assert torch.equal(got, ref)
    got2 = aggregate(plan, x, m, transpose=tr, nodew=nodew, addend2=a2)  # addend2 alone
    assert torch.equal(got2, aggregate(plan, x, m, transpose=tr, nodew=nodew) + a2)


@pytest.mark.parametrize("te", [2, 0])
def test_resbn_identity_residual_in_the_conv_store(device, te, monkeypatch):
    """SAGE-ResBN 3L/64 (configs[3]: layer 1's residual is the identity): the train step with the
    residual gradient summed in conv 1's meanᵀ store == the step with autograd's add, every
    gradient and the logits bitwise."""
    from elliptic_gnn_project_amd.conv import SAGEConv
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
    from elliptic_gnn_project_amd.train_gnn import build_model

    data = prepare_inputs(synthetic_elliptic(num_nodes=6000, num_edges=7000, seed=8),
                          dict(use_time_scalar=te == 0, symmetrize_edges=True, train_window_k=8)).to(device)
    cfg = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, time_embed_dim=te, time_embed_type="sin",
               max_timestep=49)
    res = []
    for fold in (True, False):
        if not fold:
            monkeypatch.setattr(SAGEConv, "forward_with_residual", lambda self, x, ei: (self.forward(x, ei), x))
        torch.manual_seed(3)
        model = build_model("sage_resbn", data.x.size(1), cfg).to(device)
        model.train()
        torch.manual_seed(9)
        logits = model(data.x, data.edge_index, data.timestep if te else None)
        loss = (logits.float().square() * torch.arange(1, 3, device=device)).mean()
        loss.backward()
        res.append((logits.detach(), {k: p.grad.clone() for k, p in model.named_parameters()}))
    (la, ga), (lb, gb) = res
    assert torch.equal(la, lb)
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k
