"""GPU parity of explain mode: the per-edge message multiplier that
GNNExplainer optimises (src/analysis/explain.py:593-672 via PyG set_masks) on SAGEConv.

Oracle: oracle/pyg_ref.sage_conv_explain (PyG 2.5.3 propagate with `explain` on), fp32,
rtol = atol = 1e-5 on outputs, relative L2 <= 1e-5 on the mask / x / weight gradients.
Parity against PyG itself is unpinned (PyG is not installed; the reference has no fixture).
"""
import pytest
import torch

from oracle import pyg_ref

from test_gpu_parity import GRAPHS, rand_graph, rel_l2

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("F", [1, 5, 64, 166])
def test_masked_mean_fwd_bwd(device, name, F):
    from elliptic_gnn_project_amd.aggregation import masked_mean_aggregate

    spec = GRAPHS[name]
    ei = rand_graph(**spec)
    n, E = spec["n"], ei.size(1)
    g = torch.Generator().manual_seed(17)
    x = torch.randn(n, F, generator=g)
    m = torch.rand(E, generator=g)
    xg = x.to(device).requires_grad_(True)
    mg = m.to(device).requires_grad_(True)
    out = masked_mean_aggregate(xg, ei.to(device), mg)
    xr, mr = x.clone().requires_grad_(True), m.clone().requires_grad_(True)
    ref = pyg_ref.scatter(xr.index_select(0, ei[0]) * mr.view(-1, 1), ei[1], n, "mean")
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    dy = torch.randn(n, F, generator=g)
    out.backward(dy.to(device))
    ref.backward(dy)
    assert rel_l2(xg.grad, xr.grad) <= 1e-5
    assert rel_l2(mg.grad, mr.grad) <= 1e-5


def test_sage_conv_explain_mode(device):
    from elliptic_gnn_project_amd.conv import SAGEConv, clear_masks, set_masks

    ei = rand_graph(**GRAPHS["medium"])
    n, E = GRAPHS["medium"]["n"], ei.size(1)
    torch.manual_seed(3)
    conv = SAGEConv(166, 16).to(device)
    p = {k: v.detach().cpu() for k, v in conv.state_dict().items()}
    x = torch.randn(n, 166)
    logit = torch.randn(E) * 2.0
    mg = logit.to(device).requires_grad_(True)
    set_masks(conv, mg, ei.to(device), apply_sigmoid=True)
    out = conv(x.to(device), ei.to(device))
    mr = logit.clone().requires_grad_(True)
    ref = pyg_ref.sage_conv_explain(x, ei, mr, p["lin_l.weight"], p["lin_l.bias"], p["lin_r.weight"])
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    out.square().sum().backward()
    ref.square().sum().backward()
    assert rel_l2(mg.grad, mr.grad) <= 1e-5
    assert rel_l2(conv.lin_l.weight.grad, _ref_grad(x, ei, logit, p)) <= 1e-5
    clear_masks(conv)  # back to the plain path: equals the unmasked oracle
    out2 = conv(x.to(device), ei.to(device))
    ref2 = pyg_ref.sage_conv(x, ei, p["lin_l.weight"], p["lin_l.bias"], p["lin_r.weight"])
    torch.testing.assert_close(out2.detach().cpu(), ref2, rtol=1e-5, atol=1e-5)


def _ref_grad(x, ei, logit, p):
    w = p["lin_l.weight"].clone().requires_grad_(True)
    pyg_ref.sage_conv_explain(x, ei, logit, w, p["lin_l.bias"], p["lin_r.weight"]).square().sum().backward()
    return w.grad


def test_sagenet_explain_bypasses_fused(device):
    """A SAGENet in explain mode runs the per-conv path and matches the oracle model with masks."""
    from elliptic_gnn_project_amd.conv import set_masks
    from elliptic_gnn_project_amd.gnn import SAGENet

    ei = rand_graph(**GRAPHS["small"])
    n, E = GRAPHS["small"]["n"], ei.size(1)
    torch.manual_seed(5)
    model = SAGENet(8, 16, layers=2, dropout=0.0).to(device).eval()
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    x = torch.randn(n, 8)
    logit = torch.randn(E)
    set_masks(model, logit.to(device), ei.to(device))
    out = model(x.to(device), ei.to(device))
    h = pyg_ref.sage_conv_explain(x, ei, logit, p["convs.0.lin_l.weight"], p["convs.0.lin_l.bias"],
                                  p["convs.0.lin_r.weight"]).relu()
    ref = pyg_ref.sage_conv_explain(h, ei, logit, p["convs.1.lin_l.weight"], p["convs.1.lin_l.bias"],
                                    p["convs.1.lin_r.weight"])
    torch.testing.assert_close(out.detach().cpu(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", list(GRAPHS))
def test_gcn_conv_explain_mode(device, name):
    """GCNConv explain mode: input self loops lose their mask (PyG `_loop_mask`), appended loops
    carry 1; outputs and mask / weight / bias gradients vs the oracle."""
    from elliptic_gnn_project_amd.conv import GCNConv, set_masks

    spec = GRAPHS[name]
    ei = rand_graph(**spec)
    n, E = spec["n"], ei.size(1)
    torch.manual_seed(9)
    conv = GCNConv(24, 8).to(device)
    with torch.no_grad():
        conv.bias.normal_()
    p = {k: v.detach().cpu() for k, v in conv.state_dict().items()}
    x = torch.randn(n, 24, generator=torch.Generator().manual_seed(4))
    logit = torch.randn(E, generator=torch.Generator().manual_seed(5)) * 2.0
    mg = logit.to(device).requires_grad_(True)
    set_masks(conv, mg, ei.to(device))
    out = conv(x.to(device), ei.to(device))
    mr = logit.clone().requires_grad_(True)
    w = p["lin.weight"].clone().requires_grad_(True)
    b = p["bias"].clone().requires_grad_(True)
    ref = pyg_ref.gcn_conv_explain(x, ei, mr, w, b)
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    dy = torch.randn(n, 8, generator=torch.Generator().manual_seed(6))
    out.backward(dy.to(device))
    ref.backward(dy)
    assert rel_l2(mg.grad, mr.grad) <= 1e-5
    assert rel_l2(conv.lin.weight.grad, w.grad) <= 1e-5
    assert rel_l2(conv.bias.grad, b.grad) <= 1e-5


@pytest.mark.parametrize("name", list(GRAPHS))
@pytest.mark.parametrize("cfg", [(24, 8, 4, True), (16, 2, 1, False), (12, 3, 2, False)])
def test_gat_conv_explain_mode(device, name, cfg):
    """GATConv explain mode: messages alpha * xh_j scaled by the sigmoided mask after
    the softmax, input self loops lose their mask, appended loops carry 1; outputs and the mask /
    weight / attention / bias gradients vs the oracle's PyG restatement."""
    from elliptic_gnn_project_amd.conv import GATConv, clear_masks, set_masks

    fin, C, H, concat = cfg
    spec = GRAPHS[name]
    ei = rand_graph(**spec)
    n, E = spec["n"], ei.size(1)
    torch.manual_seed(10)
    conv = GATConv(fin, C, heads=H, concat=concat).to(device)
    with torch.no_grad():
        conv.bias.normal_()
    p = {k: v.detach().cpu() for k, v in conv.state_dict().items()}
    x = torch.randn(n, fin, generator=torch.Generator().manual_seed(4))
    logit = torch.randn(E, generator=torch.Generator().manual_seed(5)) * 2.0
    mg = logit.to(device).requires_grad_(True)
    set_masks(conv, mg, ei.to(device))
    out = conv(x.to(device), ei.to(device))
    mr = logit.clone().requires_grad_(True)
    leaf = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    ref = pyg_ref.gat_conv_explain(x, ei, mr, leaf["lin.weight"], leaf["att_src"], leaf["att_dst"], leaf["bias"],
                                   H, C, concat=concat)
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    dy = torch.randn(ref.shape, generator=torch.Generator().manual_seed(6))
    out.backward(dy.to(device))
    ref.backward(dy)
    assert rel_l2(mg.grad, mr.grad) <= 1e-5
    for k, v in conv.named_parameters():
        assert rel_l2(v.grad, leaf[k].grad) <= 1e-5, k
    clear_masks(conv)  # back to the fused path: equals the unmasked oracle
    with torch.no_grad():
        plain = conv(x.to(device), ei.to(device))
    ref0 = pyg_ref.gat_conv(x, ei, p["lin.weight"], p["att_src"], p["att_dst"], p["bias"], H, C, concat=concat)
    torch.testing.assert_close(plain.cpu(), ref0, rtol=1e-5, atol=1e-5)
