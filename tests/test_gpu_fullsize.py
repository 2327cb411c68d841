"""GPU parity at the BASELINE.json sizes (N = 203,769, E0 = 234,355; Elliptic shape, seeded).

Train mode for the headline config (configs[1], SAGE 2L 166->128->2, dropout 0.5): every
parameter gradient of the fused step against the oracle run in float64 with the very same
dropout masks (oracle/dropout_hash.py), relative L2 <= 1e-5 — this exercises the full-size
TN slab reduction (~1,600 row blocks) and the hub rows' long-segment split path with gradients
on.  Eval logits of the GCN (configs[0] preset, 2L/64) and GAT (configs[2] preset, 2L 4x16)
networks at full size, rtol = atol = 1e-5.  The float64 oracle is the truth the fp32 GPU
result is held to (fp32 CPU and GPU differ from it by their own rounding).
"""
import pytest
import torch

from oracle import pyg_ref
from oracle.dropout_hash import keep_mask

pytestmark = pytest.mark.gpu

N_FULL, E_FULL = 203_769, 234_355


def rel_l2(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


_CACHE = {}


def _graph(sym):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    if sym not in _CACHE:
        _CACHE[sym] = prepare_inputs(synthetic_elliptic(num_nodes=N_FULL, num_edges=E_FULL, seed=42),
                                     dict(use_time_scalar=True, symmetrize_edges=sym, train_window_k=10))
    return _CACHE[sym]


def _f64(params):
    return {k: v.double() if v.is_floating_point() else v for k, v in params.items()}


def test_full_size_sage_train_step_gradients(device):
    """configs[1] at full size, train mode: logits and all 6 parameter gradients."""
    from elliptic_gnn_project_amd.gnn import SAGENet

    data = _graph(True)
    assert data.edge_index.size(1) == 2 * E_FULL
    N = data.x.size(0)
    torch.manual_seed(5)
    model = SAGENet(166, 128, layers=2, dropout=0.5).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    torch.manual_seed(123)
    logits = model(data.x.to(device), data.edge_index.to(device))
    torch.manual_seed(123)
    seeds = torch.randint(0, 2 ** 62, (2,), dtype=torch.int64).tolist()
    masks = [torch.from_numpy(keep_mask(seeds[0], N, 128, 0.5))]
    tm = data.train_mask
    cw = pyg_ref.class_weight(data.y[tm])
    loss = pyg_ref.ce_loss(logits[tm.to(device)], data.y[tm].to(device), cw.to(device))
    loss.backward()
    kw = dict(layers=2, dropout=0.5, training=True, dropout_masks=masks)
    x64 = data.x.double()
    ref_logits = pyg_ref.model_forward("sage", _f64(params), x64, data.edge_index, **kw)
    torch.testing.assert_close(logits.detach().cpu().double(), ref_logits, rtol=1e-5, atol=1e-5)
    ref_loss, grads = pyg_ref.train_step_grads("sage", _f64(params), x64, data.edge_index, data.y, tm,
                                               cw.double(), **kw)
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 1e-5, (k, rel_l2(v.grad, grads[k]))


@pytest.mark.parametrize("arch,hidden,heads", [("gcn", 64, 4), ("gat", 64, 4)])
def test_full_size_eval_logits(device, arch, hidden, heads):
    """configs[0] (GCN 2L/64) and configs[2] (GAT 2L, 4 heads x 16) presets at full size
    (symmetrize_edges false, self loops added by the convs), eval mode."""
    from elliptic_gnn_project_amd.train_gnn import build_model

    data = _graph(False)
    torch.manual_seed(8)
    model = build_model(arch, 166, dict(hidden_dim=hidden, layers=2, dropout=0.5, heads=heads)).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.eval()
    with torch.no_grad():
        out = model(data.x.to(device), data.edge_index.to(device)).cpu()
    ref = pyg_ref.model_forward(arch, _f64(params), data.x.double(), data.edge_index, layers=2, heads=heads)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)
