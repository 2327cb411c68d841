"""GATNet's last hidden layer with the output conv's lin on its store (ABI 24: gnn_gat_fwd_params.proj,
gnn_gat_bwd_act_proj_f32 — dh formed from d lin(h) in the kernel): the train step equals the one
with the lin as its own GEMMs (gnn._GAT_PROJ off) to fp32 accuracy, in train and eval mode, and the
fused-CE / captured paths keep working.  The full-size GAT step vs the float64 oracle
(test_gpu_fullsize.py) runs this path by default."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _graph(device, N=6000, E=15000, F=166, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, F, generator=g).to(device)
    ei = torch.randint(0, N, (2, E), generator=g)
    ei = torch.cat([ei, ei.flip(0)], 1).to(device)
    y = torch.randint(0, 2, (N,), generator=g).to(device)
    return x, ei, y


@pytest.mark.parametrize("layers,heads,hidden", [(2, 4, 64), (3, 4, 64), (2, 2, 32)])
def test_gat_proj_step_matches_unfused(device, layers, heads, hidden):
    from elliptic_gnn_project_amd import gnn

    x, ei, y = _graph(device)
    res = {}
    for on in (True, False):
        gnn._GAT_PROJ = on
        torch.manual_seed(0)
        m = gnn.GATNet(x.size(1), hidden_dim=hidden, layers=layers, dropout=0.3, heads=heads).to(device).train()
        torch.manual_seed(5)
        logits = m(x, ei)
        torch.nn.functional.cross_entropy(logits, y).backward()
        m.eval()
        with torch.no_grad():
            ev = m(x, ei)
        res[on] = (logits.detach(), ev, {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    gnn._GAT_PROJ = True
    assert _rel(res[True][0], res[False][0]) < 1e-5
    assert _rel(res[True][1], res[False][1]) < 1e-5
    for k, g in res[False][2].items():
        assert _rel(res[True][2][k], g) < 1e-5, k
