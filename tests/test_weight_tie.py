"""The fused SAGE path reads the output conv's [W_l ; W_r] as ONE buffer (fused.tie_output_weights):
the tie is made at construction and after .to()/.double()/deepcopy, survives load_state_dict, and
the stacked view always equals torch.cat(lin_l.weight, lin_r.weight).  CPU only."""
import copy

import pytest
import torch

from elliptic_gnn_project_amd import fused
from elliptic_gnn_project_amd.gnn import SAGENet


def _stack(m):
    c = m.convs[-1]
    return torch.cat([c.lin_l.weight, c.lin_r.weight], dim=0)


def _tied(m):
    return fused._tied_buffer(m.convs[-1])


@pytest.mark.parametrize("layers", [2, 3])
def test_tie_at_construction_and_after_apply(layers):
    torch.manual_seed(0)
    m = SAGENet(166, 64, layers=layers)
    assert _tied(m) is not None and torch.equal(_tied(m), _stack(m))
    m = m.double()
    assert _tied(m) is not None and _tied(m).dtype == torch.float64 and torch.equal(_tied(m), _stack(m))
    m = m.to(torch.float32)
    assert _tied(m) is not None and torch.equal(fused._output_weights(m.convs[-1]), _stack(m))


def test_tie_survives_load_state_dict_and_deepcopy():
    torch.manual_seed(1)
    a, b = SAGENet(166, 64, layers=2), SAGENet(166, 64, layers=2)
    b.load_state_dict(a.state_dict())
    assert _tied(b) is not None and torch.equal(_tied(b), _stack(a))
    sd = b.state_dict()  # two keys, values as before the tie
    assert torch.equal(sd["convs.1.lin_l.weight"], a.convs[1].lin_l.weight)
    assert torch.equal(sd["convs.1.lin_r.weight"], a.convs[1].lin_r.weight)
    c = copy.deepcopy(b)
    assert _tied(c) is not None and torch.equal(_tied(c), _stack(b))
    with torch.no_grad():
        c.convs[1].lin_r.weight.add_(1.0)  # an in-place update is seen through the view
    assert torch.equal(_tied(c), _stack(c)) and not torch.equal(_stack(c), _stack(b))


def test_replaced_parameter_falls_back_to_a_copy():
    torch.manual_seed(2)
    m = SAGENet(166, 64, layers=2)
    m.convs[1].lin_r.weight = torch.nn.Parameter(torch.randn_like(m.convs[1].lin_r.weight))
    assert _tied(m) is None
    assert torch.equal(fused._output_weights(m.convs[-1]), _stack(m))
