"""libgnnmp's four model families against vectors the REFERENCE's own composition produced
(tests/golden/reference_models.npz, tests/golden/make_reference_golden.py: /root/reference's
src/models/gnn.py run unmodified with the oracle's PyG conv restatement).  Same state_dict
loaded into elliptic_gnn_project_amd.gnn's models; train-mode logits and the loss
(rtol = atol = 1e-5), every parameter gradient (relative L2 <= 1e-5), the BatchNorm running
statistics after the step and eval-mode logits."""
import numpy as np
import pytest
import torch

from test_reference_golden import ARCH, load, rel_l2

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(ARCH))
def test_hip_models_match_reference_composition(device, name):
    from elliptic_gnn_project_amd.train_gnn import build_model

    arch, layers, kw = ARCH[name]
    g, state0, state1, grads = load(name)
    hidden = state0["convs.0.lin.weight" if arch in ("gcn", "gat") else "convs.0.lin_l.weight"].size(0)
    cfg = dict(hidden_dim=hidden, layers=layers, dropout=0.0, heads=kw.get("heads", 4),
               time_embed_dim=kw.get("time_embed_dim", 0), time_embed_type=kw.get("time_embed_type", "none"),
               max_timestep=49)
    model = build_model(arch, g["x"].size(1), cfg).to(device)
    model.load_state_dict({k: v.to(device) for k, v in state0.items()})
    model.train()
    x, ei = g["x"].to(device), g["edge_index"].to(device)
    t_idx = g["timestep"].to(device) if "time_embed_dim" in kw else None
    logits = model(x, ei, t_idx)
    torch.testing.assert_close(logits.detach().cpu(), g["logits_train"], rtol=1e-5, atol=1e-5)
    tm = g["train_mask"].to(device)
    loss = torch.nn.functional.cross_entropy(logits[tm], g["y"].to(device)[tm], weight=g["cw"].to(device),
                                             reduction="none").mean()
    assert abs(float(loss) - float(g["loss"])) < 1e-5
    loss.backward()
    for k, p in model.named_parameters():
        assert rel_l2(p.grad.cpu(), grads[k]) < 1e-5, k
    sd = model.state_dict()
    for k, v in state1.items():
        if "running" in k:
            torch.testing.assert_close(sd[k].cpu(), v, rtol=1e-5, atol=1e-6)
    model.eval()
    with torch.no_grad():
        out = model(x, ei, t_idx)
    torch.testing.assert_close(out.cpu(), g["logits_eval"], rtol=1e-5, atol=1e-5)
