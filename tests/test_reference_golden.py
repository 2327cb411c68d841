"""The oracle's model composition against vectors the REFERENCE's own code produced.

tests/golden/reference_models.npz comes from tests/golden/make_reference_golden.py, which runs
/root/reference/src/models/gnn.py unmodified (PyG's convs supplied by the oracle's restatement,
PyG not being installable here).  So this pins oracle/pyg_ref.model_forward's composition layer
— time embedding, BN order, residual projections, activations, head concat / mean — to the
reference itself: train-mode logits and every gradient, the BN running statistics after the
step, and eval-mode logits.  CPU only; tests/test_gpu_reference_golden.py replays the same
vectors through libgnnmp.
"""
import os

import numpy as np
import pytest
import torch

from oracle import pyg_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_models.npz")
ARCH = {"gcn": ("gcn", 2, {}), "sage": ("sage", 3, {}), "gat": ("gat", 2, dict(heads=4)),
        "resbn_sin": ("sage_resbn", 3, dict(time_embed_dim=2, time_embed_type="sin")),
        "resbn_learned": ("sage_resbn", 3, dict(time_embed_dim=4, time_embed_type="learned"))}


def load(name):
    z = np.load(GOLD, allow_pickle=False)
    pre = name + "/"
    g = {k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)}
    state0 = {k[len("state0/"):]: v for k, v in g.items() if k.startswith("state0/")}
    state1 = {k[len("state1/"):]: v for k, v in g.items() if k.startswith("state1/")}
    grads = {k[len("grad/"):]: v for k, v in g.items() if k.startswith("grad/")}
    return g, state0, state1, grads


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-2))


@pytest.mark.parametrize("name", sorted(ARCH))
def test_oracle_composition_matches_reference(name):
    arch, layers, kw = ARCH[name]
    g, state0, state1, grads = load(name)
    t_idx = g["timestep"] if "time_embed_dim" in kw else None
    params = {k: v for k, v in state0.items() if v.is_floating_point() and "running" not in k}
    kw = dict(kw, layers=layers, training=True, t_idx=t_idx)
    logits = pyg_ref.model_forward(arch, params, g["x"], g["edge_index"], **kw)
    torch.testing.assert_close(logits, g["logits_train"], rtol=1e-5, atol=1e-5)
    loss, gr = pyg_ref.train_step_grads(arch, params, g["x"], g["edge_index"], g["y"], g["train_mask"],
                                        g["cw"], **kw)
    assert abs(float(loss) - float(g["loss"])) < 1e-5
    for k, v in grads.items():
        assert rel_l2(gr[k], v) < 1e-5, k
    # eval mode on the reference's BN running statistics after the step
    kw_eval = dict(kw, training=False, bn_state=state1) if state1 else dict(kw, training=False)
    out = pyg_ref.model_forward(arch, params, g["x"], g["edge_index"], **kw_eval)
    torch.testing.assert_close(out, g["logits_eval"], rtol=1e-5, atol=1e-5)
