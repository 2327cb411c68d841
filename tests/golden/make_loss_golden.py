"""Golden vectors of the REFERENCE's loss variants (build container only).

Imports /root/reference/src/train_gnn.py unmodified and calls its own ``class_weight``
(src/train_gnn.py:116-123) and ``_make_loss_fn`` (src/train_gnn.py:136-183) on seeded logits:
class-weighted CE, focal loss (gamma 1 and 2), time weighting (linear / sqrt, with the 1e-3
clamp: the first training timestep's rows get weight 1e-3) and the learned-time-embedding L2.
Stored per case: the loss and d loss / d logits (and d loss / d time_emb.weight for the L2 case).
Writes tests/golden/loss_golden.npz; tests/test_loss_golden.py replays it.

Modules the reference imports that are absent here are stubbed with inert stand-ins:
``torch_geometric.{nn,loader,data}`` (the convs of the oracle, never called by the loss) and
``torch.utils.tensorboard`` (RunLogger's writer, never instantiated).  Nothing of the reference
is copied: the .npz holds arrays only.

    python tests/golden/make_loss_golden.py [/root/reference]
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

CASES = {
    # name: (cfg, model has a learned time embedding)
    "ce_weighted": (dict(), False),
    "focal_g1": (dict(focal_loss=True, focal_gamma=1.0), False),
    "focal_g2": (dict(focal_loss=True, focal_gamma=2.0), False),
    "time_linear": (dict(time_loss_weighting="linear"), False),
    "time_sqrt": (dict(time_loss_weighting="sqrt"), False),
    "focal_time_sqrt": (dict(focal_loss=True, focal_gamma=2.0, time_loss_weighting="sqrt"), False),
    "embed_l2": (dict(time_embed_l2=0.01), True),
    "time_linear_embed_l2": (dict(time_loss_weighting="linear", time_embed_l2=0.05), True),
}
T_MIN, T_MAX = 1, 34  # the split's training window (configs/split.yaml: train <= 34)


def _install_stubs():
    from make_reference_golden import _install_pyg_stub

    _install_pyg_stub()
    pyg = sys.modules["torch_geometric"]
    for sub in ("loader", "data"):
        m = types.ModuleType(f"torch_geometric.{sub}")
        setattr(pyg, sub, m)
        sys.modules[f"torch_geometric.{sub}"] = m
    sys.modules["torch_geometric.loader"].NeighborLoader = object
    sys.modules["torch_geometric.data"].Data = object
    try:
        import torch.utils.tensorboard  # noqa: F401
    except ModuleNotFoundError:
        tb = types.ModuleType("torch.utils.tensorboard")
        tb.SummaryWriter = object
        sys.modules["torch.utils.tensorboard"] = tb


class _TimeModel(torch.nn.Module):
    """Just the attributes the reference's loss probes (src/train_gnn.py:126-127,178-181)."""

    def __init__(self, with_emb: bool, gen):
        super().__init__()
        self.time_embed_dim = 4 if with_emb else 0
        self.time_emb = torch.nn.Embedding(50, 4) if with_emb else None
        if with_emb:
            with torch.no_grad():
                self.time_emb.weight.copy_(torch.randn(50, 4, generator=gen))


def main(ref_root: str = "/root/reference"):
    _install_stubs()
    sys.path.insert(0, ref_root)
    from src import train_gnn as ref

    gen = torch.Generator().manual_seed(2024)
    n = 257
    logits = torch.randn(n, 2, generator=gen) * 2.0
    y = (torch.rand(n, generator=gen) < 0.2).long()
    t_idx = torch.randint(T_MIN, T_MAX + 1, (n,), generator=gen)
    t_idx[:5] = T_MIN  # rows whose time weight is clamped to 1e-3
    cw = ref.class_weight(y)
    out = {"logits": logits.numpy(), "y": y.numpy(), "t_idx": t_idx.numpy(), "class_weight": cw.numpy(),
           "class_weight_allpos": ref.class_weight(torch.ones(7, dtype=torch.long)).numpy(),
           "t_range": np.array([T_MIN, T_MAX])}
    for name, (cfg, with_emb) in CASES.items():
        model = _TimeModel(with_emb, torch.Generator().manual_seed(7))
        fn = ref._make_loss_fn(cfg, cw, model, T_MIN, T_MAX)
        lg = logits.clone().requires_grad_(True)
        loss = fn(lg, y, t_idx)
        loss.backward()
        out[f"{name}/loss"] = np.array(loss.item(), dtype=np.float64)
        out[f"{name}/dlogits"] = lg.grad.numpy()
        if with_emb:
            out[f"{name}/demb"] = model.time_emb.weight.grad.numpy()
            out[f"{name}/emb"] = model.time_emb.weight.detach().numpy()
    dst = os.path.join(HERE, "loss_golden.npz")
    np.savez(dst, **out)
    print(f"wrote {dst}: {len(CASES)} cases")


if __name__ == "__main__":
    main(*sys.argv[1:])
