"""Golden vectors from the REFERENCE's own model composition (build container only).

Imports /root/reference/src/models/gnn.py unmodified — GCNNet, SAGENet, GATNet, SAGEResBNNet
(src/models/gnn.py:14-194) — with ``torch_geometric.nn`` (not installed here) provided by the
oracle's restatement of PyG 2.5.3's SAGEConv / GCNConv / GATConv (oracle/pyg_ref.py), then runs
each model on a small seeded Elliptic-shaped graph: train-mode logits (BatchNorm on batch
statistics, dropout 0 — torch's dropout stream cannot be reproduced on the GPU), the loss of
src/train_gnn.py:159-175 and every parameter gradient, the BatchNorm running statistics after
that step, and eval-mode logits.  Writes tests/golden/reference_models.npz.

What this pins: the composition layer (time embedding, BN order, residual projections, ELU /
ReLU placement, head concat/mean, the final layer) is the reference's own code, not a
restatement.  What it does not pin: PyG's conv internals, which are the oracle's restatement
here too (PyG is not importable).

    python tests/golden/make_reference_golden.py [/root/reference]
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyg_ref  # noqa: E402


class _SAGEConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.lin_l = nn.Linear(in_channels, out_channels, bias=True)
        self.lin_r = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x, edge_index):
        return pyg_ref.sage_conv(x, edge_index, self.lin_l.weight, self.lin_l.bias, self.lin_r.weight)


class _GCNConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def forward(self, x, edge_index):
        return pyg_ref.gcn_conv(x, edge_index, self.lin.weight, self.bias)


class _GATConv(nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True):
        super().__init__()
        self.heads, self.chans, self.concat = heads, out_channels, concat
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.zeros(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.zeros(1, heads, out_channels))
        self.bias = nn.Parameter(torch.zeros(heads * out_channels if concat else out_channels))

    def forward(self, x, edge_index):
        return pyg_ref.gat_conv(x, edge_index, self.lin.weight, self.att_src, self.att_dst, self.bias,
                                self.heads, self.chans, self.concat)


def _install_pyg_stub():
    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    pyg_nn.SAGEConv, pyg_nn.GCNConv, pyg_nn.GATConv = _SAGEConv, _GCNConv, _GATConv
    pyg.nn = pyg_nn
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.nn"] = pyg_nn


MODELS = {
    # name: (class, kwargs, time embedding used in forward)
    "gcn": ("GCNNet", dict(hidden_dim=32, layers=2, dropout=0.0), False),
    "sage": ("SAGENet", dict(hidden_dim=32, layers=3, dropout=0.0), False),
    "gat": ("GATNet", dict(hidden_dim=32, layers=2, dropout=0.0, heads=4), False),
    "resbn_sin": ("SAGEResBNNet", dict(hidden_dim=32, layers=3, dropout=0.0, time_embed_dim=2,
                                       time_embed_type="sin", max_timestep=49), True),
    "resbn_learned": ("SAGEResBNNet", dict(hidden_dim=16, layers=3, dropout=0.0, time_embed_dim=4,
                                           time_embed_type="learned", max_timestep=49), True),
}


def main(ref_root: str = "/root/reference") -> None:
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    _install_pyg_stub()
    sys.path.insert(0, ref_root)
    from src.models import gnn as ref_gnn  # the reference's own composition code

    out = {}
    for name, (cls_name, kw, use_t) in MODELS.items():
        cfg = dict(symmetrize_edges=True, train_window_k=10,
                   use_time_scalar=not use_t, time_embed_dim=kw.get("time_embed_dim", 0))
        d = prepare_inputs(synthetic_elliptic(num_nodes=400, num_edges=700, seed=2024), cfg)
        torch.manual_seed(7)
        model = getattr(ref_gnn, cls_name)(d.x.size(1), **kw)
        with torch.no_grad():  # non-trivial values everywhere (zero-initialised biases, BN affine)
            for p in model.parameters():
                p.copy_(torch.randn_like(p) * (0.3 if p.dim() > 1 else 0.2))
        state0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        model.train()
        t_idx = d.timestep if use_t else None
        logits = model(d.x, d.edge_index, t_idx)
        tm = d.train_mask
        cw = pyg_ref.class_weight(d.y[tm])
        loss = pyg_ref.ce_loss(logits[tm], d.y[tm], cw)
        loss.backward()
        state1 = {k: v.detach().clone() for k, v in model.state_dict().items()}  # BN running stats moved
        model.eval()
        with torch.no_grad():
            logits_eval = model(d.x, d.edge_index, t_idx)
        pre = name + "/"
        out[pre + "x"] = d.x.numpy()
        out[pre + "edge_index"] = d.edge_index.numpy()
        out[pre + "y"] = d.y.numpy()
        out[pre + "train_mask"] = d.train_mask.numpy()
        out[pre + "timestep"] = d.timestep.numpy()
        out[pre + "cw"] = cw.numpy()
        out[pre + "loss"] = np.array(float(loss))
        out[pre + "logits_train"] = logits.detach().numpy()
        out[pre + "logits_eval"] = logits_eval.numpy()
        for k, v in state0.items():
            out[pre + "state0/" + k] = v.numpy()
        for k, v in state1.items():
            if "running" in k or "num_batches" in k:
                out[pre + "state1/" + k] = v.numpy()
        for k, p in model.named_parameters():
            out[pre + "grad/" + k] = p.grad.numpy()
        print(f"{name}: {cls_name} loss {float(loss):.6f} params {len(state0)}")
    np.savez_compressed(os.path.join(HERE, "reference_models.npz"), **out)
    print("wrote", os.path.join(HERE, "reference_models.npz"))


if __name__ == "__main__":
    main(*sys.argv[1:])
