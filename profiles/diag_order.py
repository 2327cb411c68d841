"""Diagnostic (not part of the product): degree-ordered vs plan-order split main pass on the GCN
graph, F = 64 — max |difference| and differing rows per epilogue, to separate FMA-contraction
rounding from wrong row bookkeeping."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from elliptic_gnn_project_amd import _lib  # noqa: E402
from elliptic_gnn_project_amd.aggregation import aggregate  # noqa: E402
from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic  # noqa: E402
from elliptic_gnn_project_amd.graph import get_plan  # noqa: E402

dev = torch.device("cuda:0")
g = prepare_inputs(synthetic_elliptic(seed=42), dict(use_time_scalar=True, symmetrize_edges=False))
pl = {}
for o in ("0", "1"):
    os.environ["GNNMP_ORDER"] = o
    pl[o] = get_plan(g.edge_index.clone().to(dev), g.x.size(0), _lib.LOOPS_REPLACE)
y = torch.randn((g.x.size(0), 64), device=dev)
b = torch.randn(64, device=dev)
for name, kw in [("gcn plain", {}), ("gcn bias", dict(bias=b)), ("gcn bias relu", dict(bias=b, relu=True)),
                 ("gcn bias relu drop", dict(bias=b, relu=True, dropout_p=0.5, seed=7))]:
    outs = [aggregate(pl[o], y, mode=_lib.AGG_GCN, nodew=pl[o].dinv, **kw) for o in ("0", "1")]
    d = (outs[0] - outs[1]).abs()
    rows = (d.max(1).values > 0).nonzero().flatten()
    deg = (pl["0"].deg if hasattr(pl["0"], "deg") else None)
    print(f"{name:22s} max|d| {float(d.max()):.3e}  rel {float(d.max() / outs[0].abs().max()):.2e}  "
          f"rows differing {rows.numel()}", flush=True)
    if rows.numel():
        print("   first rows", rows[:8].tolist())
