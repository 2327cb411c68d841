"""Kernel lab: degree-ordered split main pass (K0b order) vs plan order, for the F = 64 lane-group
gathers (not part of the product).  Two plans of the same edge_index — GNNMP_ORDER=1 / 0 at
build — times each F = 64 case on both, with the rows-per-group lab variants (gnnx_set_agg_variant
0 / 5 / 6 / 8 = 2 / 4 / 8 / lps-1 rows), interleaved over rounds (median); every output is checked
bitwise against the plan-order default (the order changes which group sums a row, not the sum).

    python profiles/lab_order.py [--rounds 20] [--variants 0,5,6]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from elliptic_gnn_project_amd import _lib  # noqa: E402
from elliptic_gnn_project_amd.aggregation import agg_bytes, aggregate  # noqa: E402
from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic  # noqa: E402
from elliptic_gnn_project_amd.graph import get_plan  # noqa: E402


def plans(ei, n, loops, dev):
    out = {}
    for o in ("0", "1"):
        os.environ["GNNMP_ORDER"] = o
        out[o] = get_plan(ei.clone().to(dev), n, loops)
    os.environ["GNNMP_ORDER"] = "1"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--variants", default="0,5,6")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    from agglab import route_to_agglab  # the lab build of aggregate.hip (make lab)
    setv = route_to_agglab()
    dev = torch.device("cuda:0")
    sage = prepare_inputs(synthetic_elliptic(seed=42), dict(use_time_scalar=True, symmetrize_edges=True))
    ps = plans(sage.edge_index, sage.x.size(0), _lib.LOOPS_KEEP, dev)
    gcn = prepare_inputs(synthetic_elliptic(seed=42), dict(use_time_scalar=True, symmetrize_edges=False))
    pg = plans(gcn.edge_index, gcn.x.size(0), _lib.LOOPS_REPLACE, dev)
    N = sage.x.size(0)
    h64 = torch.randn((N, 64), device=dev)
    b = torch.randn(64, device=dev)
    cases = [
        ("sage64 mean fwd F=64", ps, h64, lambda p: dict(mode=_lib.AGG_MEAN, nodew=p.deg)),
        ("sage64 mean bwd F=64 (csc)", ps, h64, lambda p: dict(mode=_lib.AGG_MEAN_BWD, transpose=True, nodew=p.deg)),
        ("gcn fwd F=64 (+bias relu dropout)", pg, h64,
         lambda p: dict(mode=_lib.AGG_GCN, nodew=p.dinv, bias=b, relu=True, dropout_p=0.5, seed=7)),
        ("gcn bwd F=64 (csc)", pg, h64, lambda p: dict(mode=_lib.AGG_GCN, transpose=True, nodew=p.dinv)),
    ]
    for name, pl, inp, kwf in cases:
        keys = [(o, v) for o in ("0", "1") for v in variants]
        times = {k: [] for k in keys}
        outs = {}
        for r in range(args.rounds + 1):
            for o, v in keys:
                setv(v)
                plan = pl[o]
                kw = kwf(plan)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    y = aggregate(plan, inp, **kw)
                e1.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[(o, v)].append(e0.elapsed_time(e1) * 1000 / 5)
                outs[(o, v)] = y
        setv(0)
        ref = outs[("0", 0)]
        nb = agg_bytes(pl["0"], inp.size(1), kwf(pl["0"])["mode"], kwf(pl["0"]).get("transpose", False), False)
        for o, v in keys:
            t = statistics.median(times[(o, v)])
            print(f"{name:36s} order={o} v{v}: {t:7.1f} us ({nb / t / 8e6 * 100:4.1f} % HBM)"
                  f"  bitwise==plan order: {torch.equal(outs[(o, v)], ref)}", flush=True)


if __name__ == "__main__":
    main()
