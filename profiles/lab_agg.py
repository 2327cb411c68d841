"""Kernel lab for the segmented aggregation (K1/K2/K4) on the bench graphs (not part of the product).

Times gnn_aggregate_f32 launch shapes selected by gnnx_set_agg_variant (a lab knob of aggregate.hip) on the SAGE-preset graph
(symmetrized, 203,769 nodes / 468,710 slots) and the GCN-preset graph (self loops replaced),
variants interleaved over rounds (median), each checked bitwise against variant 0.

    python profiles/lab_agg.py [--rounds 20] [--variants 0,1,2,3,4]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--cases", default="sage,gcn")
    ap.add_argument("--no-order", action="store_true", help="plans built with GNNMP_ORDER=0 (split tables in plan order)")
    ap.add_argument("--cold", action="store_true",
                    help="evict L2 / Infinity Cache (write 1 GB) before every timed call, time calls one at a time")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    if args.no_order:
        os.environ["GNNMP_ORDER"] = "0"
    if any(12 <= v <= 14 for v in variants):  # wave-gather split variants need the partial buffer
        import elliptic_gnn_project_amd.aggregation as agg_mod
        agg_mod.SPLIT_MAX_F = 512
    from agglab import route_to_agglab  # the lab build of aggregate.hip (make lab)
    setv = route_to_agglab()
    dev = torch.device("cuda:0")
    cases = []
    want = set(args.cases.split(","))
    sage = prepare_inputs(synthetic_elliptic(seed=42), dict(use_time_scalar=True, symmetrize_edges=True))
    ps = get_plan(sage.edge_index.to(dev), sage.x.size(0), _lib.LOOPS_KEEP)
    x = sage.x.to(dev).contiguous()
    xp = torch.zeros((x.size(0), 168), device=dev)
    xp[:, :166] = x
    cases.append(("sage mean fwd F=166", ps, x, dict(mode=_lib.AGG_MEAN, nodew=ps.deg)))
    cases.append(("sage mean fwd F=168 (padded pitch)", ps, xp, dict(mode=_lib.AGG_MEAN, nodew=ps.deg)))
    cases.append(("sage mean bwd F=166", ps, x, dict(mode=_lib.AGG_MEAN_BWD, transpose=True, nodew=ps.deg)))
    h64 = torch.randn((x.size(0), 64), device=dev)
    cases.append(("sage64 mean fwd F=64", ps, h64, dict(mode=_lib.AGG_MEAN, nodew=ps.deg)))
    cases.append(("sage64 mean bwd F=64 (csc)", ps, h64, dict(mode=_lib.AGG_MEAN_BWD, transpose=True, nodew=ps.deg)))
    z4 = torch.randn((x.size(0), 4), device=dev)
    cases.append(("narrow mean fwd F=2 (+root, bias)", ps, z4[:, :2],
                  dict(mode=_lib.AGG_MEAN, nodew=ps.deg, addend=z4[:, 2:], bias=torch.randn(2, device=dev))))
    cases.append(("narrow mean bwd F=2 (csc)", ps, torch.randn((x.size(0), 2), device=dev),
                  dict(mode=_lib.AGG_MEAN_BWD, transpose=True, nodew=ps.deg)))
    gcn = prepare_inputs(synthetic_elliptic(seed=42), dict(use_time_scalar=True, symmetrize_edges=False))
    pg = get_plan(gcn.edge_index.to(dev), gcn.x.size(0), _lib.LOOPS_REPLACE)
    y = torch.randn((gcn.x.size(0), 64), device=dev)
    b = torch.randn(64, device=dev)
    cases.append(("gcn fwd F=64 (+bias relu dropout)", pg, y,
                  dict(mode=_lib.AGG_GCN, nodew=pg.dinv, bias=b, relu=True, dropout_p=0.5, seed=7)))
    cases.append(("gcn bwd F=64 (csc)", pg, y, dict(mode=_lib.AGG_GCN, transpose=True, nodew=pg.dinv)))
    y2 = torch.randn((gcn.x.size(0), 2), device=dev)
    cases.append(("narrow gcn fwd F=2 (+bias)", pg, y2, dict(mode=_lib.AGG_GCN, nodew=pg.dinv, bias=b[:2])))
    cases = [c for c in cases if c[0].split()[0] in want]
    flush = torch.zeros(256 * 1024 * 1024, device=dev) if args.cold else None  # 1 GB
    for name, plan, inp, kw in cases:
        ref = None
        times = {v: [] for v in variants}
        outs = {}
        for r in range(args.rounds + 1):
            for v in variants:
                setv(v)
                reps = 1 if args.cold else 5
                if args.cold:
                    flush.add_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    o = aggregate(plan, inp, **kw)
                e1.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[v].append(e0.elapsed_time(e1) * 1000 / reps)
                outs[v] = o
        setv(0)
        ref = outs[variants[0]]
        nb = agg_bytes(plan, inp.size(1), kw["mode"], kw.get("transpose", False), False)
        for v in variants:
            t = statistics.median(times[v])
            same = torch.equal(outs[v], ref)
            rel = "" if same else f" (max rel diff {float(((outs[v] - ref).abs() / ref.abs().clamp_min(1e-6)).max()):.2e})"
            print(f"{name:38s} v{v}: {t:7.1f} us  {nb / t / 1e3:7.1f} GB/s  ({nb / t / 8e6 * 100:4.1f} % HBM)"
                  f"  bitwise==v{variants[0]}: {same}{rel}", flush=True)


if __name__ == "__main__":
    main()
