"""Diagnostic: K1 (half-pair mean gather) on the largest 8-way shard, alone, with / without the
NT's B prep riding along, the keep bits, and the hub form — what sets its ~30 us."""
import sys
import torch
sys.path.insert(0, ".")
import bench
from elliptic_gnn_project_amd import distributed as gdist
from elliptic_gnn_project_amd.fused import _nt_workspace, gemm_nt
from elliptic_gnn_project_amd.graph import get_plan
from elliptic_gnn_project_amd.planes import HalfPairImage, register_input, x_padded

DEG = "powerlaw"
dev = torch.device("cuda:0")
cfg = bench.PRESETS["sage"]["cfg"]
for shards in (8, 1):
    full, key = bench.make_global_graph(1, "strong", DEG, cfg, bench.PRESETS["sage"].get("gen"))
    if shards > 1:
        parts = gdist.partition_timesteps(key, full.edge_index, shards)
        e_t = torch.bincount(key[full.edge_index[1]], minlength=int(key.max()) + 1)
        big = max(range(shards), key=lambda i: int(sum(int(e_t[t]) for t in parts[i])))
        data = gdist.shard_graph(full, shards, big, parts=parts, key=key).to(dev)
    else:
        data = full.to(dev)
    x = register_input(data.x)
    plan = get_plan(data.edge_index, x.size(0))
    im = HalfPairImage(x.size(0), x.size(1), x.size(1), dev)
    im.fill_x(x)
    xp = x_padded(x, im.col2)
    n = 128
    w1 = torch.randn(n, x.size(1), device=dev) * 0.08
    w2 = torch.randn(n, x.size(1), device=dev) * 0.08
    ws = _nt_workspace(dev, n, im.k1, im.k2)
    nt = dict(w1=w1, w2=w2, bias=torch.zeros(n, device=dev), relu=True, dropout_p=0.5, seed=9)
    prm = gemm_nt(None, None, n, planes=im, workspace=ws, b_stage="params", **nt)
    kb = torch.zeros(x.size(0), 4, dtype=torch.int32, device=dev)
    deg = plan.deg[: x.size(0)]
    print(f"shards {shards}: nodes {x.size(0)} slots {plan.num_slots} max deg {int(deg.max())} "
          f"hubs {int(plan.hub['c'].num_long) if plan.hub else 0} waves {int(plan.hub['c'].num_pieces) if plan.hub else 0}")
    for name, kw in (("plain", {}), ("pad", dict(x_pad=xp)), ("pad+keep", dict(x_pad=xp, keep=(kb, n, 0.5, 3, None))),
                     ("pad+keep+prep", dict(x_pad=xp, keep=(kb, n, 0.5, 3, None), prep_b=prm)),
                     ("pad+keep+prep nohub", dict(x_pad=xp, keep=(kb, n, 0.5, 3, None), prep_b=prm, hub=False))):
        for _ in range(5):
            im.fill_mean(plan, x, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(50):
            im.fill_mean(plan, x, **kw)
        e1.record()
        torch.cuda.synchronize()
        print(f"  K1 {name:22s} {e0.elapsed_time(e1) / 50 * 1000:7.1f} us/launch (back to back)")
