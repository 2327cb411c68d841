"""Diagnostic: K1 (half-pair mean gather + the riding B prep) alone on the largest 8-way (or N-way)
shard, for the current GNNMP_K1_WAVE_ROWS / GNNMP_K1_HUB_DEG (run once per setting).
    GNNMP_K1_WAVE_ROWS=4 python profiles/diag_k1sweep.py 8"""
import os
import sys
import torch
sys.path.insert(0, ".")
import bench
from elliptic_gnn_project_amd import distributed as gdist
from elliptic_gnn_project_amd.fused import _nt_workspace, gemm_nt
from elliptic_gnn_project_amd.graph import get_plan
from elliptic_gnn_project_amd.planes import HalfPairImage, register_input, x_padded

dev = torch.device("cuda:0")
shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = bench.PRESETS["sage"]["cfg"]
full, key = bench.make_global_graph(1, "strong", "powerlaw", cfg, bench.PRESETS["sage"].get("gen"))
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
res = []
for name, kw in (("pad", dict(x_pad=xp)), ("pad+prep", dict(x_pad=xp, prep_b=prm))):
    for _ in range(5):
        im.fill_mean(plan, x, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(50):
        im.fill_mean(plan, x, **kw)
    e1.record()
    torch.cuda.synchronize()
    res.append(f"{name} {e0.elapsed_time(e1) / 50 * 1000:6.1f}")
hub = plan.hub
print(f"shards {shards} rows {os.environ.get('GNNMP_K1_WAVE_ROWS', '-')} hubdeg {os.environ.get('GNNMP_K1_HUB_DEG', '32')}: "
      f"hubs {int(hub['c'].num_long) if hub else 0} waves {int(hub['c'].num_pieces) if hub else 0} | " + " | ".join(res) + " us")
