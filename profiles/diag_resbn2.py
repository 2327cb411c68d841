"""Diagnostic: the x-only half-pair NT calls of the registered SAGE-ResBN step, each output vs
float64 per row (outlier rows / tiles)."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_fullsize as T
from elliptic_gnn_project_amd import linear as LIN
from elliptic_gnn_project_amd.planes import register_input
from elliptic_gnn_project_amd.train_gnn import build_model

calls = []
orig = LIN.gemm_nt_input


def rec(x, n, **kw):
    out = orig(x, n, **kw)
    calls.append((x, kw.get("w1"), kw.get("bias"), out))
    return out


LIN.gemm_nt_input = rec
dev = torch.device("cuda")
data = T._resbn_data()
torch.manual_seed(4)
model = build_model("sage_resbn", data.x.size(1), T.RESBN).to(dev)
model.train()
xd = register_input(data.x.to(dev))
torch.manual_seed(11)
logits = model(xd, data.edge_index.to(dev), data.timestep.to(dev))
torch.cuda.synchronize()
for x, w, b, out in calls:
    ref = x.double() @ w.double().t() + (b.double() if b is not None else 0)
    d = (out.double() - ref).abs()
    rowerr = d.max(dim=1).values / ref.abs().max(dim=1).values.clamp_min(1e-30)
    top = torch.topk(rowerr, 5)
    print("call N", out.size(1), "relL2", float((out.double() - ref).norm() / ref.norm()), "max abs", float(d.max()))
    print("   worst rows", top.indices.tolist(), [f"{v:.2e}" for v in top.values.tolist()])
    bad = (rowerr > 1e-5).nonzero().flatten()
    print("   rows with row-relative err > 1e-5:", bad.numel(), bad[:20].tolist())
