"""Diagnostic: the bf16-storage SAGE train step's logits / gradient relL2 vs the float64 reference
with the kernels' rounding points (tests/test_gpu_bf16.py helpers) at growing graph sizes."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
from test_gpu_bf16 import _ref_sage_bf16, _ref_sage_bf16_grads  # noqa: E402

from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic  # noqa: E402
from elliptic_gnn_project_amd.gnn import SAGENet  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double().to(a.device)
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


dev = torch.device("cuda:0")
for nn, ne in [(6000, 9000), (200_000, 400_000), (2_000_000, 4_000_000)]:
    t0 = time.time()
    data = prepare_inputs(synthetic_elliptic(num_nodes=nn, num_edges=ne, seed=42),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    N = data.x.size(0)
    ei = data.edge_index.to(dev)
    torch.manual_seed(3)
    model = SAGENet(data.x.size(1), 128, layers=3, dropout=0.0).to(dev).train()
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    x_bf = data.x.to(torch.bfloat16).to(dev)
    logits = model(x_bf, ei)
    w = torch.randn(N, 2, generator=torch.Generator().manual_seed(1)).to(dev)
    st = [t.detach().clone() for t in logits.grad_fn.saved_tensors[:5]]  # hs (L), aggs (L - 1): the kernels' own
    (logits * w).sum().backward()
    own = [(st[3 + l].double() if l < 2 else None, st[l].double()) for l in range(3)]
    with torch.no_grad():
        ref, saved = _ref_sage_bf16(params, x_bf, ei, N, 3)
        le = rel(logits, ref)
        fd = {f"h{l}": rel(st[l], saved[l][1]) for l in range(3)}
        fd.update({f"agg{l}": rel(st[3 + l], saved[l][0]) for l in range(2)})
        grads = _ref_sage_bf16_grads(params, saved, w, ei, N, 3)
        grads_own = _ref_sage_bf16_grads(params, own, w, ei, N, 3)
    errs = {k: f"{rel(v.grad, grads[k]):.2e}/{rel(v.grad, grads_own[k]):.2e}" for k, v in model.named_parameters()}
    print("forward stores relL2", {k: f"{v:.2e}" for k, v in fd.items()})
    deg = torch.bincount(ei[1], minlength=N)
    print(f"N={N} E={ei.size(1)} maxdeg={int(deg.max())} logits {le:.2e} grads {errs} ({time.time() - t0:.0f}s)",
          flush=True)
    del data, ei, model, params, x_bf, logits, ref, saved, grads, grads_own, own, st, w
    torch.cuda.empty_cache()
