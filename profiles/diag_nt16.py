"""Diagnostic: the half-pair NT (16-row ring form) vs the split-bf16 image NT vs float64 on the
SAGE-ResBN layer-0 operand (K13's [x | sin(t)], registered) at full size."""
import sys
import torch
sys.path.insert(0, ".")
from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
from elliptic_gnn_project_amd.fused import gemm_nt
from elliptic_gnn_project_amd.planes import HalfPairImage, register_input, x_only_image, h2_exp
from elliptic_gnn_project_amd import fused

dev = torch.device("cuda")
data = prepare_inputs(synthetic_elliptic(num_nodes=203_769, num_edges=234_355, seed=42),
                      dict(use_time_scalar=False, symmetrize_edges=True, train_window_k=8))
x = data.x.to(dev)
t = data.timestep.to(dev)
xt = fused.time_inject_sin(x, t, 2, 49)
register_input(xt)
print("x_tinj", tuple(xt.shape), "amax", float(xt.abs().max()), "h2_exp", h2_exp(xt))
torch.manual_seed(4)
for n in (128, 64):
    w = (torch.rand(n, xt.size(1), device=dev) - 0.5) * 2 / xt.size(1) ** 0.5
    ref = xt.double() @ w.double().t()
    imh = x_only_image(xt, HalfPairImage)
    ims = x_only_image(xt)
    yh = gemm_nt(None, None, n, planes=imh, w1=w)
    ys = gemm_nt(None, None, n, planes=ims, w1=w)
    for name, y in (("half-pair ring", yh), ("split-bf16", ys)):
        d = (y.double() - ref)
        rel = float(d.norm() / ref.norm())
        col = (d.norm(dim=0) / ref.norm(dim=0)).max().item()
        print(f"N={n} {name:15s} relL2 {rel:.3e}  worst column relL2 {col:.3e}  max abs {float(d.abs().max()):.3e}")
