"""Dense transforms of the convs on the MFMA GEMM kernels (K7) instead of torch's Linear.

PyG's ``Linear`` inside SAGEConv (lin_l / lin_r, gnn.py:41-44), GCNConv (lin, gnn.py:20-23) and
GATConv (lin, gnn.py:64-67), and SAGE-ResBN's ``res_projs`` (gnn.py:118-120), are tall-skinny
fp32 GEMMs ([N≈2e5, ≤384] × [≤384, ≤128]).  Forward runs the NT kernel with the weight read in
place ([out, in] is already the K-contiguous B image), bias fused; backward runs ONE TN kernel for
dW (and db) and the NT kernel (B = W, row-major [K=out, N=in]) for the input gradient.

``linear2`` is the two-segment form ``[a1 | a2] · [W1 | W2]ᵀ + b`` — SAGEConv's
``lin_l(agg) + lin_r(x)`` as one GEMM with no concatenated copy of the operands.

Shapes past the split-bf16 kernels' envelope (out > 128 or in > 384: e.g. ``hidden_dim: 256``,
which build_model accepts, src/train_gnn.py:67-104) stay on the hand-written kernels too
(``_TiledLinear``): the forward as split-bf16 NT calls over ≤ 128-column blocks of the output,
the input gradient on the exact-f32 MFMA NT (B as the [K, N] row-major weight, any N and K — as
_MfmaLinear's), the weight gradient as TN calls over ≤ 128-row blocks of dW and ≤ 384-column
blocks of the input — never torch's hipBLASLt.  (The forward keeps the split-bf16 form's accuracy:
the exact-f32 MFMA's k-ordered f32 chain, ~1e-6 relative on K = 173, moved SAGE-ResBN's BN
outputs across ReLU ties at full size.)
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .fused import gemm_nt, gemm_nt_input, gemm_tn, gemm_tn_input

MAX_OUT = 128  # NT in-place weight form / TN dW rows
MAX_IN = 384   # TN K extent


def _rows(x: torch.Tensor) -> torch.Tensor:
    if x.stride(-1) != 1 or x.stride(0) < x.size(1):
        x = x.contiguous()
    return x


def fits(in_total: int, out: int) -> bool:
    return 1 <= out <= MAX_OUT and 1 <= in_total <= MAX_IN


class _MfmaLinear(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, a1, w1, bias, a2, w2):
        a1 = _rows(a1)
        a2 = _rows(a2) if a2 is not None else None
        w1 = w1.contiguous()
        w2 = w2.contiguous() if w2 is not None else None
        if a2 is None:  # a model input (GAT / GCN layer 1): on its cached split image
            y = gemm_nt_input(a1, w1.size(0), bias=bias, w1=w1)
        else:
            y = gemm_nt(a1, None, w1.size(0), a2=a2, bias=bias, w1=w1, w2=w2)
        ctx.save_for_backward(a1, w1, a2, w2)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        a1, w1, a2, w2 = ctx.saved_tensors
        dy = _rows(dy)  # row-strided views (K12's dz is the right half of a [N, 2C] buffer) read in place
        need = ctx.needs_input_grad
        dW1 = db = dW2 = None
        if need[1] or need[2] or need[4]:
            if a2 is None:  # a model input (GAT / GCN layer 1) on its cached split image
                (dW1, dW2), db, _, _ = gemm_tn_input(w1.size(0), a1, dy)
            else:
                (dW1, dW2), db, _, _ = gemm_tn(w1.size(0), a1, a2, g=dy)
        da1 = gemm_nt(dy, w1, w1.size(1)) if need[0] else None
        da2 = gemm_nt(dy, w2, w2.size(1)) if (a2 is not None and need[3]) else None
        return (da1, dW1 if need[1] else None, db if (ctx.has_bias and need[2]) else None,
                da2, dW2 if need[4] else None)


class _StackedLinear(torch.autograd.Function):
    """x · [W_l ; W_r]ᵀ — SAGEConv's transform-first GEMM (conv.py) — from the two weights with no
    per-step torch.cat when they are the halves of one buffer (fused.tie_output_weights): the same
    NT / TN kernels as _MfmaLinear over the stacked weight, whose TN output rows are the two
    weights' gradients (views, adopted by autograd)."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, wl, wr):
        from .fused import _tied_buffer_of

        w = _tied_buffer_of(wl, wr)
        if w is None:
            w = torch.cat([wl, wr], dim=0)
        x = _rows(x)
        y = gemm_nt_input(x, w.size(0), w1=w)
        ctx.save_for_backward(x, w)
        ctx.fo = wl.size(0)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = _rows(dy)
        need = ctx.needs_input_grad
        dWl = dWr = dx = None
        if need[1] or need[2]:
            (dW, _), _, _, _ = gemm_tn_input(w.size(0), x, dy)
            dWl, dWr = dW[:ctx.fo], dW[ctx.fo:]
        if need[0]:
            dx = gemm_nt(dy, w, w.size(1))
        return dx, dWl if need[1] else None, dWr if need[2] else None


def _tn_blocks(segs, dy: torch.Tensor, want_db: bool):
    """dW_s = dyᵀ · a_s for every segment a_s [M, k_s], and db = Σ_rows dy, as TN calls over ≤ MAX_OUT
    output rows × ≤ MAX_IN input columns (row-strided views of dy and a_s read in place)."""
    fo = dy.size(1)
    dWs = [torch.empty((fo, a.size(1)), dtype=torch.float32, device=dy.device) for a in segs]
    db = torch.empty(fo, dtype=torch.float32, device=dy.device) if want_db else None
    for r0 in range(0, fo, MAX_OUT):
        r1 = min(fo, r0 + MAX_OUT)
        g = dy[:, r0:r1]
        first = True
        for a, dW in zip(segs, dWs):
            for k0 in range(0, a.size(1), MAX_IN):
                k1 = min(a.size(1), k0 + MAX_IN)
                (d, _), dbb, _, _ = gemm_tn(r1 - r0, a[:, k0:k1], g=g)
                dW[r0:r1, k0:k1].copy_(d)
                if first and db is not None:
                    db[r0:r1].copy_(dbb)
                first = False
    return dWs, db


class _TiledLinear(torch.autograd.Function):
    """``[a1 | a2] · [W1 | W2]ᵀ + b`` for shapes outside the split-bf16 envelope (see the module
    docstring): column-blocked NT forward, exact-f32 NT input gradient, blocked TN weight gradient."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, a1, w1, bias, a2, w2):
        a1 = _rows(a1)
        a2 = _rows(a2) if a2 is not None else None
        w1 = w1.contiguous()
        w2 = w2.contiguous() if w2 is not None else None
        fo = w1.size(0)
        y = torch.empty((a1.size(0), fo), dtype=torch.float32, device=a1.device)
        for c0 in range(0, fo, MAX_OUT):  # ≤ 128 output columns per split-bf16 NT (rows of W: contiguous)
            c1 = min(fo, c0 + MAX_OUT)
            gemm_nt(a1, None, c1 - c0, a2=a2, w1=w1[c0:c1], w2=w2[c0:c1] if w2 is not None else None,
                    bias=bias[c0:c1] if bias is not None else None, out=y[:, c0:c1])
        w = w1 if a2 is None else torch.cat([w1, w2], dim=1)
        ctx.save_for_backward(a1, a2, w)
        ctx.has_bias = bias is not None
        ctx.k1 = w1.size(1)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        a1, a2, w = ctx.saved_tensors
        dy = _rows(dy)
        need = ctx.needs_input_grad
        segs = [a1] if a2 is None else [a1, a2]
        dWs, db = [None, None], None
        if need[1] or need[2] or need[4]:
            got, db = _tn_blocks(segs, dy, ctx.has_bias and need[2])
            dWs[: len(got)] = got
        da1 = da2 = None
        if need[0] or need[3]:
            dA = gemm_nt(dy, w, w.size(1), math="f32")  # [M, k1 + k2]
            da1 = dA[:, : ctx.k1] if need[0] else None
            da2 = dA[:, ctx.k1:] if (a2 is not None and need[3]) else None
        return (da1, dWs[0] if need[1] else None, db if (ctx.has_bias and need[2]) else None,
                da2, dWs[1] if need[4] else None)


def linear_stacked(x: torch.Tensor, wl: torch.Tensor, wr: torch.Tensor) -> torch.Tensor:
    """``x · [wl ; wr]ᵀ`` (= F.linear(x, torch.cat([wl, wr]))) on the MFMA kernels."""
    if not x.is_cuda:
        raise RuntimeError("elliptic_gnn_project_amd.linear_stacked runs on the HIP device only")
    if x.dim() != 2 or wl.shape != wr.shape:
        raise ValueError(f"linear_stacked needs a 2-D input and equal weights, got {tuple(x.shape)}, "
                         f"{tuple(wl.shape)}, {tuple(wr.shape)}")
    if x.size(0) == 0 or not fits(wl.size(1), 2 * wl.size(0)):
        return _TiledLinear.apply(x, torch.cat([wl, wr], dim=0), None, None, None)
    return _StackedLinear.apply(x, wl, wr)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear`` on the MFMA kernels (HIP device, fp32 compute, 2-D input)."""
    if not x.is_cuda:
        raise RuntimeError("elliptic_gnn_project_amd.linear runs on the HIP device only")
    if x.dim() != 2:
        raise ValueError(f"linear needs a 2-D input [N, in], got {tuple(x.shape)}")
    if x.size(0) == 0 or not fits(weight.size(1), weight.size(0)):
        return _TiledLinear.apply(x, weight, bias, None, None)  # outside the split-bf16 envelope
    return _MfmaLinear.apply(x, weight, bias, None, None)


def linear2(a1: torch.Tensor, a2: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor,
            bias: torch.Tensor | None = None) -> torch.Tensor:
    """``a1·W1ᵀ + a2·W2ᵀ + b`` as one GEMM over the two K segments."""
    if not a1.is_cuda:
        raise RuntimeError("elliptic_gnn_project_amd.linear2 runs on the HIP device only")
    if a1.size(0) == 0 or not fits(w1.size(1) + w2.size(1), w1.size(0)):
        return _TiledLinear.apply(a1, w1, bias, a2, w2)
    return _MfmaLinear.apply(a1, w1, bias, a2, w2)


class Linear(nn.Linear):
    """``torch.nn.Linear`` (same parameters, init and state_dict keys) whose forward runs on
    the MFMA kernels."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)
