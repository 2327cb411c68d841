"""Autograd ops over libgnnmp's aggregation kernels (no torch fallback).

Each op mirrors one PyG 2.5.3 propagate pattern used by src/models/gnn.py:
  mean_aggregate  — SAGEConv aggr='mean'   (gnn.py:41-44 construct, :49,52,187,193 call)
  gcn_aggregate   — GCNConv norm + 'add'   (gnn.py:20-23, :28,31)
  gat_attention   — GATConv softmax + 'add' (gnn.py:64-67, :72,75)
Forward and backward both run as atomic-free segmented reductions (CSR rows for
forward, CSC columns for the transposed backward), so results are bitwise
reproducible run to run.
"""
from __future__ import annotations

import os

import torch

from . import _lib
from .graph import GraphPlan, get_plan

__all__ = ["mean_aggregate", "masked_mean_aggregate", "masked_gcn_aggregate", "edge_dot", "gcn_aggregate", "gat_attention", "gat_attention_proj", "aggregate", "colsum", "KernelTimer"]


class KernelTimer:
    """Optional HIP-event bracketing of individual libgnnmp launches (bench.py roofline).

    When ``KernelTimer.active`` is set, each aggregation launch records a pair of
    torch.cuda.Events on the stream it launches on (torch's current stream), tagged
    ("agg", mode, transpose, F) with its algorithmic bytes, or ("gemm_nt"/"gemm_tn", M, K, N)
    with its FLOPs.  Off by default: zero overhead on the normal path.
    """

    active = False
    records: list = []

    @classmethod
    def start(cls):
        cls.records = []
        cls.active = True

    @classmethod
    def begin(cls):
        """Event before a launch (None when inactive); pair with ``end``."""
        if not cls.active:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    @classmethod
    def end(cls, e0, tag, amount):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        cls.records.append((tag, e0, e1, int(amount)))

    @classmethod
    def stop(cls):
        cls.active = False
        torch.cuda.synchronize()
        out = {}
        for tag, a, b, amount in cls.records:
            ms = a.elapsed_time(b)
            d = out.setdefault(tag, {"launches": 0, "ms": 0.0, "amount": 0})
            d["launches"] += 1
            d["ms"] += ms
            d["amount"] += amount
        cls.records = []
        return out

_custom_fwd = torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
_custom_bwd = torch.amp.custom_bwd(device_type="cuda")


def _as_f32_rows(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != torch.float32:
        raise TypeError(f"libgnnmp fp32 path got {x.dtype}")
    if x.dim() != 2:
        raise ValueError(f"expected [N, F] features, got {tuple(x.shape)}")
    if x.stride(1) != 1 or x.stride(0) < x.size(1):
        x = x.contiguous()
    return x


def _ld(x: torch.Tensor) -> int:
    return max(int(x.stride(0)), int(x.size(1)), 1)


SPLIT_MAX_F = 128  # widest rows the long-segment split runs for (the lane-group gather)


def aggregate(plan: GraphPlan, x: torch.Tensor, mode: int, transpose: bool = False,
              nodew: torch.Tensor | None = None, ew: torch.Tensor | None = None, heads: int = 1,
              addend: torch.Tensor | None = None, bias: torch.Tensor | None = None,
              relu: bool = False, out: torch.Tensor | None = None, dropout_p: float = 0.0, seed: int = 0,
              seed_ptr: torch.Tensor | None = None, addend2: torch.Tensor | None = None) -> torch.Tensor:
    """Raw call of gnn_aggregate_f32 (no autograd); bf16 rows go to gnn_aggregate_bf16 (bf16 out).
    ``dropout_p`` > 0: counter-hash dropout of element r·F + f after bias / ReLU (fp32 path).
    ``addend2``: a second [N, F] term summed after ``addend`` (fp32 path, ABI 20)."""
    if x.dtype == torch.bfloat16:
        if dropout_p > 0 or addend2 is not None:
            raise NotImplementedError("dropout / addend2 epilogue on the bf16-storage aggregation")
        return _aggregate_bf16(plan, x, mode, transpose, nodew, addend, bias, relu, out)
    x = _as_f32_rows(x)
    N, F = plan.num_nodes, x.size(1)
    if x.size(0) != N:
        raise ValueError(f"feature rows {x.size(0)} != plan nodes {N}")
    if out is None:
        out = torch.empty((N, F), dtype=torch.float32, device=x.device)
    if addend is not None:
        addend = _as_f32_rows(addend)
    if addend2 is not None:
        addend2 = _as_f32_rows(addend2)
    # partial-sum rows for the long-segment split (used by the lane-group gather, 8 < F <= 128;
    # the narrow F <= 4 kernels measured no faster with it on the bench graph)
    npieces = plan.split_pieces(transpose) if (mode != _lib.AGG_EDGE_W and 8 < F <= SPLIT_MAX_F) else 0
    part = torch.empty(npieces * F, dtype=torch.float32, device=x.device) if npieces else None
    p = _lib.GnnAggParams(
        mode, int(transpose), _lib.ptr(nodew), _lib.ptr(ew), int(heads),
        _lib.ptr(addend), _ld(addend) if addend is not None else 0,
        _lib.ptr(bias), int(relu), _lib.ptr(part), part.numel() * 4 if part is not None else 0,
        float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ptr),
        _lib.ptr(addend2), _ld(addend2) if addend2 is not None else 0,
    )
    if KernelTimer.active:
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
    _lib.call("gnn_aggregate_f32", plan.c_graph, p, x.data_ptr(), _ld(x), F, out.data_ptr(), _ld(out),
              _lib.stream_handle(x.device))
    if KernelTimer.active:
        b.record()
        KernelTimer.records.append((("agg", int(mode), bool(transpose), int(F)), a, b,
                                    agg_bytes(plan, F, mode, transpose, int(addend is not None) + int(addend2 is not None))))
    return out


def _aggregate_bf16(plan, x, mode, transpose, nodew, addend, bias, relu, out):
    if x.dim() != 2 or x.stride(1) != 1:
        x = x.contiguous()
    N, F = plan.num_nodes, x.size(1)
    if x.size(0) != N:
        raise ValueError(f"feature rows {x.size(0)} != plan nodes {N}")
    if out is None:
        out = torch.empty((N, F), dtype=torch.bfloat16, device=x.device)
    if out.dtype != torch.bfloat16:
        raise TypeError("bf16 aggregation writes bf16")
    if addend is not None:
        addend = _as_f32_rows(addend)
    p = _lib.GnnAggParams(
        mode, int(transpose), _lib.ptr(nodew), None, 1,
        _lib.ptr(addend), _ld(addend) if addend is not None else 0,
        _lib.ptr(bias), int(relu), None, 0,
    )
    if KernelTimer.active:
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
    _lib.call("gnn_aggregate_bf16", plan.c_graph, p, x.data_ptr(), _ld(x), F, out.data_ptr(), _ld(out),
              _lib.stream_handle(x.device))
    if KernelTimer.active:
        b.record()
        KernelTimer.records.append((("agg_bf16", int(mode), bool(transpose), int(F)), a, b,
                                    agg_bytes(plan, F, mode, transpose, addend is not None, elem=2)))
    return out


def agg_bytes(plan: GraphPlan, F: int, mode: int, transpose: bool, has_addend, elem: int = 4) -> int:
    """Algorithmic HBM bytes of one aggregation launch (fp32, int32 plan).

    rowptr/colptr 4(N+1) + neighbour ids 4S + one F-row gather per slot 4·S·F + output
    4·N·F, plus the per-node weights read (4N; per slot for MEAN_BWD/GCN) and the fused
    root addend 4·N·F when present.  (SURVEY §8d per-edge model.)
    """
    N, S = plan.num_nodes, plan.num_slots
    b = 4 * (N + 1) + 4 * S + elem * S * F + elem * N * F
    if mode in (_lib.AGG_MEAN,):
        b += 4 * N
    elif mode in (_lib.AGG_MEAN_BWD, _lib.AGG_GCN):
        b += 4 * S
    b += 4 * N * F * int(has_addend)  # (the number of fused [N, F] addends: 0, 1 or 2)
    return b


def colsum_of(x: torch.Tensor) -> torch.Tensor:
    """colsum(x), taken from the per-block column sums the kernel that wrote x left on it
    (``x._gnnmp_colsum``: the masked CE's dlogits, gnn_masked_ce_colsum_f32) when it has them —
    one small launch instead of a pass over x."""
    part = getattr(x, "_gnnmp_colsum", None)
    if part is not None and x.dim() == 2 and x.size(1) > 0 and part.numel() % x.size(1) == 0 and part.numel() > 0:
        out = torch.empty(x.size(1), dtype=torch.float32, device=x.device)
        _lib.call("gnn_colsum_finish_f32", part.data_ptr(), part.numel() // x.size(1), x.size(1), out.data_ptr(),
                  _lib.stream_handle(x.device))
        return out
    return colsum(x)


def colsum(x: torch.Tensor) -> torch.Tensor:
    """Deterministic column sum (bias gradients) via gnn_colsum_f32."""
    x = _as_f32_rows(x)
    rows, F = x.shape
    out = torch.empty(F, dtype=torch.float32, device=x.device)
    nb = _lib.c_size(0)
    _lib.call("gnn_colsum_workspace_size", rows, F, nb)
    ws = torch.empty(max(int(nb.value) // 4, 1), dtype=torch.float32, device=x.device)
    _lib.call("gnn_colsum_f32", rows, F, x.data_ptr(), _ld(x), out.data_ptr(), ws.data_ptr(),
              ws.numel() * 4, _lib.stream_handle(x.device))
    return out


# --------------------------------------------------------------------------- SAGE mean
class _MeanAggregate(torch.autograd.Function):
    @staticmethod
    @_custom_fwd
    def forward(ctx, x, plan: GraphPlan):
        ctx.plan = plan
        return aggregate(plan, x, _lib.AGG_MEAN, nodew=plan.deg)

    @staticmethod
    @_custom_bwd
    def backward(ctx, dy):
        plan = ctx.plan
        dx = None
        if ctx.needs_input_grad[0]:
            dx = aggregate(plan, dy, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg)
        return dx, None


def mean_aggregate(x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    """PyG ``scatter(x[ei[0]], ei[1], reduce='mean')`` over x's N rows."""
    plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
    return _MeanAggregate.apply(x, plan)


# --------------------------------------------------------------------------- explain mode
def edge_dot(plan: GraphPlan, a: torch.Tensor, b: torch.Tensor, nodew: torch.Tensor | None = None) -> torch.Tensor:
    """Per-edge <a[i], b[j]> / max(nodew[i], 1) in PyG edge order [E] (+N loops on REPLACE plans)."""
    a, b = _as_f32_rows(a), _as_f32_rows(b)
    N, F = plan.num_nodes, a.size(1)
    if a.size(0) != N or b.size(0) != N or b.size(1) != F:
        raise ValueError(f"edge_dot operands {tuple(a.shape)} / {tuple(b.shape)} vs plan nodes {N}")
    # REPLACE plans: appended loop of node i has id E + i, dropped input loops stay 0
    n_out = plan.num_edges + (N if plan.loops == _lib.LOOPS_REPLACE else 0)
    out = torch.zeros(n_out, dtype=torch.float32, device=a.device)
    _lib.call("gnn_edge_dot_f32", plan.c_graph, plan.csr_eid.data_ptr(), _lib.ptr(nodew), a.data_ptr(), _ld(a),
              b.data_ptr(), _ld(b), F, out.data_ptr(), _lib.stream_handle(a.device))
    return out


class _MaskedMeanAggregate(torch.autograd.Function):
    """PyG explain-mode SAGE mean: out_i = (sum_e m_e x_j) / max(deg_i, 1).

    PyG 2.5.3 MessagePassing.propagate multiplies each message by the (sigmoided) edge mask
    before ``aggr='mean'`` (the count stays the plain in-degree).  Forward and dx run the
    EDGE_W aggregation with m in CSR slot order; dm is gnn_edge_dot_f32 (SDDMM).
    """

    @staticmethod
    @_custom_fwd
    def forward(ctx, x, m, plan: GraphPlan):
        S = plan.num_slots
        ew = m.detach().float()[plan.csr_eid[:S].long()].contiguous()
        deg = plan.deg[: plan.num_nodes].clamp_min(1.0).unsqueeze(1)
        out = aggregate(plan, x, _lib.AGG_EDGE_W, ew=ew).div_(deg)
        ctx.plan = plan
        ctx.save_for_backward(x, ew)
        return out

    @staticmethod
    @_custom_bwd
    def backward(ctx, dout):
        plan = ctx.plan
        x, ew = ctx.saved_tensors
        dy = _as_f32_rows(dout) / plan.deg[: plan.num_nodes].clamp_min(1.0).unsqueeze(1)
        dx = aggregate(plan, dy, _lib.AGG_EDGE_W, transpose=True, ew=ew) if ctx.needs_input_grad[0] else None
        dm = edge_dot(plan, dy, x) if ctx.needs_input_grad[1] else None
        return dx, dm, None


def masked_mean_aggregate(x: torch.Tensor, edge_index: torch.Tensor, edge_mask: torch.Tensor) -> torch.Tensor:
    """Explain-mode ``scatter(x[ei[0]] * edge_mask[:, None], ei[1], reduce='mean')``."""
    if edge_mask.dim() != 1 or edge_mask.numel() != edge_index.size(1):
        raise ValueError(f"edge_mask must be [E={edge_index.size(1)}], got {tuple(edge_mask.shape)}")
    plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
    return _MaskedMeanAggregate.apply(x, edge_mask, plan)


class _MaskedGCNAggregate(torch.autograd.Function):
    """PyG explain-mode GCNConv propagate: message (dinv_j dinv_i) y_j times the edge mask, where
    PyG keeps the mask of non-loop edges (``edge_mask[_loop_mask]``) and gives the N appended
    self loops mask 1.  Runs EDGE_W with w_slot = m_ext[eid] * dinv_j * dinv_i; dm by K10."""

    @staticmethod
    @_custom_fwd
    def forward(ctx, y, m, plan: GraphPlan, bias):
        S, N = plan.num_slots, plan.num_nodes
        eid = plan.csr_eid[:S].long()
        seg = torch.repeat_interleave(torch.arange(N, device=y.device), plan.rowptr.diff().long(), output_size=S)
        dinv = plan.dinv
        norm = dinv[plan.col[:S].long()] * dinv[seg]
        m_ext = torch.cat([m.detach().float(), torch.ones(N, dtype=torch.float32, device=y.device)])
        ew = (m_ext[eid] * norm).contiguous()
        norm_e = torch.zeros(plan.num_edges + N, dtype=torch.float32, device=y.device)
        norm_e[eid] = norm
        ctx.plan = plan
        ctx.has_bias = bias is not None
        ctx.save_for_backward(y, ew, norm_e)
        return aggregate(plan, y, _lib.AGG_EDGE_W, ew=ew, bias=bias)

    @staticmethod
    @_custom_bwd
    def backward(ctx, dout):
        plan = ctx.plan
        y, ew, norm_e = ctx.saved_tensors
        dout = _as_f32_rows(dout)
        dy = aggregate(plan, dout, _lib.AGG_EDGE_W, transpose=True, ew=ew) if ctx.needs_input_grad[0] else None
        dm = None
        if ctx.needs_input_grad[1]:
            dm = (edge_dot(plan, dout, y) * norm_e)[: plan.num_edges]
        db = colsum_of(dout) if ctx.has_bias and ctx.needs_input_grad[3] else None
        return dy, dm, None, db


def masked_gcn_aggregate(y: torch.Tensor, edge_index: torch.Tensor, edge_mask: torch.Tensor,
                         bias: torch.Tensor | None = None) -> torch.Tensor:
    """Explain-mode GCNConv propagate of transformed features y (+ bias)."""
    if edge_mask.dim() != 1 or edge_mask.numel() != edge_index.size(1):
        raise ValueError(f"edge_mask must be [E={edge_index.size(1)}], got {tuple(edge_mask.shape)}")
    plan = get_plan(edge_index, y.size(0), _lib.LOOPS_REPLACE)
    return _MaskedGCNAggregate.apply(y, edge_mask, plan, bias)


# --------------------------------------------------------------------------- GCN
class _GCNAggregate(torch.autograd.Function):
    @staticmethod
    @_custom_fwd
    def forward(ctx, y, plan: GraphPlan, bias):
        ctx.plan = plan
        ctx.has_bias = bias is not None
        return aggregate(plan, y, _lib.AGG_GCN, nodew=plan.dinv, bias=bias)

    @staticmethod
    @_custom_bwd
    def backward(ctx, dout):
        plan = ctx.plan
        dy = aggregate(plan, dout, _lib.AGG_GCN, transpose=True, nodew=plan.dinv) \
            if ctx.needs_input_grad[0] else None
        db = colsum_of(dout) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dy, None, db


def gcn_aggregate(y: torch.Tensor, edge_index: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """PyG GCNConv propagate (gcn_norm with self loops, 'add') of transformed features y, + bias."""
    plan = get_plan(edge_index, y.size(0), _lib.LOOPS_REPLACE)
    return _GCNAggregate.apply(y, plan, bias)


# --------------------------------------------------------------------------- GAT
# GATNet's output conv (heads 1, C <= 2) in the narrow slot-parallel form with the fused CE
# (gnn_gat_out_ce_f32, round 6); GNNMP_GAT_NARROW=0: the lane-group kernel (A/B)
_GAT_NARROW = os.environ.get("GNNMP_GAT_NARROW", "1") != "0"
# GATNet: the hidden attention backward also writes max |dxh| per 16-row group for the lin's TN
# (ABI 25); GNNMP_GAT_ROWMAX=0: the TN scans dxh itself (A/B)
_GAT_ROWMAX = os.environ.get("GNNMP_GAT_ROWMAX", "1") != "0"


def tag_rowmax(g: torch.Tensor, rowmax: torch.Tensor) -> None:
    """Record on g the per-16-row maxima of |g| its producer wrote (gnn_gemm_tn_params.g_rowmax),
    keyed on g's storage and version: any in-place edit of g voids them (rowmax_of)."""
    g._gnnmp_rowmax = (rowmax, g.data_ptr(), g._version, tuple(g.shape), tuple(g.stride()))


def rowmax_of(g: torch.Tensor):
    """The row-group maxima tagged on g by its producer, if still valid for g's current data."""
    t = getattr(g, "_gnnmp_rowmax", None)
    if t is None:
        return None
    rowmax, ptr, ver, shape, stride = t
    if g.data_ptr() != ptr or g._version != ver or tuple(g.shape) != shape or tuple(g.stride()) != stride:
        return None
    return rowmax


_GAT_CE = True  # the CE in the narrow form's launch under fused_ce_target (False: its own launch; A/B, tests)


class _GATAttention(torch.autograd.Function):
    """K5/K6 with the scores formed in-kernel (gnn_gat_fwd_fused_f32) and, for GATNet's hidden
    layers, ELU + counter-hash dropout on the store; the backward undoes them in one elementwise
    pass (gnn_gat_act_bwd_f32) before the softmax / aggregation backward."""

    @staticmethod
    @_custom_fwd
    def forward(ctx, xh, att_src, att_dst, bias, plan: GraphPlan, heads: int, chans: int, concat: bool,
                slope: float, act: int, dropout_p: float, seed: int, seed_ctr):
        xh = _as_f32_rows(xh)
        N = plan.num_nodes
        dev = xh.device
        att_src = att_src.contiguous().float()
        att_dst = att_dst.contiguous().float()
        stream = _lib.stream_handle(dev)
        a_src = torch.empty((N, heads), dtype=torch.float32, device=dev)
        a_dst = torch.empty((N, heads), dtype=torch.float32, device=dev)
        alpha = torch.empty((max(plan.num_slots, 1), heads), dtype=torch.float32, device=dev)
        fo = heads * chans if concat else chans
        out = torch.empty((N, fo), dtype=torch.float32, device=dev)
        b = bias.contiguous().float() if bias is not None else None
        p = _lib.GnnGatFwdParams(
            heads, chans, int(concat), float(slope), xh.data_ptr(), _ld(xh), att_src.data_ptr(), att_dst.data_ptr(),
            _lib.ptr(b), int(act), float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ctr),
            a_src.data_ptr(), a_dst.data_ptr(), alpha.data_ptr(), out.data_ptr(), _ld(out),
        )
        t0 = KernelTimer.begin()
        ce = None
        if (heads == 1 and chans <= 2 and not concat and act == _lib.ACT_NONE and dropout_p == 0.0 and N > 0
                and _GAT_NARROW):
            # GATNet's output conv: the narrow slot-parallel form, and the step's masked CE in the
            # same launch when the training forward declared it (train_ops.fused_ce_target)
            from .train_ops import ce_target, gat_out

            tgt = ce_target() if (_GAT_CE and any(ctx.needs_input_grad)) else None
            ce = gat_out(plan, p, tgt)
        else:
            _lib.call("gnn_gat_fwd_fused_f32", plan.c_graph, p, stream)
        S = plan.num_slots
        # per slot: id 4 + xh row 4HC + alpha 8H (raw score, then normalised); per node: rowptr 4,
        # own xh row 4HC, a_src + a_dst 8H, out 4·fo
        KernelTimer.end(t0, ("gat_fwd", heads, chans, fo),
                        S * (4 + 8 * heads + 4 * heads * chans) + N * (4 + 8 * heads + 4 * heads * chans + 4 * fo))
        post = act != _lib.ACT_NONE or dropout_p > 0
        ctx.save_for_backward(xh, att_src, att_dst, a_src, a_dst, alpha, seed_ctr, out if post else None)
        ctx.meta = (plan, heads, chans, bool(concat), float(slope), bias is not None, int(act), float(dropout_p),
                    int(seed))
        if ce is not None:
            out._gnnmp_ce = ce  # masked_cross_entropy returns it (same operands) instead of launching
        return out

    @staticmethod
    @_custom_bwd
    def backward(ctx, dout):
        xh, att_src, att_dst, a_src, a_dst, alpha, seed_ctr, out = ctx.saved_tensors
        plan, heads, chans, concat, slope, has_bias, act, dropout_p, seed = ctx.meta
        dout = _as_f32_rows(dout)
        dev = xh.device
        N = plan.num_nodes
        F = heads * chans
        dxh = torch.empty((N, F), dtype=torch.float32, device=dev)
        datt_s = torch.empty(F, dtype=torch.float32, device=dev)
        datt_d = torch.empty(F, dtype=torch.float32, device=dev)
        nb = _lib.c_size(0)
        _lib.call("gnn_gat_bwd_workspace_size", N, plan.num_slots, heads, chans, nb)
        ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        t0 = KernelTimer.begin()
        if out is not None and concat:  # through dropout(act(.)): d pre formed inside the rows pass
            dpre = torch.empty_like(out)
            _lib.call("gnn_gat_bwd_act_f32", plan.c_graph, heads, chans, slope, xh.data_ptr(), _ld(xh),
                      a_src.data_ptr(), a_dst.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), alpha.data_ptr(),
                      act, dropout_p, seed & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ctr), out.data_ptr(), _ld(out),
                      dout.data_ptr(), _ld(dout), dpre.data_ptr(), _ld(dpre), dxh.data_ptr(), _ld(dxh),
                      datt_s.data_ptr(), datt_d.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
            dout = dpre
        else:
            if out is not None:  # through dropout(act(.)) first: d pre
                dpre = torch.empty_like(out)
                _lib.call("gnn_gat_act_bwd_f32", N, out.size(1), act, dropout_p, seed & 0xFFFFFFFFFFFFFFFF,
                          _lib.ptr(seed_ctr), out.data_ptr(), _ld(out), dout.data_ptr(), _ld(dout), dpre.data_ptr(),
                          _ld(dpre), _lib.stream_handle(dev))
                dout = dpre
            _lib.call("gnn_gat_bwd_f32", plan.c_graph, heads, chans, int(concat), slope, xh.data_ptr(), _ld(xh),
                      a_src.data_ptr(), a_dst.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), alpha.data_ptr(),
                      dout.data_ptr(), _ld(dout), dxh.data_ptr(), _ld(dxh), datt_s.data_ptr(), datt_d.data_ptr(),
                      ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
        S = plan.num_slots
        fo = F if concat else chans
        # rows pass (dα, de per slot): id 4 + alpha 4H + xh row 4HC + de 4H, dout row 4·fo per node;
        # cols pass (CSC): id+map 8 + alpha/de 8H + dout row 4·fo per slot, dxh 4HC + scores 8H per node
        KernelTimer.end(t0, ("gat_bwd", heads, chans, fo),
                        S * (12 + 16 * heads + 4 * heads * chans + 4 * fo) + N * (8 + 16 * heads + 4 * F + 4 * fo))
        db = colsum_of(dout) if has_bias and ctx.needs_input_grad[3] else None
        return (dxh, datt_s.view_as(att_src), datt_d.view_as(att_dst), db) + (None,) * 9


class _GATAttentionProj(torch.autograd.Function):
    """A hidden GATConv (concat, dropout(ELU(.)) on its store) whose output h feeds only a bias-free
    projection z = h · w_outᵀ — GATNet's last hidden layer and its output conv's ``lin``
    (src/models/gnn.py:72-75).  The forward writes z beside the store (gnn_gat_fwd_params.proj,
    ABI 24: the [N, 2] projection without reading h back); the backward forms dh = dz · w_out as each
    row slice loads (gnn_gat_bwd_act_proj_f32: dh is never stored) and takes dW_out = dzᵀ · h with
    the skinny TN.  Returns z; h stays internal (saved for the backward)."""

    @staticmethod
    @_custom_fwd
    def forward(ctx, xh, att_src, att_dst, bias, w_out, plan: GraphPlan, heads: int, chans: int, slope: float,
                act: int, dropout_p: float, seed: int, seed_ctr):
        xh = _as_f32_rows(xh)
        N = plan.num_nodes
        dev = xh.device
        att_src = att_src.contiguous().float()
        att_dst = att_dst.contiguous().float()
        w = w_out.contiguous().float()
        F = heads * chans
        a_src = torch.empty((N, heads), dtype=torch.float32, device=dev)
        a_dst = torch.empty((N, heads), dtype=torch.float32, device=dev)
        alpha = torch.empty((max(plan.num_slots, 1), heads), dtype=torch.float32, device=dev)
        out = torch.empty((N, F), dtype=torch.float32, device=dev)
        z = torch.empty((N, w.size(0)), dtype=torch.float32, device=dev)
        b = bias.contiguous().float() if bias is not None else None
        p = _lib.GnnGatFwdParams(
            heads, chans, 1, float(slope), xh.data_ptr(), _ld(xh), att_src.data_ptr(), att_dst.data_ptr(),
            _lib.ptr(b), int(act), float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ctr),
            a_src.data_ptr(), a_dst.data_ptr(), alpha.data_ptr(), out.data_ptr(), _ld(out), None,
            w.data_ptr(), w.size(0), z.data_ptr(), _ld(z),
        )
        t0 = KernelTimer.begin()
        _lib.call("gnn_gat_fwd_fused_f32", plan.c_graph, p, _lib.stream_handle(dev))
        S = plan.num_slots
        KernelTimer.end(t0, ("gat_fwd", heads, chans, F),
                        S * (4 + 8 * heads + 4 * F) + N * (4 + 8 * heads + 4 * F + 4 * F + 4 * w.size(0)))
        ctx.save_for_backward(xh, att_src, att_dst, a_src, a_dst, alpha, seed_ctr, out, w)
        ctx.meta = (plan, heads, chans, float(slope), bias is not None, int(act), float(dropout_p), int(seed))
        return z

    @staticmethod
    @_custom_bwd
    def backward(ctx, dz):
        from .fused import gemm_tn

        xh, att_src, att_dst, a_src, a_dst, alpha, seed_ctr, out, w = ctx.saved_tensors
        plan, heads, chans, slope, has_bias, act, dropout_p, seed = ctx.meta
        dz = _as_f32_rows(dz)
        dev = xh.device
        N = plan.num_nodes
        F = heads * chans
        need = ctx.needs_input_grad
        dW = None
        if need[4]:  # dW_out = dzᵀ · h (the skinny TN)
            (dW, _), _, _, _ = gemm_tn(w.size(0), out, g=dz)
        dxh = torch.empty((N, F), dtype=torch.float32, device=dev)
        datt_s = torch.empty(F, dtype=torch.float32, device=dev)
        datt_d = torch.empty(F, dtype=torch.float32, device=dev)
        dpre = torch.empty_like(out)
        nb = _lib.c_size(0)
        _lib.call("gnn_gat_bwd_workspace_size", N, plan.num_slots, heads, chans, nb)
        ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        # (ABI 25) max |dxh| per 16-row group, written as dxh is stored: the lin's weight-gradient TN
        # (dW = dxhᵀ · x, the g form over x's half-pair image) takes its block scales from these
        # instead of a pass over dxh (fused.gemm_tn reads the tag)
        rowmax = torch.empty(max((N + _lib.ROWMAX_ROWS - 1) // _lib.ROWMAX_ROWS, 1), dtype=torch.int32,
                             device=dev) if _GAT_ROWMAX and N > 0 else None
        t0 = KernelTimer.begin()
        _lib.call("gnn_gat_bwd_act_proj_f32", plan.c_graph, heads, chans, slope, xh.data_ptr(), _ld(xh),
                  a_src.data_ptr(), a_dst.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), alpha.data_ptr(),
                  act, dropout_p, seed & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ctr), out.data_ptr(), _ld(out),
                  dz.data_ptr(), _ld(dz), w.data_ptr(), w.size(0), dpre.data_ptr(), _ld(dpre), dxh.data_ptr(),
                  _ld(dxh), datt_s.data_ptr(), datt_d.data_ptr(), _lib.ptr(rowmax), ws.data_ptr(), ws.numel(),
                  _lib.stream_handle(dev))
        if rowmax is not None:
            tag_rowmax(dxh, rowmax)
        S = plan.num_slots
        KernelTimer.end(t0, ("gat_bwd", heads, chans, F),
                        S * (12 + 16 * heads + 4 * F + 4 * F) + N * (8 + 16 * heads + 4 * F + 4 * F))
        db = colsum(dpre) if has_bias and need[3] else None
        return (dxh, datt_s.view_as(att_src), datt_d.view_as(att_dst), db, dW) + (None,) * 8


def gat_attention_proj(xh: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor, bias: torch.Tensor | None,
                       w_out: torch.Tensor, edge_index: torch.Tensor, heads: int, chans: int,
                       negative_slope: float = 0.2, act: int = _lib.ACT_NONE, dropout_p: float = 0.0, seed: int = 0,
                       seed_ctr: torch.Tensor | None = None) -> torch.Tensor:
    """z = gat_attention(xh, ..., concat=True, act, dropout) · w_outᵀ in one launch (and its backward
    without dh): GATNet's last hidden layer feeding its output conv's ``lin`` (_GATAttentionProj)."""
    plan = get_plan(edge_index, xh.size(0), _lib.LOOPS_REPLACE)
    return _GATAttentionProj.apply(xh, att_src, att_dst, bias, w_out, plan, int(heads), int(chans),
                                   float(negative_slope), int(act), float(dropout_p), int(seed), seed_ctr)


def gat_attention(xh: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor, bias: torch.Tensor | None,
                  edge_index: torch.Tensor, heads: int, chans: int, concat: bool = True,
                  negative_slope: float = 0.2, act: int = _lib.ACT_NONE, dropout_p: float = 0.0, seed: int = 0,
                  seed_ctr: torch.Tensor | None = None) -> torch.Tensor:
    """PyG GATConv after ``lin``: scores, self-loop replacement, edge softmax, aggregation, bias;
    optionally ``dropout(act(.))`` of GATNet's hidden layers on the store (counter-hash dropout)."""
    plan = get_plan(edge_index, xh.size(0), _lib.LOOPS_REPLACE)
    return _GATAttention.apply(xh, att_src, att_dst, bias, plan, int(heads), int(chans), bool(concat),
                               float(negative_slope), int(act), float(dropout_p), int(seed), seed_ctr)


class _GATAttentionMasked(torch.autograd.Function):
    """Explain-mode GATConv propagate: every message alpha * xh[j] scaled by the per-slot mask
    value w (generic one-wave-per-row kernels; d w from gnn_gat_bwd_ew_f32)."""

    @staticmethod
    @_custom_fwd
    def forward(ctx, xh, att_src, att_dst, bias, w_slot, plan: GraphPlan, heads: int, chans: int, concat: bool,
                slope: float):
        xh = _as_f32_rows(xh)
        N = plan.num_nodes
        dev = xh.device
        att_src = att_src.contiguous().float()
        att_dst = att_dst.contiguous().float()
        w_slot = w_slot.contiguous().float()
        a_src = torch.empty((N, heads), dtype=torch.float32, device=dev)
        a_dst = torch.empty((N, heads), dtype=torch.float32, device=dev)
        alpha = torch.empty((max(plan.num_slots, 1), heads), dtype=torch.float32, device=dev)
        fo = heads * chans if concat else chans
        out = torch.empty((N, fo), dtype=torch.float32, device=dev)
        b = bias.contiguous().float() if bias is not None else None
        p = _lib.GnnGatFwdParams(
            heads, chans, int(concat), float(slope), xh.data_ptr(), _ld(xh), att_src.data_ptr(), att_dst.data_ptr(),
            _lib.ptr(b), _lib.ACT_NONE, 0.0, 0, None, a_src.data_ptr(), a_dst.data_ptr(), alpha.data_ptr(),
            out.data_ptr(), _ld(out), w_slot.data_ptr(),
        )
        _lib.call("gnn_gat_fwd_fused_f32", plan.c_graph, p, _lib.stream_handle(dev))
        ctx.save_for_backward(xh, att_src, att_dst, a_src, a_dst, alpha, w_slot)
        ctx.meta = (plan, heads, chans, bool(concat), float(slope), bias is not None)
        return out

    @staticmethod
    @_custom_bwd
    def backward(ctx, dout):
        xh, att_src, att_dst, a_src, a_dst, alpha, w_slot = ctx.saved_tensors
        plan, heads, chans, concat, slope, has_bias = ctx.meta
        dout = _as_f32_rows(dout)
        dev = xh.device
        N = plan.num_nodes
        F = heads * chans
        dxh = torch.empty((N, F), dtype=torch.float32, device=dev)
        datt_s = torch.empty(F, dtype=torch.float32, device=dev)
        datt_d = torch.empty(F, dtype=torch.float32, device=dev)
        dw = torch.empty_like(w_slot)
        nb = _lib.c_size(0)
        _lib.call("gnn_gat_bwd_workspace_size", N, plan.num_slots, heads, chans, nb)
        ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        _lib.call("gnn_gat_bwd_ew_f32", plan.c_graph, heads, chans, int(concat), slope, xh.data_ptr(), _ld(xh),
                  a_src.data_ptr(), a_dst.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), alpha.data_ptr(),
                  dout.data_ptr(), _ld(dout), dxh.data_ptr(), _ld(dxh), datt_s.data_ptr(), datt_d.data_ptr(),
                  w_slot.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
        db = colsum_of(dout) if has_bias and ctx.needs_input_grad[3] else None
        return (dxh, datt_s.view_as(att_src), datt_d.view_as(att_dst), db, dw) + (None,) * 5


def masked_gat_attention(xh: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor, bias: torch.Tensor | None,
                         edge_index: torch.Tensor, edge_mask: torch.Tensor, heads: int, chans: int,
                         concat: bool = True, negative_slope: float = 0.2) -> torch.Tensor:
    """Explain-mode GATConv after ``lin``: ``edge_mask`` [E] (already sigmoided if so configured)
    scales each input edge's message; input self loops are replaced (their mask unused) and the
    appended loops carry 1, as PyG's ``edge_mask[self._loop_mask]`` + ones."""
    if edge_mask.dim() != 1 or edge_mask.numel() != edge_index.size(1):
        raise ValueError(f"edge_mask must be [E={edge_index.size(1)}], got {tuple(edge_mask.shape)}")
    plan = get_plan(edge_index, xh.size(0), _lib.LOOPS_REPLACE)
    S = plan.num_slots
    eid = plan.csr_eid[:S].long()  # original edge id per CSR slot (appended loop of i: E + i)
    m_ext = torch.cat([edge_mask.float(), edge_mask.new_ones(plan.num_nodes, dtype=torch.float32)])
    w_slot = m_ext.index_select(0, eid)
    return _GATAttentionMasked.apply(xh, att_src, att_dst, bias, w_slot, plan, int(heads), int(chans),
                                     bool(concat), float(negative_slope))
