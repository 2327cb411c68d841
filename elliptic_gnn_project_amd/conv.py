"""Drop-in replacements for ``torch_geometric.nn.{SAGEConv, GCNConv, GATConv}`` (PyG 2.5.3).

The reference imports these at src/models/gnn.py:8 and constructs them at
gnn.py:20-23 (GCN), :41-44 and :125-128 (SAGE), :64-67 (GAT).  Constructor arguments,
parameter names (hence ``state_dict`` keys, a compatibility contract with
best.ckpt consumers such as src/analysis/hub_ablation.py:88-98) and the
``forward(x, edge_index)`` signature are PyG's; the neighbour aggregation runs in
libgnnmp's HIP kernels and the dense transforms in libgnnmp's MFMA GEMMs (K7, csrc/gemm_*.hip).

Only PyG's defaults used by the reference are implemented (SAGE: aggr='mean',
normalize=False, root_weight=True, project=False; GCN: improved=False,
cached=False, add_self_loops=True, normalize=True; GAT: dropout=0, edge_dim=None,
add_self_loops=True, fill_value='mean').  Anything else raises.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .aggregation import (aggregate, colsum, colsum_of, gat_attention, gat_attention_proj, gcn_aggregate, masked_gat_attention, masked_gcn_aggregate,
                          masked_mean_aggregate, mean_aggregate)
from .graph import GraphPlan, get_plan
from .linear import Linear, linear, linear2, linear_stacked

# a transform-first output conv under the step's fused_ce_target runs its mean and the masked CE in
# one launch (gnn_sage_out_mean_ce_f32, as the fused 2-layer SAGE does); GNNMP_OUT_CE=0: A/B
_OUT_CE = os.environ.get("GNNMP_OUT_CE", "1") != "0"
# the aggregate-first SAGEConv (SAGE-ResBN's hidden layers) on the in-kernel half-pair GEMMs
# (GNN_MATH_HALF_PAIR, round 6); GNNMP_H2S=0 keeps them on split-bf16 (A/B)
_H2S = os.environ.get("GNNMP_H2S", "1") != "0"

__all__ = ["SAGEConv", "GCNConv", "GATConv"]


def _glorot_(t: torch.Tensor) -> None:
    # torch_geometric.nn.inits.glorot
    stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-stdv, stdv)


class _MeanAggRootBias(torch.autograd.Function):
    """out = mean_{j->i} y[j, :Fo] + y[i, Fo:] + b  (K1 with the root term and bias fused in its epilogue).

    ``y`` is the single GEMM output x·[W_l; W_r]ᵀ; its gradient is assembled in place
    (transposed mean into the left half, dout into the right half) — no slice copies.
    """

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, y, bias, plan: GraphPlan, fo: int):
        ctx.plan = plan
        ctx.fo = fo
        ctx.has_bias = bias is not None
        from .train_ops import ce_target, sage_out_mean_ce

        tgt = ce_target()
        if (tgt is not None and _OUT_CE and any(ctx.needs_input_grad) and fo <= 4 and y.size(0) > 0
                and y.dtype == torch.float32 and y.stride(1) == 1):
            # a network's output conv under the step's fused_ce_target (SAGE-ResBN): the mean and the
            # masked CE in one launch, dlogits' column sums beside them (the bias gradient)
            out, ce = sage_out_mean_ce(plan, y, fo, bias, tgt, colsum=True)
            out._gnnmp_ce = ce
            return out
        return aggregate(plan, y[:, :fo], _lib.AGG_MEAN, nodew=plan.deg, addend=y[:, fo:], bias=bias)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dout):
        plan, fo = ctx.plan, ctx.fo
        N = dout.size(0)
        dy = None
        # dout may already be the right half of an [N, 2·fo] buffer (the fused CE's dlogits, K12's
        # dz): then only the left half is written here, no copy
        buf = getattr(dout, "_gnnmp_dz", None)
        if (ctx.needs_input_grad[0] and buf is not None and buf.shape == (N, 2 * fo)
                and dout.stride() == (2 * fo, 1) and dout.data_ptr() == buf.data_ptr() + fo * buf.element_size()):
            dy = buf
            u = getattr(dout, "_gnnmp_u", None)
            if u is not None and u.shape == (N, fo):  # dlogits / max(deg, 1) from the fused CE: meanᵀ = CSC sum
                aggregate(plan, u, _lib.AGG_SUM, transpose=True, out=dy[:, :fo])
            else:
                aggregate(plan, dout, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, out=dy[:, :fo])
        elif ctx.needs_input_grad[0]:
            dout = dout.contiguous()
            dy = torch.empty((N, 2 * fo), dtype=torch.float32, device=dout.device)
            aggregate(plan, dout, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, out=dy[:, :fo])
            dy[:, fo:].copy_(dout)
        db = colsum_of(dout) if ctx.has_bias and ctx.needs_input_grad[1] else None
        return dy, db, None, None


class _SAGEAggregateFirst(torch.autograd.Function):
    """out = [mean_{j->i} x_j | x_i] · [W_l | W_r]ᵀ + b (PyG's order) with a one-pass backward for
    the input: [dG_l | dG_r] = dout · [W_l | W_r] as ONE split-bf16 NT GEMM (dout read once), then
    dx = meanᵀ(dG_l) + dG_r with dG_r added in the transposed aggregation's epilogue — instead of
    two NT GEMMs and an add kernel.  dW_l, dW_r, db from one TN over [agg | x] as linear2.
    ``res``: also return x itself (an alias) for an identity residual branch that consumes it
    (SAGE-ResBN's hidden layers, gnn.py:187-194); its gradient dr is then summed in the same
    transposed aggregation's store, dx = meanᵀ(dG_l) + dG_r + dr (gnn_agg_params.addend2),
    instead of autograd adding the two branches' gradients in a separate pass."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, wl, wr, bias, plan: GraphPlan, res: bool = False):
        from .fused import gemm_nt, h2s_nt_ok
        from .linear import _rows
        x = _rows(x)
        agg = aggregate(plan, x, _lib.AGG_MEAN, nodew=plan.deg)
        wl = wl.contiguous()
        wr = wr.contiguous()
        fi, fo = wl.size(1), wl.size(0)
        # the half-pair GEMMs (3 f16 products, operands split in the kernel with per-row / per-block
        # power-of-two scales: gnnmp.h GNN_MATH_HALF_PAIR) when all three shapes take them: the
        # forward NT writes the row exponents of [agg | x] that the backward's TN bounds A with
        h2 = _H2S and h2s_nt_ok(fo, fi, fi) and h2s_nt_ok(2 * fi, fo, 0) and fo % 4 == 0 and x.size(0) >= 16
        rexp = torch.empty(x.size(0), dtype=torch.int32, device=x.device) if h2 else None
        y = gemm_nt(agg, None, fo, a2=x, bias=bias, w1=wl, w2=wr, math="half_pair" if h2 else None, row_exp=rexp)
        ctx.save_for_backward(agg, x, wl, wr, rexp)
        ctx.plan = plan
        ctx.has_bias = bias is not None
        ctx.res = bool(res)
        return (y, x.view_as(x)) if res else y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy, dr=None):
        from .fused import gemm_nt, gemm_tn
        from .linear import _rows
        agg, x, wl, wr, rexp = ctx.saved_tensors
        plan = ctx.plan
        dy = _rows(dy)
        need = ctx.needs_input_grad
        dWl = dWr = db = dx = None
        gmath = "half_pair" if rexp is not None else None
        if need[1] or need[2] or need[3]:
            (dWl, dWr), db, _, _ = gemm_tn(wl.size(0), agg, x, g=dy, math=gmath, row_exp=rexp)
        if need[0]:
            fi = wl.size(1)
            wt = torch.cat([wl.t(), wr.t()], dim=0)  # [2·F_in, F_out]: Linear-weight form, one copy kernel
            d = gemm_nt(dy, None, 2 * fi, w1=wt, math=gmath)
            dx = aggregate(plan, d[:, :fi], _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, addend=d[:, fi:],
                           addend2=dr if (ctx.res and dr is not None) else None)
        return (dx, dWl if need[1] else None, dWr if need[2] else None,
                db if (ctx.has_bias and need[3]) else None, None, None)


class SAGEConv(nn.Module):
    """GraphSAGE ``out_i = W_l · mean_{j->i} x_j + b_l + W_r · x_i`` (PyG SAGEConv, aggr='mean').

    ``order`` picks where ``lin_l`` runs relative to the (linear) mean:
      'aggregate_first' — PyG's own order (aggregate width F_in);
      'transform_first' — one GEMM x·[W_l;W_r]ᵀ, then the mean over F_out columns with
                           the root term and bias fused into the aggregation epilogue;
      'auto'            — transform first when out_channels < in_channels.
    Both are the same linear map; results agree to fp32 rounding (tests: 1e-5).
    """

    def __init__(self, in_channels: int, out_channels: int, aggr: str = "mean", normalize: bool = False,
                 root_weight: bool = True, project: bool = False, bias: bool = True, order: str = "auto",
                 **kwargs):
        super().__init__()
        if aggr != "mean" or normalize or not root_weight or project or kwargs:
            raise NotImplementedError("only SAGEConv(aggr='mean', normalize=False, root_weight=True, "
                                      "project=False) — the configuration src/models/gnn.py uses")
        if order not in ("auto", "aggregate_first", "transform_first"):
            raise ValueError(f"unknown order {order!r}")
        self.in_channels = int(in_channels)
        self.out_channels = int(out_channels)
        self.aggr = aggr
        self.order = order
        self.lin_l = Linear(self.in_channels, self.out_channels, bias=bias)
        self.lin_r = Linear(self.in_channels, self.out_channels, bias=False)
        self._tie()

    def _tie(self) -> None:
        # transform first: lin_l.weight and lin_r.weight laid out as the halves of ONE [2·F_out,
        # F_in] buffer, the stacked weight of its GEMM (no per-step torch.cat; fused.tie_output_weights)
        if self._transform_first():
            from .fused import tie_output_weights

            tie_output_weights(self)

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self._tie()  # .to() / .cuda() / .float() give new tensors: lay them out again
        return out

    def reset_parameters(self) -> None:
        self.lin_l.reset_parameters()
        self.lin_r.reset_parameters()

    def _transform_first(self) -> bool:
        if self.order == "auto":
            return self.out_channels < self.in_channels
        return self.order == "transform_first"

    def _aggregate_first_ok(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dim() == 2 and x.size(0) > 0 and x.dtype != torch.bfloat16
                and 2 * self.in_channels <= 128 and self.out_channels <= 128)

    def forward_with_residual(self, x: torch.Tensor, edge_index: torch.Tensor):
        """(forward(x, edge_index), r) with r == x for an identity residual branch: on the fused
        aggregate-first path r is an alias whose gradient the conv's backward sums into dx in its
        own aggregation store (internal to SAGEResBNNet.forward; not part of PyG's API)."""
        if (not getattr(self, "explain", False) and not self._transform_first()
                and self._aggregate_first_ok(x) and torch.is_grad_enabled()):
            plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
            return _SAGEAggregateFirst.apply(x, self.lin_l.weight, self.lin_r.weight, self.lin_l.bias, plan, True)
        return self.forward(x, edge_index), x

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        if getattr(self, "explain", False) and getattr(self, "_edge_mask", None) is not None:
            # PyG explain mode (set_masks): messages x_j scaled by the (sigmoided) edge mask
            m = self._edge_mask.sigmoid() if getattr(self, "_apply_sigmoid", True) else self._edge_mask
            agg = masked_mean_aggregate(x, edge_index, m)
            return linear2(agg, x, self.lin_l.weight, self.lin_r.weight, self.lin_l.bias)
        if self._transform_first():
            fo = self.out_channels
            y = linear_stacked(x, self.lin_l.weight, self.lin_r.weight)  # [N, 2*F_out]: MFMA GEMM (K7)
            plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
            return _MeanAggRootBias.apply(y, self.lin_l.bias, plan, fo)
        if self._aggregate_first_ok(x):
            plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
            return _SAGEAggregateFirst.apply(x, self.lin_l.weight, self.lin_r.weight, self.lin_l.bias, plan)
        agg = mean_aggregate(x, edge_index)
        return linear2(agg, x, self.lin_l.weight, self.lin_r.weight, self.lin_l.bias)  # one K7 GEMM

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, aggr={self.aggr})"


class GCNConv(nn.Module):
    """GCN ``out_i = sum_{j->i, incl. self loop} dinv_j dinv_i (W x_j) + b`` (PyG GCNConv defaults)."""

    def __init__(self, in_channels: int, out_channels: int, improved: bool = False, cached: bool = False,
                 add_self_loops: bool = True, normalize: bool = True, bias: bool = True, **kwargs):
        super().__init__()
        if improved or not add_self_loops or not normalize or kwargs:
            raise NotImplementedError("only GCNConv(improved=False, add_self_loops=True, normalize=True)")
        self.in_channels = int(in_channels)
        self.out_channels = int(out_channels)
        self.cached = cached  # plans are cached per edge_index regardless
        self.lin = Linear(self.in_channels, self.out_channels, bias=False)
        self.bias = nn.Parameter(torch.empty(self.out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        _glorot_(self.lin.weight)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        if getattr(self, "explain", False) and getattr(self, "_edge_mask", None) is not None:
            m = self._edge_mask.sigmoid() if getattr(self, "_apply_sigmoid", True) else self._edge_mask
            return masked_gcn_aggregate(self.lin(x), edge_index, m, self.bias)
        y = self.lin(x)  # transform first (PyG order): aggregation width = out_channels
        return gcn_aggregate(y, edge_index, self.bias)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


class GATConv(nn.Module):
    """GAT (PyG GATConv, v1 attention) with ``heads`` heads of ``out_channels`` each."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim=None, fill_value="mean", bias: bool = True, **kwargs):
        super().__init__()
        if dropout != 0.0 or not add_self_loops or edge_dim is not None or kwargs:
            raise NotImplementedError("only GATConv(dropout=0, add_self_loops=True, edge_dim=None)")
        self.in_channels = int(in_channels)
        self.out_channels = int(out_channels)
        self.heads = int(heads)
        self.concat = bool(concat)
        self.negative_slope = float(negative_slope)
        self.lin = Linear(self.in_channels, self.heads * self.out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, self.heads, self.out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, self.heads, self.out_channels))
        nb = self.heads * self.out_channels if self.concat else self.out_channels
        self.bias = nn.Parameter(torch.empty(nb)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        _glorot_(self.lin.weight)
        _glorot_(self.att_src)
        _glorot_(self.att_dst)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        # PyG < 2.5 stored the shared projection as lin_src (== lin_dst): accept both spellings.
        old = prefix + "lin_src.weight"
        if old in state_dict and prefix + "lin.weight" not in state_dict:
            state_dict[prefix + "lin.weight"] = state_dict.pop(old)
            state_dict.pop(prefix + "lin_dst.weight", None)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, *, _post=None) -> torch.Tensor:
        """``_post`` = (act, dropout_p, seed, seed_ctr): GATNet's ``dropout(elu(.))`` applied on the
        kernel's store (gnn.py:72-74) — internal to GATNet.forward, not part of PyG's API."""
        if getattr(self, "explain", False) and getattr(self, "_edge_mask", None) is not None:
            # PyG explain mode: each message alpha * xh_j scaled by the (sigmoided) edge mask
            m = self._edge_mask.sigmoid() if getattr(self, "_apply_sigmoid", True) else self._edge_mask
            return masked_gat_attention(self.lin(x), self.att_src, self.att_dst, self.bias, edge_index, m,
                                        self.heads, self.out_channels, self.concat, self.negative_slope)
        xh = self.lin(x)  # [N, H*C]
        act, p, seed, ctr = _post if _post is not None else (_lib.ACT_NONE, 0.0, 0, None)
        return gat_attention(xh, self.att_src, self.att_dst, self.bias, edge_index, self.heads,
                             self.out_channels, self.concat, self.negative_slope, act, p, seed, ctr)

    def _forward_proj(self, x: torch.Tensor, edge_index: torch.Tensor, w_out: torch.Tensor, _post) -> torch.Tensor:
        """forward(x, edge_index, _post=_post) · w_outᵀ with the projection on the attention kernel's
        store (aggregation.gat_attention_proj) — internal to GATNet.forward: its last hidden layer and
        the output conv's ``lin``."""
        act, p, seed, ctr = _post
        return gat_attention_proj(self.lin(x), self.att_src, self.att_dst, self.bias, w_out, edge_index,
                                  self.heads, self.out_channels, self.negative_slope, act, p, seed, ctr)

    def _forward_from_xh(self, xh: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        """forward() with ``lin(x)`` already given (GATNet.forward's fused projection)."""
        return gat_attention(xh, self.att_src, self.att_dst, self.bias, edge_index, self.heads,
                             self.out_channels, self.concat, self.negative_slope)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, heads={self.heads})"


def set_masks(model: nn.Module, mask: torch.Tensor, edge_index: torch.Tensor, apply_sigmoid: bool = True) -> None:
    """PyG ``torch_geometric.explain.algorithm.utils.set_masks``: put every conv of ``model`` in
    explain mode with the per-edge message multiplier ``mask`` [E] (GNNExplainer's hook,
    src/analysis/explain.py:593-672)."""
    loop_mask = edge_index[0] != edge_index[1]
    for module in model.modules():
        if isinstance(module, (SAGEConv, GCNConv, GATConv)):
            module.explain = True
            module._edge_mask = mask
            module._loop_mask = loop_mask
            module._apply_sigmoid = apply_sigmoid


def clear_masks(model: nn.Module) -> nn.Module:
    """PyG ``clear_masks``: leave explain mode."""
    for module in model.modules():
        if isinstance(module, (SAGEConv, GCNConv, GATConv)):
            module.explain = False
            module._edge_mask = None
            module._loop_mask = None
            module._apply_sigmoid = True
    return model
