"""ORACLE — test infrastructure only.  CPU restatement of the reference hot path.

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline.  The product path
(elliptic_gnn_project_amd) never imports it.

What it restates
----------------
The arithmetic of the reference's hot path lives in the third-party package
**torch-geometric 2.5.3** (pinned in the reference's CI: .github/workflows/ci.yml:17,39,
with torch 2.2.0 at :16,29).  PyG is not vendored in /root/reference and is not installed
in this image, so this module restates its published algorithm for the calls
src/models/gnn.py makes, using the same ATen op sequence PyG 2.5.3 issues on CPU for a
dense ``edge_index`` (so it doubles as the "PyG-CPU" timing stand-in):

  utils.scatter(reduce='sum'|'mean'|'max')   scatter_add_ / count-divide / scatter_reduce_(amax)
  MessagePassing.propagate                   x.index_select(0, edge_index[0]) -> aggregate at [1]
  SAGEConv(aggr='mean')                      lin_l(mean) + lin_r(x)               (gnn.py:41-44)
  GCNConv + gcn_norm                         add_remaining_self_loops, deg^-1/2   (gnn.py:20-23)
  GATConv + utils.softmax                    leaky_relu(a_j + a_i), softmax +1e-16 (gnn.py:64-67)

Model composition follows src/models/gnn.py:14-194 and the loss/step follow
src/train_gnn.py:136-209.

Parity pinning
--------------
The reference holds no golden vectors, fixtures or tests for this path (its only tests,
tests/test_masks_and_metrics.py, cover masks and metrics), and PyG cannot be imported
here, so **parity against the reference's own outputs is unpinned**.  This restatement
is pinned instead by hand-derived known-answer tests (tests/test_oracle_kat.py) and by
cross-checks against the independent pure-Python loop forms in oracle/loops.py.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


# ----------------------------------------------------------------------------- utils.scatter
def _broadcast(index: Tensor, src: Tensor) -> Tensor:
    # torch_geometric.utils._scatter.broadcast for dim=0
    view = [-1] + [1] * (src.dim() - 1)
    return index.view(view).expand_as(src)


def scatter(src: Tensor, index: Tensor, dim_size: int, reduce: str = "sum") -> Tensor:
    """PyG 2.5.3 utils.scatter along dim 0 (torch>=1.12 branch)."""
    size = (dim_size,) + tuple(src.shape[1:])
    if reduce in ("sum", "add"):
        return src.new_zeros(size).scatter_add_(0, _broadcast(index, src), src)
    if reduce == "mean":
        count = src.new_zeros(dim_size)
        count.scatter_add_(0, index, src.new_ones(src.size(0)))
        count = count.clamp(min=1)
        out = src.new_zeros(size).scatter_add_(0, _broadcast(index, src), src)
        return out / count.view([-1] + [1] * (out.dim() - 1))
    if reduce in ("max", "amax"):
        return src.new_zeros(size).scatter_reduce_(0, _broadcast(index, src), src, reduce="amax",
                                                   include_self=False)
    raise ValueError(reduce)


def softmax(src: Tensor, index: Tensor, num_nodes: int) -> Tensor:
    """PyG 2.5.3 utils.softmax (index form)."""
    src_max = scatter(src.detach(), index, num_nodes, reduce="max")
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = scatter(out, index, num_nodes, reduce="sum") + 1e-16
    return out / out_sum.index_select(0, index)


def remove_self_loops(edge_index: Tensor) -> Tensor:
    return edge_index[:, edge_index[0] != edge_index[1]]


def add_self_loops(edge_index: Tensor, num_nodes: int) -> Tensor:
    loop = torch.arange(num_nodes, dtype=torch.long, device=edge_index.device).unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1)


def add_remaining_self_loops(edge_index: Tensor, num_nodes: int) -> Tensor:
    # edge_attr=None branch: keep non-loop edges, append one loop per node
    return add_self_loops(remove_self_loops(edge_index), num_nodes)


# ----------------------------------------------------------------------------- convs
def sage_conv(x: Tensor, edge_index: Tensor, lin_l_w: Tensor, lin_l_b: Optional[Tensor],
              lin_r_w: Tensor) -> Tensor:
    """SAGEConv(aggr='mean', root_weight=True): lin_l(mean_j x_j) + lin_r(x)."""
    x_j = x.index_select(0, edge_index[0])
    agg = scatter(x_j, edge_index[1], x.size(0), reduce="mean")
    return F.linear(agg, lin_l_w, lin_l_b) + F.linear(x, lin_r_w)


def sage_conv_explain(x: Tensor, edge_index: Tensor, edge_mask: Tensor, lin_l_w: Tensor,
                      lin_l_b: Optional[Tensor], lin_r_w: Tensor, apply_sigmoid: bool = True) -> Tensor:
    """SAGEConv in explain mode [PyG 2.5.3 MessagePassing.propagate, `if self._explain`]:
    the message x_j is multiplied by edge_mask (sigmoided when `_apply_sigmoid`) before the
    'mean' aggregation; the count stays the in-degree.  Set by `explain.algorithm.utils.set_masks`
    (GNNExplainer, src/analysis/explain.py:593-672)."""
    m = edge_mask.sigmoid() if apply_sigmoid else edge_mask
    x_j = x.index_select(0, edge_index[0]) * m.view(-1, 1)
    agg = scatter(x_j, edge_index[1], x.size(0), reduce="mean")
    return F.linear(agg, lin_l_w, lin_l_b) + F.linear(x, lin_r_w)


def gcn_norm(edge_index: Tensor, num_nodes: int, dtype=torch.float32):
    ei = add_remaining_self_loops(edge_index, num_nodes)
    w = torch.ones(ei.size(1), dtype=dtype, device=ei.device)
    row, col = ei[0], ei[1]
    deg = scatter(w, col, num_nodes, reduce="sum")
    dinv = deg.pow_(-0.5)
    dinv.masked_fill_(dinv == float("inf"), 0)
    return ei, dinv[row] * w * dinv[col]


def gcn_conv(x: Tensor, edge_index: Tensor, lin_w: Tensor, bias: Optional[Tensor]) -> Tensor:
    ei, w = gcn_norm(edge_index, x.size(0), x.dtype)
    h = F.linear(x, lin_w)
    out = scatter(w.view(-1, 1) * h.index_select(0, ei[0]), ei[1], x.size(0), reduce="sum")
    return out + bias if bias is not None else out


def gcn_conv_explain(x: Tensor, edge_index: Tensor, edge_mask: Tensor, lin_w: Tensor, bias: Optional[Tensor],
                     apply_sigmoid: bool = True) -> Tensor:
    """GCNConv in explain mode [PyG 2.5.3 propagate]: messages w_e * h_j times the mask; the mask of
    the non-loop input edges is kept (`edge_mask[self._loop_mask]`) and the appended loops get 1."""
    m = edge_mask.sigmoid() if apply_sigmoid else edge_mask
    keep = edge_index[0] != edge_index[1]
    m = torch.cat([m[keep], m.new_ones(x.size(0))])
    ei, w = gcn_norm(edge_index, x.size(0), x.dtype)
    h = F.linear(x, lin_w)
    out = scatter((w.view(-1, 1) * h.index_select(0, ei[0])) * m.view(-1, 1), ei[1], x.size(0), reduce="sum")
    return out + bias if bias is not None else out


def gat_conv(x: Tensor, edge_index: Tensor, lin_w: Tensor, att_src: Tensor, att_dst: Tensor,
             bias: Optional[Tensor], heads: int, chans: int, concat: bool = True,
             negative_slope: float = 0.2, return_alpha: bool = False):
    N = x.size(0)
    xh = F.linear(x, lin_w).view(-1, heads, chans)
    a_src = (xh * att_src).sum(dim=-1)
    a_dst = (xh * att_dst).sum(dim=-1)
    ei = add_self_loops(remove_self_loops(edge_index), N)
    alpha = a_src.index_select(0, ei[0]) + a_dst.index_select(0, ei[1])
    alpha = F.leaky_relu(alpha, negative_slope)
    alpha = softmax(alpha, ei[1], N)
    msg = alpha.unsqueeze(-1) * xh.index_select(0, ei[0])
    out = scatter(msg, ei[1], N, reduce="sum")
    out = out.reshape(N, heads * chans) if concat else out.mean(dim=1)
    if bias is not None:
        out = out + bias
    return (out, alpha, ei) if return_alpha else out


def gat_conv_explain(x: Tensor, edge_index: Tensor, edge_mask: Tensor, lin_w: Tensor, att_src: Tensor,
                     att_dst: Tensor, bias: Optional[Tensor], heads: int, chans: int, concat: bool = True,
                     negative_slope: float = 0.2, apply_sigmoid: bool = True) -> Tensor:
    """GATConv in explain mode [PyG 2.5.3 MessagePassing.propagate, `if self._explain`]: the
    message alpha * xh_j (after the edge softmax) is multiplied by the edge mask; the mask of the
    non-loop input edges is kept (`edge_mask[self._loop_mask]`) and the appended loops get 1.
    The reference drives it through GNNExplainer on GAT models (src/analysis/explain.py:309,593-672)."""
    N = x.size(0)
    m = edge_mask.sigmoid() if apply_sigmoid else edge_mask
    keep = edge_index[0] != edge_index[1]
    m = torch.cat([m[keep], m.new_ones(N)])
    xh = F.linear(x, lin_w).view(-1, heads, chans)
    a_src = (xh * att_src).sum(dim=-1)
    a_dst = (xh * att_dst).sum(dim=-1)
    ei = add_self_loops(remove_self_loops(edge_index), N)
    alpha = F.leaky_relu(a_src.index_select(0, ei[0]) + a_dst.index_select(0, ei[1]), negative_slope)
    alpha = softmax(alpha, ei[1], N)
    msg = (alpha.unsqueeze(-1) * xh.index_select(0, ei[0])) * m.view(-1, 1, 1)
    out = scatter(msg, ei[1], N, reduce="sum")
    out = out.reshape(N, heads * chans) if concat else out.mean(dim=1)
    return out + bias if bias is not None else out


# ----------------------------------------------------------------------------- models (gnn.py)
def _dropout(h: Tensor, p: float, training: bool, mask: Optional[Tensor]) -> Tensor:
    if not training or p == 0.0:
        return h
    if mask is None:
        return F.dropout(h, p=p, training=True)
    return h * (mask.to(h.dtype) / (1.0 - p))  # ATen dropout: input * (bernoulli(1-p) / (1-p))


def sinusoid(t_idx: Tensor, dim: int, max_timestep: int) -> Tensor:
    """SAGEResBNNet._sinusoid (src/models/gnn.py:146-166)."""
    t = torch.clamp(t_idx.long() - 1, 0, max_timestep - 1).to(torch.float32)
    t = t / max(float(max_timestep - 1), 1.0)
    half = dim // 2
    freqs = torch.arange(1, half + 1, dtype=t.dtype) * (2.0 * math.pi)
    ang = t.unsqueeze(1) * freqs.unsqueeze(0)
    feat = torch.cat([torch.sin(ang), torch.cos(ang)], dim=1)
    if feat.size(1) < dim:
        feat = torch.cat([feat, torch.zeros(feat.size(0), dim - feat.size(1), dtype=feat.dtype)], dim=1)
    return feat


def model_forward(arch: str, p: Dict[str, Tensor], x: Tensor, edge_index: Tensor,
                  layers: int, dropout: float = 0.0, training: bool = False, heads: int = 4,
                  t_idx: Optional[Tensor] = None, time_embed_dim: int = 0, time_embed_type: str = "none",
                  max_timestep: int = 49, use_bn: bool = True, dropout_masks=None,
                  bn_state: Optional[Dict[str, Tensor]] = None, relu_force=None, trace=None) -> Tensor:
    """Forward of GCNNet / SAGENet / GATNet / SAGEResBNNet with PyG-keyed parameters ``p``.

    Test hooks (SAGE-ResBN): ``trace`` (a list) receives each hidden layer's pre-ReLU BatchNorm
    output; ``relu_force`` ({layer: (flat indices, bool keep)}) fixes the ReLU decision of those
    elements — ties (|BN(z)| at the fp32 rounding of z) that an fp32 device may resolve either way,
    so a parity test can check the device against the oracle for the tie resolution it took."""
    masks = list(dropout_masks) if dropout_masks is not None else [None] * layers
    h = x
    if arch == "sage":
        for i in range(layers):
            h = sage_conv(h, edge_index, p[f"convs.{i}.lin_l.weight"], p.get(f"convs.{i}.lin_l.bias"),
                          p[f"convs.{i}.lin_r.weight"])
            if i < layers - 1:
                h = _dropout(F.relu(h), dropout, training, masks[i])
        return h
    if arch == "gcn":
        for i in range(layers):
            h = gcn_conv(h, edge_index, p[f"convs.{i}.lin.weight"], p.get(f"convs.{i}.bias"))
            if i < layers - 1:
                h = _dropout(F.relu(h), dropout, training, masks[i])
        return h
    if arch == "gat":
        for i in range(layers):
            last = i == layers - 1
            H = 1 if last else heads
            w = p[f"convs.{i}.lin.weight"]
            C = w.size(0) // H
            h = gat_conv(h, edge_index, w, p[f"convs.{i}.att_src"], p[f"convs.{i}.att_dst"],
                         p.get(f"convs.{i}.bias"), H, C, concat=not last)
            if not last:
                h = _dropout(F.elu(h), dropout, training, masks[i])
        return h
    if arch in ("sage_resbn", "sage_bn", "sage_res"):
        if time_embed_dim > 0 and t_idx is not None:
            if time_embed_type == "sin":
                h = torch.cat([h, sinusoid(t_idx, time_embed_dim, max_timestep)], dim=1)
            elif time_embed_type == "learned":
                te = p["time_emb.weight"][torch.clamp(t_idx.long() - 1, 0, max_timestep - 1)]
                h = torch.cat([h, te], dim=1)
        for i in range(layers - 1):
            h_in = h
            z = sage_conv(h, edge_index, p[f"convs.{i}.lin_l.weight"], p.get(f"convs.{i}.lin_l.bias"),
                          p[f"convs.{i}.lin_r.weight"])
            if use_bn:
                rm = bn_state.get(f"bns.{i}.running_mean") if bn_state else None
                rv = bn_state.get(f"bns.{i}.running_var") if bn_state else None
                z = F.batch_norm(z, rm, rv, p[f"bns.{i}.weight"], p[f"bns.{i}.bias"], training or rm is None,
                                 0.1, 1e-5)
            if trace is not None:
                trace.append(z.detach())
            if relu_force is not None and i in relu_force:
                idx, keep = relu_force[i]
                on = (z > 0).flatten().clone()
                on[idx] = keep
                z = _dropout(z * on.view_as(z).to(z.dtype), dropout, training, masks[i])
            else:
                z = _dropout(F.relu(z), dropout, training, masks[i])
            rp = p.get(f"res_projs.{i}.weight")
            h = z + (F.linear(h_in, rp) if rp is not None else h_in)
        i = layers - 1
        return sage_conv(h, edge_index, p[f"convs.{i}.lin_l.weight"], p.get(f"convs.{i}.lin_l.bias"),
                         p[f"convs.{i}.lin_r.weight"])
    raise ValueError(f"unknown arch {arch}")


# ----------------------------------------------------------------------------- loss / step (train_gnn.py)
def class_weight(train_y: Tensor) -> Tensor:
    """src/train_gnn.py:116-123."""
    pos = int((train_y == 1).sum())
    neg = int((train_y == 0).sum())
    if pos == 0 or neg == 0:
        return torch.tensor([1.0, 1.0], dtype=torch.float32)
    return torch.tensor([(pos + neg) / (2.0 * neg), (pos + neg) / (2.0 * pos)], dtype=torch.float32)


def ce_loss(logits: Tensor, target: Tensor, cw: Tensor) -> Tensor:
    """src/train_gnn.py:159-175 (CE path): weighted per-sample CE, unweighted mean."""
    return F.cross_entropy(logits, target, weight=cw, reduction="none").mean()


def train_step_grads(arch: str, params: Dict[str, Tensor], x: Tensor, edge_index: Tensor, y: Tensor,
                     train_mask: Tensor, cw: Tensor, **kw):
    """fwd + masked loss + bwd (src/train_gnn.py:192-202); returns (loss, {name: grad})."""
    leaf = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in params.items()}
    logits = model_forward(arch, leaf, x, edge_index, **kw)
    loss = ce_loss(logits[train_mask], y[train_mask], cw)
    loss.backward()
    return loss.detach(), {k: v.grad for k, v in leaf.items() if v.grad is not None}
