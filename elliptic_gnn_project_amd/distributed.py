"""Timestep-partitioned data parallelism: one process per MI355X, RCCL over xGMI.

Why it is exact: every Elliptic edge joins two nodes of the same timestep (the loader drops
the rest: src/data/dataset_elliptic.py:235-243), so the graph is block-diagonal over the 49
timesteps and any depth of message passing on a subset of whole timesteps needs no halo.

  partition_timesteps   greedy LPT bin-packing of timesteps (cost a·N_t + b·E_t) onto ranks
  local_subgraph        a rank's node rows + its edges relabelled to local ids
  shard_graph           a prepared graph's rows / edges / masks for one rank (host side)
  gather_rows           every rank's per-node outputs back into one [N, ...] tensor (eval)
  global_class_weight_and_count
                        class weights from the GLOBAL train labels (src/train_gnn.py:362-365)
                        and the global train count, so sum-over-ranks of the per-rank
                        ``sum(loss)/count`` equals the single-device ``.mean()`` (:175)
  GradBucket            all parameter gradients as views of ONE flat fp32 buffer: one
                        all-reduce per step (≈170 KB for the SAGE preset: latency-bound, so
                        a single bucket beats per-tensor calls on point-to-point xGMI)
  SyncBatchNorm1d       BatchNorm over all N nodes across ranks (SAGEResBNNet, gnn.py:188-189):
                        all-reduce of (Σx, Σx², n) forward and (Σdy, Σdy·x̂) backward
Collectives go through torch.distributed: backend "nccl" (= RCCL) on MI355X, "gloo" in the
CPU tests.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn


def partition_timesteps(timestep: torch.Tensor, edge_index: torch.Tensor, world: int,
                        node_cost: float = 1.0, edge_cost: float = 1.0) -> List[List[int]]:
    """LPT: heaviest timestep first onto the least-loaded rank.  Deterministic."""
    ts = torch.unique(timestep).tolist()
    n_t = torch.bincount(timestep, minlength=max(ts) + 1).double()
    e_t = torch.bincount(timestep[edge_index[1]], minlength=max(ts) + 1).double() \
        if edge_index.numel() else torch.zeros_like(n_t)
    cost = {t: node_cost * float(n_t[t]) + edge_cost * float(e_t[t]) for t in ts}
    bins: List[List[int]] = [[] for _ in range(world)]
    load = [0.0] * world
    for t in sorted(ts, key=lambda t: (-cost[t], t)):
        r = min(range(world), key=lambda i: (load[i], i))
        bins[r].append(t)
        load[r] += cost[t]
    return [sorted(b) for b in bins]


def local_subgraph(timestep: torch.Tensor, edge_index: torch.Tensor, steps: Sequence[int]
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    """(global node ids of this rank, edge_index relabelled to local ids, edge order kept)."""
    sel = torch.isin(timestep, torch.as_tensor(list(steps), dtype=timestep.dtype))
    nodes = torch.nonzero(sel, as_tuple=False).flatten()
    local = torch.full((timestep.numel(),), -1, dtype=torch.long)
    local[nodes] = torch.arange(nodes.numel())
    keep = sel[edge_index[0]] & sel[edge_index[1]]
    if bool((sel[edge_index[0]] != sel[edge_index[1]]).any()):
        raise ValueError("edge crosses a timestep partition: the graph is not block-diagonal in time")
    return nodes, local[edge_index[:, keep]]


def shard_graph(data, world: int, rank: int, parts: Optional[List[List[int]]] = None,
                key: Optional[torch.Tensor] = None):
    """This rank's whole-timestep shard of a prepared graph (prepare_inputs output, on the host).

    Returns a GraphData with the local rows of every node tensor (x, y, timestep, the split
    masks and their indices), the relabelled local ``edge_index`` (PyG edge order kept) and
    ``nodes`` (global row ids, ascending), plus ``parts`` (the timesteps of every rank).
    ``key`` (default ``data.timestep``) is the per-node partition unit: bench.py's weak-scaling
    graph of several Elliptic blocks partitions by (block, timestep)."""
    from .dataset_elliptic import GraphData, index_masks

    key = data.timestep if key is None else key
    if parts is None:
        parts = partition_timesteps(key, data.edge_index, world)
    nodes, ei = local_subgraph(key, data.edge_index, parts[rank])
    local = {"edge_index": ei, "nodes": nodes}
    n = data.timestep.numel()
    for k in data.keys():
        v = getattr(data, k)
        if k in ("edge_index",) or k.endswith("_idx"):
            continue
        if v.dim() >= 1 and v.size(0) == n:
            local[k] = v.index_select(0, nodes)
    out = GraphData(**local)
    out.parts = parts
    return index_masks(out)


def gather_rows(values: torch.Tensor, nodes: torch.Tensor, num_nodes: int, dist) -> torch.Tensor:
    """Scatter every rank's per-node ``values`` (rows of its local ``nodes``) into one [num_nodes,
    ...] tensor on every rank (all_gather of zero-padded blocks; the shards are disjoint)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        out = values.new_zeros((num_nodes,) + tuple(values.shape[1:]))
        out[nodes.to(values.device)] = values
        return out
    world = dist.get_world_size()
    if values.is_cuda and dist.get_backend() == "gloo":  # gloo gathers host tensors
        return gather_rows(values.cpu(), nodes.cpu(), num_nodes, dist).to(values.device)
    cnt = torch.tensor([values.size(0)], dtype=torch.int64, device=values.device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    mx = int(max(int(c) for c in cnts))
    pad_v = values.new_zeros((mx,) + tuple(values.shape[1:]))
    pad_v[: values.size(0)] = values
    pad_n = torch.full((mx,), -1, dtype=torch.int64, device=values.device)
    pad_n[: values.size(0)] = nodes.to(values.device)
    vs = [torch.empty_like(pad_v) for _ in range(world)]
    ns = [torch.empty_like(pad_n) for _ in range(world)]
    dist.all_gather(vs, pad_v)
    dist.all_gather(ns, pad_n)
    out = values.new_zeros((num_nodes,) + tuple(values.shape[1:]))
    for v, nn_, c in zip(vs, ns, cnts):
        c = int(c)
        out[nn_[:c]] = v[:c]
    return out


def global_class_weight_and_count(y: torch.Tensor, train_mask: torch.Tensor, dist=None
                                  ) -> Tuple[torch.Tensor, int]:
    yt = y[train_mask]
    cnt = torch.stack([(yt == 0).sum(), (yt == 1).sum()]).to(torch.float64)
    if dist is not None and dist.is_initialized():
        dist.all_reduce(cnt)
    neg, pos = float(cnt[0]), float(cnt[1])
    if pos == 0 or neg == 0:
        cw = torch.tensor([1.0, 1.0], dtype=torch.float32)
    else:
        cw = torch.tensor([(pos + neg) / (2.0 * neg), (pos + neg) / (2.0 * pos)], dtype=torch.float32)
    return cw, int(pos + neg)


class GradBucket:
    """Flat gradient buffer; every ``p.grad`` is a view into it (zero_grad(set_to_none=False)).

    Overlap with the backward ("one fused bucket, overlapped with the last
    backward kernels").  In a net whose layers are separate autograd nodes (SAGE-ResBN, GAT, the
    per-conv paths) the later layers' gradients are final while the first layer's backward still
    runs (its weight-gradient TN is the longest kernel of the backward).  The flat buffer is then
    laid out as [early | late]: a post-accumulate hook on the early parameters issues the early
    slice's all-reduce asynchronously (``async_op``: RCCL runs it on its own stream, inside a
    captured step as a fork / join of the graph) as soon as the last of them has landed, and
    ``allreduce_`` reduces the late slice and waits for both.  Two collectives instead of one, so
    only worth it when the early gradients really come before the last producer:

      early=None      observe the first backward — parameters whose gradients landed before the
                      last batch of gradient producers (libgnnmp calls counted between the hooks,
                      _lib.CALLS) form the early slice; one batch (a fused single-node net: SAGE
                      2L, GCN) keeps one bucket
      early=[names]   the early slice by parameter name (any backend; the CPU gloo tests)
      overlap=False   one bucket, one collective after the backward (the round-5 form)

    The re-layout happens inside the first ``allreduce_`` after the observation (values copied,
    ``p.grad`` re-pointed); ``flat_in_param_order()`` gives the gradients in parameter order."""

    def __init__(self, model: nn.Module, early=None, overlap: bool = True):
        named = [(k, p) for k, p in model.named_parameters() if p.requires_grad]
        self.names = [k for k, _ in named]
        self.params = [p for _, p in named]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.order = list(range(len(self.params)))  # flat layout: parameter indices in order
        self._views()
        self.overlap = bool(overlap) and len(self.params) > 1
        self.n_early = 0          # parameters in the early slice (the first n_early of self.order)
        self.early_elems = 0
        self._arrivals = []       # (param index, _lib.CALLS) of the observed backward
        self._landed = 0
        self._work = None
        self._dist = None
        self._planned = False
        self._want = None if early is None else set(early)
        self._hooks = []
        if self.overlap:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._hook_for(i)))

    def _views(self) -> None:
        off = 0
        for i in self.order:
            p = self.params[i]
            p.grad = self.flat[off: off + p.numel()].view_as(p)
            off += p.numel()

    def _hook_for(self, i: int):
        def hook(_p):
            if not self._planned:
                from . import _lib
                self._arrivals.append((i, _lib.CALLS[0]))
                return
            if i >= len(self._is_early) or not self._is_early[i]:
                return
            self._landed += 1
            if self._landed == self.n_early and self._dist is not None and self._work is None:
                d = self._dist
                if d.get_backend() == "gloo" and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                    return  # gloo cannot be captured: allreduce_ reduces it (the split-graph form)
                self._work = d.all_reduce(self.flat[: self.early_elems], async_op=True)
        return hook

    def _plan(self) -> None:
        """Choose the early slice from the observed arrivals (or the given names) and re-lay the
        flat buffer out as [early | late], keeping the current gradient values."""
        self._planned = True
        idx = {k: i for i, k in enumerate(self.names)}
        if self._want is not None:
            early = [idx[k] for k in self.names if k in self._want]
        else:
            arr = self._arrivals
            early = []
            if arr and len({c for _, c in arr}) > 1:
                last = arr[-1][1]
                early = [i for i, c in arr if c < last]
        late = [i for i in range(len(self.params)) if i not in set(early)]
        self._is_early = [False] * len(self.params)
        for i in early:
            self._is_early[i] = True
        if not early or not late:
            self.n_early, self.early_elems = 0, 0
            return
        vals = [p.grad.detach().clone() for p in self.params]
        self.order = early + late
        self.n_early = len(early)
        self.early_elems = sum(self.params[i].numel() for i in early)
        self._views()
        for p, v in zip(self.params, vals):
            p.grad.copy_(v)

    def flat_in_param_order(self) -> torch.Tensor:
        return torch.cat([p.grad.detach().flatten() for p in self.params])

    def arm(self, dist) -> None:
        """Before the first backward: the early slice's hook may issue its collective on ``dist``
        (later backwards use the ``dist`` of the previous ``allreduce_``)."""
        self._dist = dist
        self._landed = 0
        self._work = None

    def allreduce_(self, dist) -> None:
        for p in self.params:  # re-attach if an optimizer set grads to None
            if p.grad is None or p.grad.data_ptr() < self.flat.data_ptr() or \
                    p.grad.data_ptr() >= self.flat.data_ptr() + self.flat.numel() * 4:
                raise RuntimeError("GradBucket: gradients detached from the flat buffer; "
                                   "use optimizer.zero_grad(set_to_none=False)")
        self._dist = dist  # the next backward's early hook issues on it
        if not self.overlap or not self._planned:
            dist.all_reduce(self.flat)
            if self.overlap and (self._arrivals or self._want is not None):
                self._plan()  # the next backward overlaps (values kept)
            return
        if self.n_early == 0:
            dist.all_reduce(self.flat)
            return
        work, self._work = self._work, None
        if work is None:  # the hook did not fire (not armed, a gloo capture, a missing gradient)
            dist.all_reduce(self.flat[: self.early_elems])
        dist.all_reduce(self.flat[self.early_elems:])
        if work is not None:
            work.wait()
        self._landed = 0


def global_batch_stats(x: torch.Tensor, dist) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(mean, biased var, n) of the rows of ``x`` over every rank, with ONE all-reduce.

    Each rank contributes its centred statistics (Chan's parallel merge, all-reduce-only form):
    n_r, n_r·m_r, n_r·m_r² and M2_r = Σ(x − m_r)² (local, fp32 two-pass), summed in float64:
        mean = Σ n_r m_r / n,   var = (Σ M2_r + Σ n_r m_r² − n·mean²) / n
    so features with a large mean and a small spread keep their precision (no E[x²] − mean²
    over raw fp32 sums), and the variance is never negative."""
    C = x.size(1)
    n_r = x.size(0)
    if n_r > 0:
        m_r = x.mean(0)
        m2_r = (x - m_r).pow(2).sum(0)
    else:
        m_r = x.new_zeros(C)
        m2_r = x.new_zeros(C)
    m_d = m_r.double()
    stats = torch.cat([m_d * n_r, m_d * m_d * n_r, m2_r.double(),
                       torch.full((1,), float(n_r), dtype=torch.float64, device=x.device)])
    if dist is not None:
        dist.all_reduce(stats)
    n = stats[3 * C]
    mean = stats[:C] / n
    var = ((stats[2 * C: 3 * C] + stats[C: 2 * C] - n * mean * mean) / n).clamp_(min=0.0)
    return mean.to(x.dtype), var.to(x.dtype), n


class _SyncBNFn(torch.autograd.Function):
    """y = (x − mean)·invstd·w + b with (mean, invstd) over all ranks' rows (computed by the
    caller, so the running statistics reuse them: one collective forward, one backward)."""

    @staticmethod
    def forward(ctx, x, weight, bias, mean, invstd, n, group_dist):
        xhat = (x - mean) * invstd
        ctx.save_for_backward(xhat, invstd, weight)
        ctx.n = n
        ctx.dist = group_dist
        return xhat * weight + bias

    @staticmethod
    def backward(ctx, dy):
        xhat, invstd, weight = ctx.saved_tensors
        C = dy.size(1)
        red = torch.cat([dy.sum(0), (dy * xhat).sum(0)])
        dbias_w = red.clone()
        if ctx.dist is not None:
            ctx.dist.all_reduce(red)
        n = ctx.n.to(dy.dtype)
        sdy, sdyx = red[:C], red[C:]
        dx = (weight * invstd) * (dy - sdy / n - xhat * sdyx / n)
        # parameter grads are LOCAL sums; the gradient all-reduce adds the other ranks'
        return dx, dbias_w[C:], dbias_w[:C], None, None, None, None


class SyncBatchNorm1d(nn.BatchNorm1d):
    """BatchNorm1d whose training-mode statistics span every rank's nodes (exact full-graph BN).

    Training mode: one all-reduce of the merged (mean, M2, n) statistics forward (shared by the
    normalisation and the running-stat update), one of (Σdy, Σdy·x̂) backward."""

    dist = None  # set to torch.distributed once the process group is up

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        d = self.dist if (self.dist is not None and self.dist.is_initialized()) else None
        if not self.training or d is None:
            return super().forward(x)
        with torch.no_grad():
            mean, var, n = global_batch_stats(x.detach(), d)
            invstd = torch.rsqrt(var + self.eps)
            if self.track_running_stats:  # as BatchNorm1d: momentum update, unbiased variance
                self.num_batches_tracked += 1
                # momentum None: cumulative average, as nn.BatchNorm1d
                m = self.momentum if self.momentum is not None else 1.0 / float(self.num_batches_tracked)
                unbiased = var * (n / torch.clamp(n - 1, min=1)).to(var.dtype)
                self.running_mean.mul_(1 - m).add_(m * mean)
                self.running_var.mul_(1 - m).add_(m * unbiased)
        w = self.weight if self.affine else torch.ones_like(mean)
        b = self.bias if self.affine else torch.zeros_like(mean)
        return _SyncBNFn.apply(x, w, b, mean, invstd, n, d)


def convert_sync_batchnorm(model: nn.Module, dist) -> nn.Module:
    """Swap every BatchNorm1d for SyncBatchNorm1d (state_dict keys unchanged)."""
    for name, mod in model.named_children():
        if isinstance(mod, nn.BatchNorm1d) and not isinstance(mod, SyncBatchNorm1d):
            new = SyncBatchNorm1d(mod.num_features, mod.eps, mod.momentum, mod.affine, mod.track_running_stats)
            new.load_state_dict(mod.state_dict())
            new.to(next(mod.parameters()).device if mod.affine else mod.running_mean.device)
            new.dist = dist
            setattr(model, name, new)
        else:
            convert_sync_batchnorm(mod, dist)
    return model
