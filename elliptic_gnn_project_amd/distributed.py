"""Timestep-partitioned data parallelism: one process per MI355X, RCCL over xGMI.

Why it is exact: every Elliptic edge joins two nodes of the same timestep (the loader drops
the rest: src/data/dataset_elliptic.py:235-243), so the graph is block-diagonal over the 49
timesteps and any depth of message passing on a subset of whole timesteps needs no halo.

  partition_timesteps   greedy LPT bin-packing of timesteps (cost a·N_t + b·E_t) onto ranks
  local_subgraph        a rank's node rows + its edges relabelled to local ids
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
    """Flat gradient buffer; every ``p.grad`` is a view into it (zero_grad(set_to_none=False))."""

    def __init__(self, model: nn.Module):
        self.params = [p for p in model.parameters() if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.flat[off: off + p.numel()].view_as(p)
            off += p.numel()

    def allreduce_(self, dist) -> None:
        for p in self.params:  # re-attach if an optimizer set grads to None
            if p.grad is None or p.grad.data_ptr() < self.flat.data_ptr() or \
                    p.grad.data_ptr() >= self.flat.data_ptr() + self.flat.numel() * 4:
                raise RuntimeError("GradBucket: gradients detached from the flat buffer; "
                                   "use optimizer.zero_grad(set_to_none=False)")
        dist.all_reduce(self.flat)


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, group_dist):
        dist = group_dist
        n_local = torch.tensor([float(x.size(0))], dtype=x.dtype, device=x.device)
        stats = torch.cat([x.sum(0), (x * x).sum(0), n_local])
        if dist is not None:
            dist.all_reduce(stats)
        C = x.size(1)
        n = stats[2 * C]
        mean = stats[:C] / n
        var = stats[C: 2 * C] / n - mean * mean  # biased, as BatchNorm normalises with
        invstd = torch.rsqrt(var + eps)
        xhat = (x - mean) * invstd
        ctx.save_for_backward(xhat, invstd, weight)
        ctx.n = n
        ctx.dist = dist
        return xhat * weight + bias

    @staticmethod
    def backward(ctx, dy):
        xhat, invstd, weight = ctx.saved_tensors
        C = dy.size(1)
        red = torch.cat([dy.sum(0), (dy * xhat).sum(0)])
        dbias_w = red.clone()
        if ctx.dist is not None:
            ctx.dist.all_reduce(red)
        sdy, sdyx = red[:C], red[C:]
        dx = (weight * invstd) * (dy - sdy / ctx.n - xhat * sdyx / ctx.n)
        # parameter grads are LOCAL sums; the gradient all-reduce adds the other ranks'
        return dx, dbias_w[C:], dbias_w[:C], None, None


class SyncBatchNorm1d(nn.BatchNorm1d):
    """BatchNorm1d whose training-mode statistics span every rank's nodes (exact full-graph BN)."""

    dist = None  # set to torch.distributed once the process group is up

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        d = self.dist if (self.dist is not None and self.dist.is_initialized()) else None
        if not self.training or d is None:
            return super().forward(x)
        y = _SyncBNFn.apply(x, self.weight, self.bias, self.eps, d)
        with torch.no_grad():  # running stats as BatchNorm1d: momentum update, unbiased variance
            m = self.momentum if self.momentum is not None else 0.1
            n_local = torch.tensor([float(x.size(0))], device=x.device, dtype=x.dtype)
            stats = torch.cat([x.sum(0), (x * x).sum(0), n_local])
            d.all_reduce(stats)
            C = x.size(1)
            n = stats[2 * C]
            mean = stats[:C] / n
            var = (stats[C: 2 * C] / n - mean * mean) * n / torch.clamp(n - 1, min=1)
            self.running_mean.mul_(1 - m).add_(m * mean)
            self.running_var.mul_(1 - m).add_(m * var)
            self.num_batches_tracked += 1
        return y


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
