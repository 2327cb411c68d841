"""NeighborLoader — mini-batch neighbour sampling on the MI355X (K11, csrc/sample.hip).

The reference's mini-batch path (``mini_batch: true``, src/train_gnn.py:329-348) wraps the
graph in ``torch_geometric.loader.NeighborLoader(data, num_neighbors=fanout,
batch_size=batch_size, input_nodes=idx, shuffle=...)`` and trains / evaluates on
``logits[:batch.batch_size]`` of every sampled subgraph (train_epoch_minibatch :212-245,
eval_val_minibatch :260-276).  This class keeps that constructor and the batch attributes the
reference reads (``x``, ``edge_index``, ``y``, ``timestep``, ``batch_size``) plus PyG's
bookkeeping (``n_id``, ``e_id``, ``input_id``, ``num_sampled_nodes``, ``num_sampled_edges``).

The sampling itself is one C-ABI call per batch (``gnn_neighbor_sample``) over the cached
CSR-by-target plan of the full graph; the subgraph it returns is an ordinary ``edge_index``
that the full-batch kernels run on unchanged.  Draws come from a counter hash seeded from
torch's default generator (so ``set_seed`` makes an epoch reproducible); PyG's own draws
(pyg-lib RNG) cannot be reproduced, so parity here is the sampling CONTRACT — see
tests/test_gpu_sampler.py.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sequence

import torch

from . import _lib
from .dataset_elliptic import GraphData
from .graph import get_plan


class NeighborLoader:
    """``torch_geometric.loader.NeighborLoader`` for homogeneous graphs (the reference's use).

    ``num_neighbors[h]``: in-neighbours sampled per node in hop h (-1 = all); ``input_nodes``:
    seed nodes (index tensor, boolean mask, or None = every node); ``shuffle`` draws a new seed
    order every epoch from torch's default generator, as PyG's DataLoader does.
    """

    def __init__(self, data: GraphData, num_neighbors: Sequence[int], batch_size: int = 1,
                 input_nodes: Optional[torch.Tensor] = None, shuffle: bool = False, drop_last: bool = False,
                 device: Optional[torch.device] = None):
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        self.num_neighbors = [int(k) for k in num_neighbors]
        for k in self.num_neighbors:
            if k == 0 or k < -1:
                raise ValueError(f"num_neighbors entries must be -1 or >= 1, got {k}")
        dev = torch.device(device) if device is not None else data.x.device
        if dev.type != "cuda":
            raise RuntimeError("NeighborLoader samples on the MI355X (HIP) device; pass device='cuda' "
                               "or move the data there (there is no CPU fallback)")
        self.device = dev
        self.data = data if data.x.device == dev else data.to(dev)
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        N = self.data.num_nodes
        self.num_nodes = N
        if input_nodes is None:
            idx = torch.arange(N, device=dev)
        else:
            idx = input_nodes.to(dev)
            if idx.dtype == torch.bool:
                idx = idx.nonzero().view(-1)
        self.input_nodes = idx.to(torch.int64)
        ei = self.data.edge_index
        self.num_edges = int(ei.size(1))
        self.plan = get_plan(ei, N, _lib.LOOPS_KEEP)
        # capacities: a batch holds at most B·Π(fanout) new nodes per hop (N overall), and every
        # node is expanded at most once, so at most every slot once
        B = self.batch_size
        node_cap, edge_cap, width = B, 0, B
        S = self.plan.num_slots
        for k in self.num_neighbors:
            edge_cap += S if k < 0 else width * k  # a hop's edges: Σ min(deg, k) over its frontier
            width = N if k < 0 else min(width * k, N)
            node_cap += width
        self.node_cap = max(1, min(node_cap, N))
        self.edge_cap = max(1, min(edge_cap, self.plan.num_slots))
        lib = _lib.load()
        nb = _lib.c_size(0)
        _lib.check(lib.gnn_neighbor_sample_workspace_size(N, self.node_cap, self.edge_cap, nb),
                   "gnn_neighbor_sample_workspace_size")
        self._ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        self._fan = (ctypes_i32 * max(1, len(self.num_neighbors)))(*self.num_neighbors)
        self._node_keys = [k for k in self.data.keys()
                           if k != "edge_index" and getattr(self.data, k).dim() >= 1
                           and getattr(self.data, k).size(0) == N]
        self._edge_keys = [k for k in self.data.keys()
                           if k.startswith("edge_") and k != "edge_index"
                           and getattr(self.data, k).size(0) == self.num_edges]

    def __len__(self) -> int:
        n = int(self.input_nodes.numel())
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def __iter__(self) -> Iterator[GraphData]:
        n = int(self.input_nodes.numel())
        if self.shuffle:
            order = torch.randperm(n).to(self.device)  # torch's default generator, as RandomSampler
        else:
            order = torch.arange(n, device=self.device)
        for b in range(len(self)):
            pos = order[b * self.batch_size:(b + 1) * self.batch_size]
            yield self.sample(self.input_nodes.index_select(0, pos), input_id=pos)

    def sample(self, seeds: torch.Tensor, seed: Optional[int] = None,
               input_id: Optional[torch.Tensor] = None) -> GraphData:
        """One batch around ``seeds`` (distinct node ids).  ``seed`` fixes the draws (default:
        the next 63-bit value of torch's default generator)."""
        if seed is None:
            seed = int(torch.randint(0, 2 ** 63 - 1, (1,)).item())
        seeds32 = seeds.to(device=self.device, dtype=torch.int32).contiguous()
        B = int(seeds32.numel())
        if B > self.node_cap:
            raise ValueError(f"{B} seeds exceed the loader's batch_size {self.batch_size}")
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        n_id = torch.empty(self.node_cap, **i32)
        e_src = torch.empty(self.edge_cap, **i32)
        e_dst = torch.empty(self.edge_cap, **i32)
        e_id = torch.empty(self.edge_cap, **i32)
        H = len(self.num_neighbors)
        hop_nodes = (ctypes_i64 * (H + 1))()
        hop_edges = (ctypes_i64 * max(1, H))()
        lib = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(lib.gnn_neighbor_sample(
                self.plan.c_graph, self.plan.csr_eid.data_ptr(), seeds32.data_ptr(), B, H, _lib.ctypes.addressof(self._fan),
                seed & 0xFFFFFFFFFFFFFFFF, n_id.data_ptr(), self.node_cap, e_src.data_ptr(), e_dst.data_ptr(),
                e_id.data_ptr(), self.edge_cap, _lib.ctypes.addressof(hop_nodes), _lib.ctypes.addressof(hop_edges), self._ws.data_ptr(), self._ws.numel(),
                _lib.stream_handle(dev)), "gnn_neighbor_sample")
        nn = sum(hop_nodes[h] for h in range(H + 1))
        ne = sum(hop_edges[h] for h in range(H))
        n_id = n_id[:nn].to(torch.int64)
        e_id = e_id[:ne].to(torch.int64)
        out = {k: getattr(self.data, k).index_select(0, n_id) for k in self._node_keys}
        out.update({k: getattr(self.data, k).index_select(0, e_id) for k in self._edge_keys})
        out["edge_index"] = torch.stack([e_src[:ne], e_dst[:ne]]).to(torch.int64)
        out["n_id"] = n_id
        out["e_id"] = e_id
        if input_id is not None:
            out["input_id"] = input_id
        batch = GraphData(**out)
        batch.batch_size = B
        batch.num_sampled_nodes = [int(hop_nodes[h]) for h in range(H + 1)]
        batch.num_sampled_edges = [int(hop_edges[h]) for h in range(H)]
        return batch


ctypes_i32 = _lib.ctypes.c_int32
ctypes_i64 = _lib.ctypes.c_int64
