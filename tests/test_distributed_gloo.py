"""CPU, world_size 2 over gloo: the timestep-partitioned data-parallel machinery is exact.

Each rank holds whole timesteps (no halo — the graph is block-diagonal in time), computes the
loss with the GLOBAL train count as divisor, and all-reduces one flat gradient bucket; the
summed gradient equals the single-process full-graph gradient.  SyncBatchNorm1d reproduces
BatchNorm over all N nodes.  The model arithmetic here is the CPU oracle (the HIP path needs a
GPU); what is under test is elliptic_gnn_project_amd.distributed.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from elliptic_gnn_project_amd import distributed as gdist
from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
from oracle import pyg_ref


class OracleSAGE(nn.Module):
    def __init__(self, state):
        super().__init__()
        self.names = list(state)
        self.ps = nn.ParameterList([nn.Parameter(state[k].clone()) for k in self.names])

    def forward(self, x, ei):
        return pyg_ref.model_forward("sage", dict(zip(self.names, self.ps)), x, ei, layers=2)


def _data():
    return prepare_inputs(synthetic_elliptic(num_nodes=3000, num_edges=4000, seed=8),
                          dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))


def _state():
    g = torch.Generator().manual_seed(1)
    return {"convs.0.lin_l.weight": torch.randn(16, 166, generator=g) * 0.1,
            "convs.0.lin_l.bias": torch.randn(16, generator=g) * 0.1,
            "convs.0.lin_r.weight": torch.randn(16, 166, generator=g) * 0.1,
            "convs.1.lin_l.weight": torch.randn(2, 16, generator=g) * 0.1,
            "convs.1.lin_l.bias": torch.randn(2, generator=g) * 0.1,
            "convs.1.lin_r.weight": torch.randn(2, 16, generator=g) * 0.1}


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = _data()
    parts = gdist.partition_timesteps(data.timestep, data.edge_index, world)
    nodes, ei = gdist.local_subgraph(data.timestep, data.edge_index, parts[rank])
    x, y, tm = data.x[nodes], data.y[nodes], data.train_mask[nodes]
    cw, denom = gdist.global_class_weight_and_count(y, tm, dist)
    model = OracleSAGE(_state())
    bucket = gdist.GradBucket(model)
    logits = model(x, ei)
    loss = torch.nn.functional.cross_entropy(logits[tm], y[tm], weight=cw, reduction="none").sum() / denom
    loss.backward()
    bucket.allreduce_(dist)
    # SyncBN: BN over all ranks' rows == BN over the full tensor
    g = torch.Generator().manual_seed(5)
    full = torch.randn(10, 7, generator=g) * 3 + 1
    rows = full[rank * 5:(rank + 1) * 5].clone().requires_grad_(True)
    bn = gdist.SyncBatchNorm1d(7)
    bn.dist = dist
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 2.0, 7))
        bn.bias.copy_(torch.linspace(-1.0, 1.0, 7))
    out = bn(rows)
    (out * torch.arange(7.0)).sum().backward()
    gw = bn.weight.grad.clone()
    dist.all_reduce(gw)
    if rank == 0:
        torch.save({"grad": bucket.flat.clone(), "bn_out0": out.detach(), "bn_dx0": rows.grad.clone(), "bn_dw": gw,
                    "running_mean": bn.running_mean.clone(), "running_var": bn.running_var.clone()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_partition_covers_and_balances():
    data = _data()
    parts = gdist.partition_timesteps(data.timestep, data.edge_index, 4)
    flat = sorted(t for p in parts for t in p)
    assert flat == sorted(torch.unique(data.timestep).tolist())
    loads = [int(torch.isin(data.timestep, torch.tensor(p)).sum()) for p in parts]
    assert max(loads) / min(loads) < 1.3
    nodes, ei = gdist.local_subgraph(data.timestep, data.edge_index, parts[1])
    sel = torch.isin(data.timestep, torch.tensor(parts[1]))
    keep = sel[data.edge_index[0]]
    assert torch.equal(nodes[ei], data.edge_index[:, keep])  # relabelled edges map back, order kept


def test_two_rank_gloo_matches_full_graph(tmp_path):
    out_path = str(tmp_path / "rank0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out_path), nprocs=2, join=True)
    got = torch.load(out_path, weights_only=True)
    # single-process reference: full graph, mean over all train rows
    data = _data()
    model = OracleSAGE(_state())
    cw = pyg_ref.class_weight(data.y[data.train_mask])
    loss = pyg_ref.ce_loss(model(data.x, data.edge_index)[data.train_mask], data.y[data.train_mask], cw)
    loss.backward()
    ref = torch.cat([p.grad.flatten() for p in model.ps])
    assert float((got["grad"] - ref).norm() / ref.norm()) < 1e-5
    g = torch.Generator().manual_seed(5)
    full = (torch.randn(10, 7, generator=g) * 3 + 1).requires_grad_(True)
    bn = nn.BatchNorm1d(7)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 2.0, 7))
        bn.bias.copy_(torch.linspace(-1.0, 1.0, 7))
    out = bn(full)
    (out * torch.arange(7.0)).sum().backward()
    torch.testing.assert_close(got["bn_out0"], out[:5].detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got["bn_dx0"], full.grad[:5], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got["bn_dw"], bn.weight.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got["running_mean"], bn.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(got["running_var"], bn.running_var, rtol=1e-5, atol=1e-6)
