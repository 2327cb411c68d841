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
        torch.save({"grad": bucket.flat_in_param_order(), "bn_out0": out.detach(), "bn_dx0": rows.grad.clone(), "bn_dw": gw,
                    "running_mean": bn.running_mean.clone(), "running_var": bn.running_var.clone()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


class OracleResBN(nn.Module):
    """SAGEResBNNet (src/models/gnn.py:82-194) with the oracle's SAGE conv and REAL BatchNorm1d
    modules (swapped for SyncBatchNorm1d on the ranks), sin time embedding, fixed dropout masks
    indexed by GLOBAL node id (so the partitioned and full-graph runs draw the same mask)."""

    def __init__(self, state, hidden, layers, masks):
        super().__init__()
        self.conv_names = [k for k in state if k.startswith(("convs.", "res_projs."))]
        self.ps = nn.ParameterList([nn.Parameter(state[k].clone()) for k in self.conv_names])
        self.bns = nn.ModuleList(nn.BatchNorm1d(hidden) for _ in range(layers - 1))
        for i, bn in enumerate(self.bns):
            with torch.no_grad():
                bn.weight.copy_(state[f"bns.{i}.weight"])
                bn.bias.copy_(state[f"bns.{i}.bias"])
        self.layers = layers
        self.masks = masks  # [layers-1] x [N_global, hidden] keep masks

    def forward(self, x, ei, t_idx, nodes, p=0.2):
        prm = dict(zip(self.conv_names, self.ps))
        h = torch.cat([x, pyg_ref.sinusoid(t_idx, 2, 49)], dim=1)
        for i in range(self.layers - 1):
            h_in = h
            z = pyg_ref.sage_conv(h, ei, prm[f"convs.{i}.lin_l.weight"], prm[f"convs.{i}.lin_l.bias"],
                                  prm[f"convs.{i}.lin_r.weight"])
            z = self.bns[i](z)
            z = torch.relu(z) * (self.masks[i][nodes] / (1 - p))
            rp = prm.get(f"res_projs.{i}.weight")
            h = z + (h_in @ rp.t() if rp is not None else h_in)
        i = self.layers - 1
        return pyg_ref.sage_conv(h, ei, prm[f"convs.{i}.lin_l.weight"], prm[f"convs.{i}.lin_l.bias"],
                                 prm[f"convs.{i}.lin_r.weight"])


_RB_HID, _RB_L = 16, 3


def _rb_data():
    return prepare_inputs(synthetic_elliptic(num_nodes=3000, num_edges=4000, seed=11),
                          dict(use_time_scalar=False, symmetrize_edges=True, train_window_k=8, time_embed_dim=2))


def _rb_state():
    g = torch.Generator().manual_seed(3)
    fi = 165 + 2
    s = {}
    dims = [(fi, _RB_HID), (_RB_HID, _RB_HID), (_RB_HID, 2)]
    for i, (a, b) in enumerate(dims):
        s[f"convs.{i}.lin_l.weight"] = torch.randn(b, a, generator=g) * 0.1
        s[f"convs.{i}.lin_l.bias"] = torch.randn(b, generator=g) * 0.1
        s[f"convs.{i}.lin_r.weight"] = torch.randn(b, a, generator=g) * 0.1
    for i in range(_RB_L - 1):
        s[f"bns.{i}.weight"] = 1.0 + 0.1 * torch.randn(_RB_HID, generator=g)
        s[f"bns.{i}.bias"] = 0.1 * torch.randn(_RB_HID, generator=g)
    s["res_projs.0.weight"] = torch.randn(_RB_HID, fi, generator=g) * 0.1
    return s


def _rb_masks(n):
    g = torch.Generator().manual_seed(9)
    return [(torch.rand(n, _RB_HID, generator=g) >= 0.2).float() for _ in range(_RB_L - 1)]


def _rb_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _rb_data()
    sh = gdist.shard_graph(full, world, rank)
    cw, denom = gdist.global_class_weight_and_count(sh.y, sh.train_mask, dist)
    model = OracleResBN(_rb_state(), _RB_HID, _RB_L, _rb_masks(full.num_nodes))
    gdist.convert_sync_batchnorm(model, dist)
    bucket = gdist.GradBucket(model)
    logits = model(sh.x, sh.edge_index, sh.timestep, sh.nodes)
    tm = sh.train_mask
    loss = torch.nn.functional.cross_entropy(logits[tm], sh.y[tm], weight=cw, reduction="none").sum() / denom
    loss.backward()
    bucket.allreduce_(dist)
    glog = gdist.gather_rows(logits.detach(), sh.nodes, full.num_nodes, dist)
    if rank == 0:
        torch.save({"grad": bucket.flat_in_param_order(), "logits": glog, "denom": denom,
                    "rm": [bn.running_mean.clone() for bn in model.bns],
                    "rv": [bn.running_var.clone() for bn in model.bns],
                    "types": [type(bn).__name__ for bn in model.bns]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _rb_overlap_worker(rank, world, port, out_path):
    """As _rb_worker, three backwards through an overlapped GradBucket: the later layers'
    gradients (convs.2, convs.1, the BN affines) in the early slice, all-reduced from their
    post-accumulate hooks while layer 0's backward still runs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _rb_data()
    sh = gdist.shard_graph(full, world, rank)
    cw, denom = gdist.global_class_weight_and_count(sh.y, sh.train_mask, dist)
    model = OracleResBN(_rb_state(), _RB_HID, _RB_L, _rb_masks(full.num_nodes))
    gdist.convert_sync_batchnorm(model, dist)
    names = [k for k, _ in model.named_parameters()]
    early = [k for k in names if k.startswith("bns.")] + \
        [f"ps.{i}" for i, k in enumerate(model.conv_names) if not k.startswith(("convs.0.", "res_projs."))]
    bucket = gdist.GradBucket(model, early=early)
    issued = []
    for it in range(3):
        for p in model.parameters():
            p.grad.zero_()
        for bn in model.bns:  # the same BN running-stat state each pass
            bn.reset_running_stats()
        logits = model(sh.x, sh.edge_index, sh.timestep, sh.nodes)
        tm = sh.train_mask
        loss = torch.nn.functional.cross_entropy(logits[tm], sh.y[tm], weight=cw, reduction="none").sum() / denom
        loss.backward()
        issued.append(bucket._work is not None)
        bucket.allreduce_(dist)
    if rank == 0:
        torch.save({"grad": bucket.flat_in_param_order(), "issued": issued, "n_early": bucket.n_early,
                    "order": bucket.order}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_overlapped_bucket_matches_full_graph(tmp_path):
    """the gradient all-reduce overlapped with the backward (two slices, the early
    one issued from the hooks) still gives the full-graph gradient on every step."""
    out_path = str(tmp_path / "rbo0.pt")
    mp.spawn(_rb_overlap_worker, args=(2, _free_port(), out_path), nprocs=2, join=True)
    got = torch.load(out_path, weights_only=True)
    assert got["issued"] == [False, True, True]  # step 0 lays the buffer out, then the hooks issue
    assert 0 < got["n_early"] < len(got["order"])
    full = _rb_data()
    model = OracleResBN(_rb_state(), _RB_HID, _RB_L, _rb_masks(full.num_nodes))
    nodes = torch.arange(full.num_nodes)
    logits = model(full.x, full.edge_index, full.timestep, nodes)
    tm = full.train_mask
    pyg_ref.ce_loss(logits[tm], full.y[tm], pyg_ref.class_weight(full.y[tm])).backward()
    ref = torch.cat([p.grad.flatten() for p in model.parameters()])
    assert float((got["grad"] - ref).norm() / ref.norm()) < 1e-5


def test_two_rank_sage_resbn_partitioned_matches_full_graph(tmp_path):
    """rec_k8's claim: SAGE-ResBN with SyncBN inside the model, timestep-partitioned
    over 2 ranks with the global train divisor, gives the full-graph logits, gradients (every
    parameter: convs, BN affine, residual projection) and BN running statistics."""
    out_path = str(tmp_path / "rb0.pt")
    mp.spawn(_rb_worker, args=(2, _free_port(), out_path), nprocs=2, join=True)
    got = torch.load(out_path, weights_only=True)
    assert got["types"] == ["SyncBatchNorm1d"] * (_RB_L - 1)
    full = _rb_data()
    model = OracleResBN(_rb_state(), _RB_HID, _RB_L, _rb_masks(full.num_nodes))
    nodes = torch.arange(full.num_nodes)
    logits = model(full.x, full.edge_index, full.timestep, nodes)
    tm = full.train_mask
    assert got["denom"] == int(tm.sum())
    cw = pyg_ref.class_weight(full.y[tm])
    pyg_ref.ce_loss(logits[tm], full.y[tm], cw).backward()
    torch.testing.assert_close(got["logits"], logits.detach(), rtol=1e-5, atol=1e-5)
    ref = torch.cat([p.grad.flatten() for p in model.parameters()])
    assert float((got["grad"] - ref).norm() / ref.norm()) < 1e-5
    for i, bn in enumerate(model.bns):
        torch.testing.assert_close(got["rm"][i], bn.running_mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(got["rv"][i], bn.running_var, rtol=1e-5, atol=1e-6)


def test_sync_bn_large_mean_matches_batchnorm():
    """Merged centred statistics: features with mean ~1e3 and std ~1 keep fp32 precision
    (the former E[x²] − mean² form lost it); single process, world 1 merge path."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(4096, 8, generator=g) + 1000.0
    mean, var, n = gdist.global_batch_stats(x, None)
    xd = x.double()
    torch.testing.assert_close(mean.double(), xd.mean(0), rtol=1e-7, atol=1e-5)
    torch.testing.assert_close(var.double(), xd.var(0, unbiased=False), rtol=1e-4, atol=1e-5)
    assert float(n) == 4096.0


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
