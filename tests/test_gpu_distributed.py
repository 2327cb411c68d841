"""GPU: the timestep-partitioned path of BASELINE configs[3] (rec_k8, SAGE-ResBN) on libgnnmp.

* one rank's shard: the HIP SAGE-ResBN (sin time embedding, BatchNorm, residual projection)
  on ``shard_graph``'s local subgraph against the oracle on the same subgraph — logits and
  every parameter gradient;
* two ranks on this one device (gloo carries the collectives; RCCL refuses two ranks on one
  GPU): the partitioned HIP step — SyncBatchNorm1d inside the model, the global train divisor,
  one flat gradient all-reduce — against the single-process full-graph HIP step: logits,
  gradients and BN running statistics;
* bench.py's multi-rank code path (2 ranks, gloo, one device) and train_gnn.main's
  (world_size 2, partition timestep) end to end.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from oracle import pyg_ref

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.0, use_bn=True, residual=True,
           time_embed_dim=2, time_embed_type="sin", use_time_scalar=False, symmetrize_edges=True, train_window_k=8)


def rel_l2(a, b, floor=1e-7):
    """Relative L2 with an absolute floor (as test_gpu_parity): a conv bias feeding BatchNorm has
    an exactly-zero gradient, so both sides are rounding noise at the 1e-9 level there."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), floor / 1e-5))


def _data(n=6000, e=9000, seed=31):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    return prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed), CFG)


def _model(device):
    from elliptic_gnn_project_amd.train_gnn import build_model

    torch.manual_seed(17)
    m = build_model("sage_resbn", 165, CFG).to(device)
    with torch.no_grad():  # non-trivial BN affine parameters
        for bn in m.bns:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    return m


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_subgraph_matches_oracle(device):
    from elliptic_gnn_project_amd import distributed as gdist

    full = _data()
    sh = gdist.shard_graph(full, 2, 1)
    assert 0 < sh.x.size(0) < full.x.size(0)
    model = _model(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    logits = model(sh.x.to(device), sh.edge_index.to(device), sh.timestep.to(device))
    tm = sh.train_mask
    cw = pyg_ref.class_weight(sh.y[tm])
    pyg_ref.ce_loss(logits[tm.to(device)], sh.y[tm].to(device), cw.to(device)).backward()
    kw = dict(layers=3, training=True, t_idx=sh.timestep, time_embed_dim=2, time_embed_type="sin")
    ref = pyg_ref.model_forward("sage_resbn", params, sh.x, sh.edge_index, **kw)
    torch.testing.assert_close(logits.detach().cpu(), ref, rtol=1e-5, atol=1e-5)
    _, grads = pyg_ref.train_step_grads("sage_resbn", params, sh.x, sh.edge_index, sh.y, tm, cw, **kw)
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 1e-5, k


def _rank_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from elliptic_gnn_project_amd import distributed as gdist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _data()
    sh = gdist.shard_graph(full, world, rank).to(dev)
    model = _model(dev)
    gdist.convert_sync_batchnorm(model, dist)
    bucket = gdist.GradBucket(model)
    cw, denom = gdist.global_class_weight_and_count(full.y, full.train_mask, None)
    model.train()
    logits = model(sh.x, sh.edge_index, sh.timestep)
    tm = sh.train_mask
    loss = torch.nn.functional.cross_entropy(logits[tm], sh.y[tm], weight=cw.to(dev), reduction="none").sum() / denom
    loss.backward()
    bucket.allreduce_(dist)
    glog = gdist.gather_rows(logits.detach(), sh.nodes, full.num_nodes, dist)
    if rank == 0:
        torch.save({"grad": bucket.flat_in_param_order().cpu(), "logits": glog.cpu(),
                    "rm": [bn.running_mean.cpu() for bn in model.bns],
                    "rv": [bn.running_var.cpu() for bn in model.bns]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_partitioned_hip_step_matches_full_graph(device, tmp_path):
    out_path = str(tmp_path / "r0.pt")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, out_path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = torch.load(out_path, weights_only=True)
    full = _data()
    model = _model(device)
    model.train()
    d = full.to(device)
    logits = model(d.x, d.edge_index, d.timestep)
    tm = d.train_mask
    cw = pyg_ref.class_weight(full.y[full.train_mask]).to(device)
    pyg_ref.ce_loss(logits[tm], d.y[tm], cw).backward()
    torch.testing.assert_close(got["logits"], logits.detach().cpu(), rtol=1e-5, atol=1e-5)
    ref = torch.cat([p.grad.flatten() for p in model.parameters()]).cpu()
    assert rel_l2(got["grad"], ref) < 1e-5
    for i, bn in enumerate(model.bns):
        torch.testing.assert_close(got["rm"][i], bn.running_mean.cpu(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(got["rv"][i], bn.running_var.cpu(), rtol=1e-5, atol=1e-6)


def _torchrun(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("arch", ["sage_resbn", "sage"])
@pytest.mark.parametrize("scale", ["weak", "strong"])
def test_bench_two_rank_path(device, scale, arch):
    """bench.py's N > 1 path (two ranks on the one card, gloo): configs[3] and the headline preset —
    under strong scaling each rank's half of the graph runs the shard-sized schedule (the TN with
    the folded CSC sum, ABI 26)."""
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                   "--no-roofline", "--dist-backend", "gloo", "--arch", arch, "--scale", scale])
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["scaling"] == scale
    assert out["config"]["global_edges"] == (2 if scale == "weak" else 1) * 468_710
    assert out["config"]["parallelism"].startswith("dp2 timestep-partitioned")


def test_train_main_two_ranks(device, tmp_path):
    import yaml

    cfg = dict(CFG, run_name="dp2", output_root=str(tmp_path), max_epochs=3, patience=5, lr=5e-4,
               weight_decay=5e-5, grad_clip=1.0, amp=False, calibrate_temperature=True, ablate_hubs_frac=0.01,
               world_size=2, partition="timestep", dist_backend="gloo",
               synthetic=dict(num_nodes=6000, num_edges=9000, seed=31))
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = _torchrun(["-m", "elliptic_gnn_project_amd.train_gnn", "--config", str(p)])
    assert r.returncode == 0, r.stderr[-3000:]
    out = tmp_path / "gnn" / "dp2"
    m = json.loads((out / "metrics.json").read_text())
    for k in ("pr_auc_illicit", "test_pr_auc_by_time", "pr_auc_last1", "best_val_pr_auc"):
        assert k in m
    h = json.loads((out / "metrics_hub_removed.json").read_text())
    assert h["n_hubs"] == 60 and h["n_edges_remaining"] < 18000
    rows = (out / "training_log.csv").read_text().strip().splitlines()
    assert rows[0] == "epoch,train_loss,val_pr_auc" and len(rows) == 4


def _nccl_capture_worker(port, out_path):
    """World size 1 over RCCL on this device: the SAGE-ResBN step with SyncBatchNorm1d (K12's
    statistics all-reduce forward, the (Σdy, Σdy·x̂) all-reduce backward) and the flat gradient
    bucket, 5 eager steps vs 3 eager warm-up steps + capture + 2 replays of ONE graph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from elliptic_gnn_project_amd import distributed as gdist
    from elliptic_gnn_project_amd.train_gnn import CapturedStep, _make_loss_fn
    from elliptic_gnn_project_amd.train_ops import ClipAdam

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    full = _data()
    d = full.to(dev)
    cw, denom = gdist.global_class_weight_and_count(full.y, full.train_mask, None)
    states = []
    for captured in (False, True):
        model = _model(dev)
        gdist.convert_sync_batchnorm(model, dist)
        assert sum(isinstance(m, gdist.SyncBatchNorm1d) for m in model.modules()) == 2
        bucket = gdist.GradBucket(model)
        opt = ClipAdam(model.parameters(), lr=0.01, weight_decay=1e-4, max_norm=1.0)
        loss_fn = _make_loss_fn({}, cw.to(dev), model, 1, 34)

        def step():
            model.train()
            opt.zero_grad(set_to_none=False)
            loss = loss_fn.full(model(d.x, d.edge_index, d.timestep), d.y, d.train_mask, denom=denom)
            loss.backward()
            bucket.allreduce_(dist)
            opt.step()
            return loss.detach()

        if captured:
            cs = CapturedStep(step, warmup=3)
            cs()
            cs()
        else:
            for _ in range(5):
                step()
        torch.cuda.synchronize()
        states.append({k: v.detach().cpu().clone() for k, v in model.state_dict().items()})
    torch.save(states, out_path)
    dist.destroy_process_group()


def test_rccl_captured_step_matches_eager(device, tmp_path):
    """The N>1 bench step over RCCL is one HIP graph with its collectives captured (bench.py,
    train_gnn.CapturedStep): replaying it leaves exactly the parameters, BN running statistics
    and counters of the eager steps (bitwise)."""
    out_path = str(tmp_path / "nccl.pt")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_nccl_capture_worker, args=(_free_port(), out_path))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    eager, graph = torch.load(out_path, weights_only=True)
    assert eager.keys() == graph.keys()
    for k in eager:
        assert torch.equal(eager[k], graph[k]), k
