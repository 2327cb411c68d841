"""Headline benchmark: edges/s of full-batch GraphSAGE fwd+bwd on the Elliptic shape (BASELINE.json).

Workload (BASELINE.json configs[1]): configs/sage.yaml with symmetrize_edges=true — 2-layer
SAGE 166->128->2, dropout 0.5, fp32, N=203,769 nodes, E=468,710 symmetrized edges
(synthetic, seeded; the Elliptic CSVs are LFS pointers in the reference).  One step =
the reference's train_epoch (src/train_gnn.py:187-209): forward + masked weighted CE +
backward + clip_grad_norm_(1.0) + Adam; the loss stays on device (no per-step .item()).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--arch A] [--scale weak|strong]

N > 1 (launched by torch.distributed.run, one rank per GPU): ONE global graph is partitioned
by whole timesteps over the ranks (distributed.shard_graph: LPT bin-packing, no cross-timestep
edges, so no halo exchange); gradients are summed with one flat RCCL all-reduce per step, the
loss is normalised by the global train count and BatchNorm (SAGE-ResBN) is SyncBN.
  --scale strong (default) the global graph is the ONE 203,769-node Elliptic graph split N
                 ways — the metric's named workload ("Elliptic 203k/234k/166-feat, 1->8 MI355X"),
                 so the 1/2/4/8 lines form a strong-scaling curve over it.
  --scale weak   the global graph is N Elliptic-shaped blocks (seeds 42..42+N-1, 49 timesteps
                 each), partitioned by (block, timestep): per-GPU work fixed.
value = edges of the global graph x steps / max-over-ranks wall time.

Extra fields: ``roofline`` (dominant libgnnmp kernel: algorithmic bytes per launch / its
HIP-event-timed average duration, on the launch stream) and ``cpu_baseline`` (the oracle —
the PyG-2.5.3 ATen op sequence — timed on this host's cores, rank 0 at N=1 only, bounded
sample; all usable physical cores and a 1-thread figure, with the host's model/sockets/cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "edges/s full-batch SAGE fwd+bwd, Elliptic 203k/234k/166-feat, 1→8 MI355X"

# Workloads.  "sage" is the headline (BASELINE.json configs[1]); the others are the other
# BASELINE configs, run through the same step for the DESIGN.md kernel table.
PRESETS = {
    "sage": dict(cfg=dict(arch="sage", hidden_dim=128, layers=2, dropout=0.5, symmetrize_edges=True,
                          use_time_scalar=True, train_window_k=10),
                 workload="configs/sage.yaml + symmetrize_edges=true: SAGE 2L 166->128->2, dropout 0.5"),
    "gcn": dict(cfg=dict(arch="gcn", hidden_dim=64, layers=2, dropout=0.5, symmetrize_edges=False,
                         use_time_scalar=True, train_window_k=10),
                workload="BASELINE configs[0] preset on the GPU: GCN 2L 166->64->2, dropout 0.5, self loops"),
    "gat": dict(cfg=dict(arch="gat", hidden_dim=64, layers=2, heads=4, dropout=0.5, symmetrize_edges=False,
                         use_time_scalar=True, train_window_k=10),
                workload="BASELINE configs[2] preset: GAT 2L 4 heads 166->4x16->2, dropout 0.5, self loops"),
    "sage_scaled": dict(cfg=dict(arch="sage", hidden_dim=128, layers=3, dropout=0.5, symmetrize_edges=True,
                                 use_time_scalar=True, train_window_k=10),
                        gen=dict(num_nodes=2_000_000, num_edges=4_000_000), dtype="bf16",
                        metric="edges/s full-batch SAGE fwd+bwd, scaled Elliptic 2M/4M/166-feat bf16, 1→8 MI355X",
                        workload="BASELINE configs[4]: synthetic scaled Elliptic 2M nodes / 4M edges (8M "
                                 "symmetrized) / 166 feats, SAGE 3L 166->128->128->2, bf16 storage, f32 accumulate"),
    "sage_resbn": dict(cfg=dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, symmetrize_edges=True,
                                use_time_scalar=False, time_embed_dim=2, time_embed_type="sin",
                                train_window_k=8, use_bn=True, residual=True),
                       workload="configs/rec_k8.yaml: SAGE-ResBN 3L 167->64->64->2, BN, sin time embedding"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--degree", default="powerlaw", choices=["powerlaw", "uniform"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python each step (default: replay the step as captured "
                         "HIP graphs; N>1: forward+backward graph, eager all-reduce, optimizer graph)")
    ap.add_argument("--graph", action="store_true", help=argparse.SUPPRESS)  # the default; kept for old scripts
    ap.add_argument("--arch", default="sage", choices=sorted(PRESETS), help="workload (sage = headline)")
    ap.add_argument("--aten-step", action="store_true",
                    help="loss/clip/Adam with the ATen ops instead of the fused libgnnmp step ops")
    ap.add_argument("--scale", default="strong", choices=["weak", "strong"],
                    help="N>1: strong (default) = the one Elliptic graph split N ways; weak = one Elliptic "
                         "block per rank")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only for multi-rank tests on one device")
    ap.add_argument("--cpu-1t-seconds", type=float, default=8.0, help="1-thread CPU baseline sample budget")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU rehearsal of the N>1 launch (tests): ranks rendezvous, build and shard the global "
                         "graph, time an empty step, reduce and report; no device work")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests: this rank raises
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="before the warm-up: hold the GPU busy this long with a device-to-device copy loop (no "
                         "step work) so the timed steps do not run on clocks still ramping up from the idle "
                         "setup phase; 0 disables")
    ap.add_argument("--rehearse-shard", type=int, default=0, metavar="N",
                    help="diagnostic (N=1 only): time the largest shard of the N-way timestep partition of "
                         "the global graph on this one GPU, without collectives — the per-GPU compute of a "
                         "strong-scaling N-GPU run (the line's value is then that shard's edges/s)")
    ap.add_argument("--separate-ce", action="store_true",
                    help="A/B: launch the masked CE on its own instead of in the output layer's mean")
    ap.add_argument("--step-trace", action="store_true",
                    help="diagnostic: record a HIP event between the timed steps and print each step's GPU "
                         "time (and the host's enqueue time) to stderr")
    return ap.parse_args()


def self_launch(args) -> int:
    """`python bench.py --gpus N` without a launcher (N > 1, WORLD_SIZE unset): start N rank
    processes through torch.distributed.run (127.0.0.1, a free port) as CHILD processes — this
    process never touches the GPU and never exec()s — relay rank 0's JSON line on stdout (the
    ranks' other output goes to stderr) and return non-zero if any rank failed."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / tensor sharing across ranks)
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    line_out = None
    for line in proc.stdout:
        txt = line.strip()
        if txt.startswith("{") and '"metric"' in txt and line_out is None:
            line_out = txt
            print(txt, flush=True)
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and line_out is None:
        sys.stderr.write("bench.py: the ranks exited without a result line\n")
        return 1
    return rc


def make_global_graph(world: int, scale: str, degree: str, cfg, gen=None):
    """The bench's global graph (prepared as train_gnn.main prepares it) and its partition key.

    world 1 / strong: the seeded Elliptic-shaped graph (seed 42).  weak: world such blocks
    (seeds 42 + b) as one disjoint union, partitioned by (block, timestep)."""
    from elliptic_gnn_project_amd.dataset_elliptic import concat_graphs, prepare_inputs, synthetic_elliptic

    nblk = world if (scale == "weak" and world > 1) else 1
    blocks = [prepare_inputs(synthetic_elliptic(degree=degree, seed=42 + b, **(gen or {})), cfg) for b in range(nblk)]
    if nblk == 1:
        return blocks[0], blocks[0].timestep
    g = concat_graphs(blocks)
    return g, g.part_key


def host_cpu_info():
    """(model, sockets, physical cores, usable threads) of this host: /proc/cpuinfo topology and
    the CPU share this process may use (affinity and the cgroup quota)."""
    import os as _os

    model, phys, sockets = "unknown", set(), set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as fh:
            for line in list(fh) + ["\n"]:
                if not line.strip():
                    if "core id" in cur or "physical id" in cur:
                        phys.add((cur.get("physical id", "0"), cur.get("core id", cur.get("processor"))))
                        sockets.add(cur.get("physical id", "0"))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name":
                    model = v.strip()
    except OSError:
        pass
    ncpu = _os.cpu_count() or 1
    cores = len(phys) or ncpu
    usable = len(_os.sched_getaffinity(0)) if hasattr(_os, "sched_getaffinity") else ncpu
    try:  # cgroup v2 quota, e.g. "1600000 100000" -> 16 CPUs
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = min(usable, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return model, max(1, len(sockets)), cores, max(1, min(cores, usable))


def cpu_baseline(data, state, cw, denom, cfg, budget_s: float, budget_1t: float):
    """Oracle (PyG-2.5.3 ATen op sequence) train step on the host CPU, same step definition
    (fwd + masked weighted CE + bwd + clip + Adam), SURVEY §8(d): all usable physical cores
    (torch.set_num_threads) and one thread, each on a bounded sample: the full graph when a
    step fits the budget, else a prefix of whole timesteps (edges/s is per-edge work)."""
    from elliptic_gnn_project_amd.distributed import local_subgraph
    from oracle import pyg_ref

    model, sockets, cores, threads = host_cpu_info()
    kw = dict(layers=cfg["layers"], dropout=cfg["dropout"], training=True, heads=cfg.get("heads", 4),
              time_embed_dim=cfg.get("time_embed_dim", 0), time_embed_type=cfg.get("time_embed_type", "none"))

    def sample(max_edges):
        if data.edge_index.size(1) <= max_edges:
            return data.x, data.edge_index, data.y, data.train_mask, data.timestep, "full graph"
        ts = sorted(torch.unique(data.timestep).tolist())
        e_t = torch.bincount(data.timestep[data.edge_index[1]], minlength=max(ts) + 1)
        keep, acc = [], 0
        for t in ts:
            if keep and acc + int(e_t[t]) > max_edges:
                break
            keep.append(t)
            acc += int(e_t[t])
        nodes, ei = local_subgraph(data.timestep, data.edge_index, keep)
        return (data.x[nodes], ei, data.y[nodes], data.train_mask[nodes], data.timestep[nodes],
                f"timesteps {keep[0]}..{keep[-1]} ({len(keep)} of {len(ts)})")

    def run(nthreads, budget, max_edges):
        torch.set_num_threads(nthreads)
        x, ei, y, m, t_idx, what = sample(max_edges)
        params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in state.items()
                  if v.is_floating_point()}
        opt = torch.optim.Adam(params.values(), lr=0.003, weight_decay=1e-4)

        def step():
            opt.zero_grad(set_to_none=True)
            logits = pyg_ref.model_forward(cfg["arch"], params, x, ei, t_idx=t_idx, **kw)
            loss = torch.nn.functional.cross_entropy(logits[m], y[m], weight=cw, reduction="none").sum() / denom
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
            opt.step()

        step()  # warm-up (allocator, thread pool)
        n, t0 = 0, time.perf_counter()
        while True:
            step()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= 50:
                break
        return ei.size(1) * n / el, 1e3 * el / n, f"{n} steps on {what} (N={x.size(0)}, E={ei.size(1)}), {el:.1f}s"

    t0 = torch.get_num_threads()
    try:
        v, ms, smp = run(threads, budget_s, 2_000_000)
        v1, ms1, smp1 = run(1, budget_1t, 480_000)
    finally:
        torch.set_num_threads(t0)
    return {
        "value": v,
        "unit": "edges/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{smp}; oracle/pyg_ref.py (PyG 2.5.3 ATen op sequence) on CPU, {threads} threads",
        "ms_per_step": ms,
        "one_thread": {"value": v1, "ms_per_step": ms1, "sample": smp1},
        "host_cpu": model, "sockets": sockets, "physical_cores": cores,
        "threads_note": "threads = min(physical cores, this process's CPU share: affinity / cgroup quota)",
    }


MFMA_F32_PEAK_TFS = 157.3  # gfx950 dense fp32 MFMA (= vector fp32) peak, MI355X_MICROARCH.md


def traffic_file(arch):
    """The PMC traffic summary of this workload: profiles/collect.sh (ARCH=<arch>) writes
    traffic.json for the bench command of that arch; the committed copy is profiles/traffic_<arch>.json."""
    return os.path.join(ROOT, "profiles", f"traffic_{arch}.json")


def kernel_pattern(tag):
    """Regex of the libgnnmp kernel a timed launch runs, keyed on its template signature (the tag
    fixes the instantiation's leading parameters): NT k-steps = ceil(K/16), TN k-tiles = ceil(K/32),
    the aggregation mode and its kernel family by width.  None when no family is known."""
    import re

    if tag[0] == "gemm_nt":
        return re.compile(r"gemm_nt_(planes|ws|img16|h2|h2s)_kernel<%d[,>]" % -(-tag[2] // 16))
    if tag[0] == "gemm_tn":
        kt = -(-tag[2] // 32)
        return re.compile(r"gemm_tn_(planes|img16)_kernel<\w+, \w+, %d,|gemm_tn_h2_kernel<%d," % (kt, kt))
    if tag[0] == "agg":
        mode, F = tag[1], tag[3]
        fam = "agg_wave_kernel" if F > 128 else "agg_narrow_lds_kernel" if F <= 4 else "agg_flat(_pieces)?_kernel"
        return re.compile(r"%s<%d," % (fam, mode))
    return None


def measured_traffic(tag, arch):
    """(HBM bytes per launch, source) of the timed kernel from the committed PMC summary of this
    same bench command (profiles/pmc_summary.py over separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes, gfx950-corrected), matched on the kernel's template signature; (None, None)
    when the summary lacks it or the match is ambiguous."""
    pat = kernel_pattern(tag)
    path = traffic_file(arch)
    try:
        with open(path) as fh:
            rows = json.load(fh)["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    cand = [r for r in rows if pat is not None and pat.search(r["kernel"]) and r.get("traffic_bytes")]
    if len(cand) != 1:
        return None, None
    return int(cand[0]["traffic_bytes"]), f"{os.path.relpath(path, ROOT)}: {cand[0]['kernel']}"


BF16_MFMA_PEAK_TFS = 2500.0  # gfx950 dense bf16 MFMA peak (MI355X_MICROARCH.md)


def gemm_floor(tag):
    """(bytes, time at the HBM roofline, time at the MFMA roofline, MFMA peak) of one GEMM launch.

    Algorithmic bytes: NT reads A [M, K] and writes C [M, N]; TN reads A [M, K] and h [M, N]
    (weights, slabs and the 4-wide dz are < 1 %).  MFMA time: 2·M·K·N FLOPs at the peak of the
    arithmetic used — split-bf16 (6 bf16 products per f32 product: 2.5 PF / 6), bf16 storage
    (one product: 2.5 PF) or exact f32 (157.3 TF)."""
    kind, M, K, N, ea, ec, prod = tag
    byts = M * K * ea + M * N * ec
    peak = MFMA_F32_PEAK_TFS if prod <= 0 else BF16_MFMA_PEAK_TFS / prod  # VALU f32 peak = MFMA f32
    return byts, byts / (HBM_PEAK_GBS * 1e9), 2.0 * M * K * N / (peak * 1e12), peak


def roofline(recs, arch="sage"):
    """Dominant libgnnmp kernel (by total HIP-event time) against its roofline.

    Aggregations are HBM-bound: achieved = algorithmic bytes per launch / average duration.
    GEMMs are priced against whichever roofline bounds them (the larger of the HBM time of their
    algorithmic bytes and the MFMA time of their FLOPs at the peak of the arithmetic they use).
    Also reports every timed kernel's share and rooflines for the DESIGN.md breakdown.
    """
    names = {0: "sum", 1: "mean_fwd", 2: "mean_bwd", 3: "gcn", 4: "edge_w"}

    def label(tag):
        if tag[0].startswith("agg"):
            return f"{tag[0]}[{names[tag[1]]},{'csc' if tag[2] else 'csr'},F={tag[3]}]"
        if tag[0].startswith("gat"):
            return f"{tag[0]}[H={tag[1]},C={tag[2]},out={tag[3]}]"
        math = {-1: "valu-f32", 0: "f32", 1: "bf16", 3: "half-pair-f16", 6: "split-bf16"}[tag[6]]
        return f"{tag[0]}[M={tag[1]},K={tag[2]},N={tag[3]},{math}]"

    if not recs:
        return None
    hbm = lambda t: t[0].startswith("agg") or t[0].startswith("gat")  # noqa: E731

    tot = sum(r["ms"] for r in recs.values())
    tag, r = max(recs.items(), key=lambda kv: kv[1]["ms"])
    avg_ms = r["ms"] / r["launches"]
    per = r["amount"] / r["launches"]
    if hbm(tag):
        ach = per / (avg_ms * 1e-3) / 1e9
        out = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
    else:
        byts, t_hbm, t_mfma, peak = gemm_floor(tag)
        if t_hbm >= t_mfma:
            ach = byts / (avg_ms * 1e-3) / 1e9
            out = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes": int(byts)}
        else:
            ach = per / (avg_ms * 1e-3) / 1e12
            out = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                   "frac": round(ach / peak, 4), "traffic": None}
    out["traffic"], src = measured_traffic(tag, arch)
    if out["traffic"] is not None:
        out["traffic_source"] = src
    timed = {}
    for t, v in recs.items():
        us = v["ms"] / v["launches"] * 1e3
        e = {"us_per_launch": round(us, 1), "share": round(v["ms"] / tot, 3)}
        if hbm(t):  # HBM-bound: algorithmic bytes per launch / duration
            gbs = v["amount"] / v["launches"] / (us * 1e-6) / 1e9
            e.update({"hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)})
        else:
            byts, t_hbm, t_mfma, peak = gemm_floor(t)
            e.update({"hbm_frac": round(t_hbm / (us * 1e-6), 4), "mfma_frac": round(t_mfma / (us * 1e-6), 4),
                      "floor_us": round(max(t_hbm, t_mfma) * 1e6, 1)})
        tb = measured_traffic(t, arch)[0]
        if tb is not None:
            e["traffic"] = tb
        timed[label(t)] = e
    out.update({"kernel": label(tag), "avg_us": round(avg_ms * 1e3, 2), "per_launch": int(per),
                "timed_kernels": timed})
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))  # before any GPU call: the parent only launches and relays
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    check = args.launch_check
    if check:
        dev = torch.device("cpu")
        args.dist_backend = "gloo"
    else:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % max(ndev, 1))
        dev = torch.device("cuda", local % max(ndev, 1))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    if rank == args.fail_rank:
        raise RuntimeError(f"--fail-rank {rank}")

    from elliptic_gnn_project_amd import distributed as gdist
    from elliptic_gnn_project_amd.aggregation import KernelTimer
    from elliptic_gnn_project_amd.planes import register_input
    from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, build_model

    preset = PRESETS[args.arch]
    cfg = preset["cfg"]
    full, key = make_global_graph(world, args.scale, args.degree, cfg, preset.get("gen"))
    E_global = full.edge_index.size(1)
    data_cpu = gdist.shard_graph(full, world, rank, key=key) if world > 1 else full
    if args.rehearse_shard > 1 and world == 1:  # diagnostic: one GPU runs the largest shard alone
        parts = gdist.partition_timesteps(key, full.edge_index, args.rehearse_shard)
        e_t = torch.bincount(key[full.edge_index[1]], minlength=int(key.max()) + 1)
        big = max(range(args.rehearse_shard), key=lambda i: int(sum(int(e_t[t]) for t in parts[i])))
        data_cpu = gdist.shard_graph(full, args.rehearse_shard, big, parts=parts, key=key)
        E_global = data_cpu.edge_index.size(1)
    if check:
        return report(args, preset, full, E_global, data_cpu, dist, world, rank, dev, lambda: None, False,
                      None, None, launch_check=True)
    data = data_cpu.to(dev)
    bf16 = preset.get("dtype") == "bf16"
    if bf16:  # bf16 storage of the node features (and, through the fused path, every activation)
        data.x = data.x.to(torch.bfloat16)
    register_input(data.x)  # constant node features: GCN / GAT layer 1 read their split image
    torch.manual_seed(42)  # identical initial weights on every rank
    model = build_model(cfg["arch"], data.x.size(1), cfg).to(dev)
    if dist is not None:
        gdist.convert_sync_batchnorm(model, dist)  # exact full-graph BN (SAGE-ResBN); no-op otherwise
    state0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    # HIP-graph replay of the step (the MI355X stand-in for a tracing compiler).  N=1, and N>1 over
    # RCCL: ONE graph for the whole step, the RCCL collectives (SyncBN statistics forward and
    # backward, the gradient bucket) captured in it.  gloo (CPU collectives, tests only): a
    # forward+backward graph and an optimizer graph with the all-reduce eager between them, and
    # eager launch when SyncBatchNorm's collectives sit inside the forward/backward.
    has_sync_bn = any(isinstance(m, gdist.SyncBatchNorm1d) for m in model.modules())
    rccl = dist is not None and args.dist_backend == "nccl"
    use_graph = not args.eager and not (dist is not None and not rccl and has_sync_bn)
    if args.aten_step:
        opt = torch.optim.Adam(model.parameters(), lr=0.003, weight_decay=1e-4, fused=True, capturable=use_graph)
    else:  # clip_grad_norm_(1.0) + Adam fused (train_ops.ClipAdam: 2 launches, device step counter)
        from elliptic_gnn_project_amd.train_ops import ClipAdam
        opt = ClipAdam(model.parameters(), lr=0.003, weight_decay=1e-4, max_norm=1.0)
    # class weights and the loss divisor from the GLOBAL train labels (src/train_gnn.py:175,362-365)
    cw, denom = gdist.global_class_weight_and_count(full.y, full.train_mask, None)
    loss_fn = _make_loss_fn({}, cw, model, 1, 34)
    bucket = gdist.GradBucket(model) if dist is not None else None
    tidx = data.train_idx
    t_idx = data.timestep if cfg.get("time_embed_dim", 0) > 0 else None
    ytr = data.y.index_select(0, tidx)

    from elliptic_gnn_project_amd.train_ops import unit_gradient

    def fwd_bwd():
        model.train()
        opt.zero_grad(set_to_none=bucket is None)
        if args.aten_step or args.separate_ce:
            logits = model(data.x, data.edge_index, t_idx)
        else:  # the fused SAGE output layer computes the step's masked CE in its mean's launch
            with loss_fn.target(data.y, data.train_mask, denom):
                logits = model(data.x, data.edge_index, t_idx)
        if args.aten_step:
            loss = loss_fn(logits.index_select(0, tidx), ytr, denom=denom)
        else:  # the same masked weighted CE, one fused kernel (fwd + dlogits)
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
        loss.backward(unit_gradient(loss.device))  # = loss.backward(), without the per-step fill
        return loss.detach()  # drop the autograd graph now (a live one would pin this step's streams)

    def allreduce():
        bucket.allreduce_(dist)

    def opt_step():
        if args.aten_step:
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()

    def eager_step():
        loss = fwd_bwd()
        if bucket is not None:
            allreduce()
        opt_step()
        return loss

    if use_graph:
        from elliptic_gnn_project_amd.train_gnn import CapturedStep
        # defer_loss: the loss is read only after the step (returned, never used inside it)
        if bucket is None or rccl:
            step = CapturedStep(eager_step, defer_loss=True)
        else:
            step = CapturedStep(fwd_bwd, mid=allreduce, tail=opt_step, defer_loss=True)
    else:
        step = eager_step

    def extras(value):
        """roofline (instrumented eager steps) and the CPU baseline, after the timed region."""
        roof = None
        if not args.no_roofline:
            KernelTimer.start()
            for _ in range(5):
                # hold the stream in a spin kernel while Python enqueues the whole step, so each event
                # pair brackets back-to-back GPU work only (an idle stream would count the host's
                # launch latency between an event and its kernel as kernel time)
                torch.cuda._sleep(50_000_000)
                eager_step()
            recs = KernelTimer.stop()
            roof = roofline(recs, args.arch)
            if roof is not None:  # an event pair also spans its kernel's launch boundary (~1.5-3 us)
                roof["timing_note"] = ("HIP-event brackets behind a busy stream; each includes its kernel's launch "
                                       "boundary (~1.5-3 us), which rocprofv3's kernel durations exclude")

        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(data_cpu, state0, cw.cpu(), denom, cfg, args.cpu_seconds, args.cpu_1t_seconds)
            cpu["speedup_gpu_over_cpu"] = round(value / cpu["value"], 1)
        return roof, cpu

    launch = ("eager" if not use_graph else "hip-graph replay of the whole step" if bucket is None
              else "hip-graph replay of the whole step, RCCL collectives captured" if rccl
              else "hip-graph replay of fwd+bwd and of the optimizer, eager all-reduce between")
    return report(args, preset, full, E_global, data, dist, world, rank, dev, step, bf16, extras, launch)


def settle(dev, ms: float):
    """Bring the GPU out of its idle clock state before the warm-up: the setup phase (graph build,
    capture) leaves it idle for seconds, and the first ~30 replayed steps then run 5-10 % slow
    while the clocks ramp (profiles/r22_timing.txt: per-step events 0.34-0.37 ms for the first
    15 steps, 0.32 ms after).  A device-to-device copy loop over two 256 MiB scratch buffers — no
    model, graph or optimizer state is touched, nothing of the step runs — for ``ms`` of wall
    time.  Returns the description the JSON line carries, or None."""
    if dev.type != "cuda" or ms <= 0:
        return None
    a = torch.empty(64 << 20, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.zero_()
    t0 = time.perf_counter()
    n = 0
    while 1e3 * (time.perf_counter() - t0) < ms:
        for _ in range(8):
            b.copy_(a)
            a.copy_(b)
        n += 16
        torch.cuda.synchronize(dev)
    del a, b
    return f"{n} device copies of 256 MiB ({1e3 * (time.perf_counter() - t0):.0f} ms) before the warm-up: clock ramp, no step work"


def report(args, preset, full, E_global, data, dist, world, rank, dev, step, bf16, extras, launch,
           launch_check=False):
    """Warm-up, the timed region (barrier + synchronize on both sides, max over ranks), and rank
    0's JSON line."""
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    settled = settle(dev, args.settle_ms)
    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    sync()
    trace = args.step_trace and dev.type == "cuda"
    evs, host = [], []
    if trace:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        if trace:
            evs[i].record()
            host.append(time.perf_counter())
        step()
    if trace:
        evs[-1].record()
    sync()
    if trace:
        gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
        hst = [1e3 * (b - a) for a, b in zip(host, host[1:])]
        sys.stderr.write("step-trace gpu ms: " + " ".join(f"{g:.4f}" for g in gpu) + "\n")
        sys.stderr.write("step-trace host enqueue ms: " + " ".join(f"{h:.4f}" for h in hst) + "\n")
        sys.stderr.write(f"step-trace first-event lag ms: {1e3 * (host[0] - t0):.4f}\n")
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    n_local = torch.tensor([float(data.x.size(0)), float(data.edge_index.size(1))], dtype=torch.float64)
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
        nl = n_local.to(t.device)
        dist.all_reduce(nl, op=dist.ReduceOp.MAX)
        n_local = nl.cpu()
    value = E_global * args.steps / el
    roof, cpu = extras(value) if extras is not None else (None, None)
    if rank == 0:
        # the scale mode the N-GPU lines of the same command use (at N = 1 both modes run the one
        # Elliptic graph): the driver's 1 -> 8 curve reads one label across its points
        scaling = args.scale
        line = {
            "metric": preset.get("metric") or (METRIC if args.arch == "sage" else METRIC.replace("SAGE", args.arch.upper())),
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * el / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "bf16" if bf16 else "f32",
            "data": f"synthetic Elliptic-shape ({args.degree} in-degree, seeded)",
            "config": {
                "workload": preset["workload"] + ", full-batch train step (fwd+masked CE+bwd+clip+Adam)",
                "global_nodes": full.num_nodes, "global_edges": E_global, "feats": data.x.size(1),
                "max_nodes_per_gpu": int(n_local[0]), "max_edges_per_gpu": int(n_local[1]),
                "parallelism": f"dp{world} timestep-partitioned ({args.scale})" if world > 1 else "single",
                "collective": f"{args.dist_backend} all-reduce of one flat fp32 gradient bucket per step" if world > 1 else None,
                "launch": launch,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if settled:
            line["settle"] = settled
        if args.rehearse_shard > 1 and world == 1:
            line["rehearsal"] = (f"largest shard of a {args.rehearse_shard}-way timestep partition on one GPU, "
                                 "no collectives (diagnostic, not the metric's workload)")
        if launch_check:
            line["launch_check"] = "CPU rehearsal of the launch: empty step, no device work (not a measurement)"
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
