"""bench.py --gpus N launches its own ranks when no launcher set WORLD_SIZE:
the parent starts torch.distributed.run as a child, touches no device, relays rank 0's ONE JSON
line and propagates a failing rank's exit status."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, timeout=400):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _one_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_self_launch_two_ranks_cpu_rehearsal():
    """The default N > 1 line measures the metric's own workload: the ONE 203,769-node Elliptic
    graph split over the ranks (strong scaling)."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["value"] > 0
    assert line["scaling"] == "strong"
    assert line["config"]["parallelism"] == "dp2 timestep-partitioned (strong)"
    assert line["config"]["global_nodes"] == 203_769 and line["config"]["global_edges"] == 468_710
    assert line["config"]["max_nodes_per_gpu"] < 203_769  # each rank holds about half
    assert line["launch_check"]


def test_self_launch_two_ranks_weak_scaling_option():
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--launch-check",
              "--scale", "weak"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    assert line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "dp2 timestep-partitioned (weak)"
    assert line["config"]["global_nodes"] > 2 * 200_000  # two Elliptic-shaped blocks
    assert line["launch_check"]


def test_self_launch_propagates_rank_failure():
    # rank 1 raises after the rendezvous: the parent must exit non-zero with no result line
    r = _run(["--gpus", "2", "--launch-check", "--steps", "1", "--fail-rank", "1"])
    assert r.returncode != 0
    assert r.stdout.strip() == ""


@pytest.mark.gpu
def test_self_launch_two_ranks_on_the_gpu():
    """The real step on one device with two gloo ranks (RCCL needs one GPU per rank; the driver's
    8-GPU node runs the nccl form): one JSON line with n_gpus 2 and a measured value."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--no-roofline"], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    assert line["n_gpus"] == 2 and line["value"] > 0 and "launch_check" not in line
