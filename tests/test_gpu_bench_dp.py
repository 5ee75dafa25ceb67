"""GPU: bench.py's multi-rank path end to end (BASELINE cfg 3's launch form), rehearsed on ONE
GPU: `python -m torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 ...` with gloo in place of RCCL
(MERLIN_DIST_BACKEND) and both ranks pinned to device 0 (MERLIN_BENCH_DEVICE), as a fresh child process.
The run must end by itself (no rank left waiting on a collective its partner never issues), print exactly
one JSON line from rank 0 with n_gpus 2 and the per-rank spread, and report the whole-job rate."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_on_one_gpu_ends_with_one_line():
    env = dict(os.environ, MERLIN_DIST_BACKEND="gloo", MERLIN_BENCH_DEVICE="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--num-envs", "256", "--k-steps", "16", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2 * 256 * 16
    assert out["value"] > 0 and out["scaling"] == "weak"
    ranks = out["ranks"]
    for k in ("rollout_ms", "update_ms", "kernel_ms_per_iter", "distinct_frames_per_sample"):
        assert len(ranks[k]) == 2, (k, ranks)
    # whole-job rate: both ranks' env-steps over the max-over-ranks time
    assert abs(out["value"] - 2 * 2 * 256 * 16 / (out["ms_per_step"] * 2 / 1e3)) / out["value"] < 0.01


def test_bench_eight_ranks_on_one_gpu_ends_with_one_line():
    """Round-4 verdict item 1: bench.py's launch form for cfg 3 at its world size (8 ranks through
    torch.distributed.run, gloo, all on device 0) at a small per-rank shape: one JSON line, 8 entries per rank
    field."""
    env = dict(os.environ, MERLIN_DIST_BACKEND="gloo", MERLIN_BENCH_DEVICE="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
           "--num-envs", "128", "--k-steps", "16", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["global_batch"] == 8 * 128 * 16
    for k in ("rollout_ms", "update_ms", "kernel_ms_per_iter", "distinct_frames_per_sample"):
        assert len(out["ranks"][k]) == 8, (k, out["ranks"])
    assert abs(out["value"] - 2 * 8 * 128 * 16 / (out["ms_per_step"] * 2 / 1e3)) / out["value"] < 0.01


def test_bench_eight_ranks_cfg3_envs_on_one_gpu():
    """Round-5 verdict item 1: bench.py at cfg 3's workload, 8 ranks x 4096 envs x 256 steps (32,768 envs; gloo, all
    on device 0), one timed iteration: one JSON line whose global batch is 8 * 4096 * 256."""
    env = dict(os.environ, MERLIN_DIST_BACKEND="gloo", MERLIN_BENCH_DEVICE="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
           "--num-envs", "4096", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["global_batch"] == 8 * 4096 * 256
    for k in ("rollout_ms", "update_ms", "kernel_ms_per_iter", "distinct_frames_per_sample"):
        assert len(out["ranks"][k]) == 8, (k, out["ranks"])
    assert abs(out["value"] - 8 * 4096 * 256 / (out["ms_per_step"] / 1e3)) / out["value"] < 0.01
