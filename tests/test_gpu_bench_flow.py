"""GPU: the N > 1 bench flow the driver runs on 8 GPUs (torch.distributed.run, one process per rank,
barrier + max-over-ranks timing, one JSON line from rank 0), rehearsed with two ranks on the one GPU of
the box over gloo (DCT3D_BENCH_BACKEND=gloo; RCCL takes one GPU per rank).  Weak scaling (c2: stacks per
rank fixed) and strong scaling (c4: one job split over the ranks); the line carries the job-aggregate
roofline (peak N x 8 TB/s) with per_rank and min_rank_frac."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args):
    env = dict(os.environ, DCT3D_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--no-cpu-baseline",
           "--no-ceiling"] + args
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("config,args,scaling", [
    ("c2", ["--stacks", "4"], "weak"),
    ("c4", ["--config", "c4_encode_4k", "--job-stacks", "4"], "strong"),
])
def test_two_rank_bench_line(config, args, scaling):
    d = _run(args)
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == scaling
    assert d["value"] > 0 and d["ms_per_step"] > 0
    pr = d["per_rank"]
    assert sorted(p["rank"] for p in pr) == [0, 1]
    r = d["roofline"]
    assert r["peak"] == 2 * 8000.0
    assert 0 < r["min_rank_frac"] <= 1 and 0 < r["frac"] <= 1
    cubes = sum(p["cubes"] for p in pr)
    if scaling == "weak":
        assert pr[0]["cubes"] == pr[1]["cubes"] == d["config"]["cubes_per_gpu_step"]
    else:  # the 4-stack job split 2 / 2: the job's cubes once
        assert cubes == 4 * (3840 // 8) * (2160 // 8)
    # value = every rank's cubes per step over the slowest rank's time per step
    assert abs(d["value"] - cubes / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]


def test_rccl_path_single_rank():
    """The RCCL ("nccl") branch of the N > 1 flow -- init_process_group with the rank's device, barrier,
    the per-rank all_gather, the max / sum all-reduces and the --xgmi leg's collectives -- executed for
    real on the box's one GPU as a one-rank job (DCT3D_BENCH_FORCE_DIST=1; RCCL takes one GPU per rank,
    so two ranks on one GPU can only rehearse over gloo, above)."""
    env = dict(os.environ, DCT3D_BENCH_FORCE_DIST="1", DCT3D_BENCH_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--no-cpu-baseline",
           "--no-ceiling", "--stacks", "4", "--xgmi"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert [p["rank"] for p in d["per_rank"]] == [0]
    assert d["xgmi"] is not None and d["xgmi"]["verified"]
