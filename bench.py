#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X 3D-DCT hot path.

BASELINE.json metric: 8x8x8 cubes/s (encode DCT+quant) on 1080p x 8-frame stacks; % HBM roofline.
Workload (config 2): 1920x1080 grayscale, 8-frame stacks, forward 3D DCT + quantise, B = 128
device-resident stacks per step per GPU (4,147,200 cubes).  One step = one
dct3d_encode_stacks_dev call over the batch (8x8x8: ONE launch of the fused encode kernel, which
replays its rare uncertified coefficients itself), inputs resident in HBM (synthetic, generated on
device).  N GPUs: one process per GPU (torch.distributed.run), each encodes its own 128 stacks (weak
scaling, no data-path collective); config c4_encode_4k is one job of 64 4K stacks split over the
ranks (strong scaling).  Barrier + synchronize bracket the K timed steps, the time is the max over
ranks.

Prints ONE JSON line (rank 0) with `roofline` (algorithmic bytes of a step / device time per step,
from HIP events on the bench stream around the timed region; the dominant kernel's own rate as
kernel_only_*), `ceiling` (this device's rates for the same traffic: memory-only twins, probes) and
`cpu_baseline` (the Java-algorithm restatement, oracle/, timed on the host cores at N=1).
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (width, height, block_depth, stacks per GPU, direction); stacks None = a fixed job split
    # over the ranks (JOB_STACKS, strong scaling)
    # BASELINE config 1: the reference's own CPU-runnable case, the Java Encoder path (Encoder.java:47-89)
    # on one 64x64 8-frame stack, no GPU: timed through its restatement (bench_c1, n_gpus 0)
    "c1_java_cpu_64x64": (64, 64, 8, 1, "java_cpu"),
    "c2_encode_1080p": (1920, 1080, 8, 128, "encode"),
    "c3_decode_1080p": (1920, 1080, 8, 128, "decode"),
    # BASELINE config 4: ONE job of 64 4K stacks, each rank encodes shard(64, N, rank) of them
    # (contiguous ranges, Transform.java:88-104's per-cube independence; no data-path collective)
    "c4_encode_4k": (3840, 2160, 8, None, "encode"),
    "c5_encode_1080p_d4": (1920, 1080, 4, 128, "encode"),
    "c6_decode_1080p_d4": (1920, 1080, 4, 128, "decode"),
    # encode to the Exp-Golomb stream: DCT + quantise + diagonal order + EG per step
    "c7_encode_eg_1080p": (1920, 1080, 8, 128, "encode_eg"),
    # decode from the Exp-Golomb stream: EG decode + dequantise + IDCT per step
    "c8_decode_eg_1080p": (1920, 1080, 8, 128, "decode_eg"),
    # drop-in (A), the reference's own device block (encoder.c:209-254 / decoder.c:246-292): float
    # cube-major in -> float cube-major out, DCT / IDCT + clamp, fp64 internal
    "c9_forward_f32_1080p": (1920, 1080, 8, 128, "forward_f32"),
    "c10_inverse_f32_1080p": (1920, 1080, 8, 128, "inverse_f32"),
}

# what one step computes, per direction (the headline metric is BASELINE.json's, config c2)
WHAT = {
    "java_cpu": "forward 3D DCT + quantise, the Java CPU Encoder path (restated), no GPU",
    "encode": "forward 3D DCT + quantise",
    "decode": "dequantise + inverse 3D DCT",
    "encode_eg": "forward 3D DCT + quantise + diagonal order + Exp-Golomb stream",
    "decode_eg": "Exp-Golomb decode + dequantise + inverse 3D DCT",
    "forward_f32": "drop-in (A) forward 3D DCT, f32 cube-major in/out",
    "inverse_f32": "drop-in (A) inverse 3D DCT + clamp, f32 cube-major in/out",
}
JOB_STACKS = {"c4_encode_4k": 64}
HEADLINE_METRIC = "8×8×8 cubes/s (encode DCT+quant) on 1080p×8-frame stacks; % HBM roofline at 1/2/4/8 GPUs"


def metric_name(direction: str, depth: int, width: int = 1920, height: int = 1080) -> str:
    """BASELINE.json's metric for the 1080p encode at depth 8 (the headline, config 2); the same form,
    naming what is timed, for the other configs (they are parity / coverage lines, not the headline)."""
    if direction == "encode" and depth == 8 and (width, height) == (1920, 1080):
        return HEADLINE_METRIC
    unit = "8×8×8" if depth == 8 else "8×8×4"
    size = "1080p" if (width, height) == (1920, 1080) else f"{width}×{height}"
    tail = "" if direction == "java_cpu" else "; % HBM roofline"
    return f"{unit} cubes/s ({WHAT[direction]}) on {size}×{depth}-frame stacks{tail}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2_encode_1080p", choices=sorted(CONFIGS))
    ap.add_argument("--stacks", type=int, default=None, help="override stacks per GPU (weak scaling)")
    ap.add_argument("--job-stacks", type=int, default=None,
                    help="strong scaling: one job of this many stacks split over the ranks (sharding.shard); "
                         "the default for c4_encode_4k is 64")
    ap.add_argument("--kind", default="ramp", choices=["ramp", "uniform"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true")
    ap.add_argument("--xgmi", action="store_true",
                    help="N>1, encode configs: also time the optional host-of-record distribution (SURVEY.md §8e): "
                         "rank 0 scatters every rank's u8 stacks and gathers the int32 cubes back over RCCL p2p "
                         "(reported under 'xgmi', never part of 'value')")
    ap.add_argument("--settle-ms", type=float, default=4000.0,
                    help="untimed steps for at least this much wall time before the warmup steps (the GPU's "
                         "power-management transient, ~30 ms of load; 4 s so that a sampler of GPU activity "
                         "polling every few seconds sees the run: 150 vs 3000 ms measured the same c2 "
                         "line, profiles/r05/settle/); 0 = off")
    ap.add_argument("--kernel-events", default="separate", choices=["separate", "timed"],
                    help="where the library's per-launch events (kernel_ms) run: a separate pass after the timed "
                         "region (default) or inside it (adds their device cost to every step)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B knob: a context option (DCT3D_OPT_<NAME>, dct3d_ctx_set_option) set before the run; "
                         "options change how results are reached, never the results")
    ap.add_argument("--eg-two-step", action="store_true",
                    help="c7 / c8: the int32 cube-major intermediate plus the stand-alone Exp-Golomb stage (A/B)")
    return ap.parse_args()


def rank_stacks(config: str, stacks_override, job_override, world: int, rank: int):
    """This rank's work: (first stack, stacks, job stacks or None, scaling).  Strong scaling (a job
    config such as c4_encode_4k, or --job-stacks): one job of J stacks, rank r encodes its contiguous
    shard sharding.shard(J, world, r).  Weak scaling: every rank encodes its own `stacks` stacks, rank r
    the r-th slice of one long synthetic video."""
    sharding = importlib.import_module("3ddctvideoencoding_amd.sharding")
    per_gpu = CONFIGS[config][3]
    job = job_override or (JOB_STACKS.get(config) if per_gpu is None and not stacks_override else None)
    if job:
        first, n = sharding.shard(job, world, rank)
        return first, n, job, "strong"
    n = stacks_override or per_gpu or JOB_STACKS.get(config, 1)
    return rank * n, n, None, "weak"


def java_available_processors() -> tuple[int, str]:
    """What the reference's pool size, Runtime.getRuntime().availableProcessors() (Transform.java:63-64),
    returns on this host: a container-aware JVM counts the CPUs in the process's affinity mask, capped by
    the cgroup CPU quota (ceil(quota / period)) when one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = "affinity"
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and txt and txt[0] != "max":
            quota, period = int(txt[0]), int(txt[1])
        elif path.endswith("cfs_quota_us") and txt and int(txt[0]) > 0:
            quota = int(txt[0])
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().split()[0])
        else:
            continue
        q = max(1, -(-quota // period))
        if q < n:
            n, src = q, "cgroup quota"
        break
    return n, src


def cpu_baseline(width, height, depth, budget_s, kind):
    """Java-algorithm restatement (oracle/java_dct3d.c: grouped coefficients, memoised sums, one task
    per cube on a fixed thread pool, Math.round quantisation) on a bounded sample of the workload.
    Pool size = the reference's rule, availableProcessors() (Transform.java:63-64), except that an
    explicit OMP_NUM_THREADS (the GPU box sets it to the CPU share granted per GPU, 16) caps it: the
    machine's other cores belong to other jobs."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure, used here only as the CPU baseline leg

    pkg = importlib.import_module("3ddctvideoencoding_amd")
    avail, avail_src = java_available_processors()
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(avail, env) if env > 0 else avail
    plan = oracle.Plan(8, 8, depth)
    cubes_per_stack = (width // 8) * (height // 8)
    done, t_total, stacks = 0, 0.0, 0
    while t_total < budget_s and stacks < 64:
        fr = pkg.synthetic.frames(width, height, depth, frame0=stacks * depth, kind=kind)
        t0 = time.perf_counter()
        plan.encode_q(fr, threads=threads)
        t_total += time.perf_counter() - t0
        done += cubes_per_stack
        stacks += 1
    return {"value": done / t_total, "unit": "cubes/s", "cores": threads, "threads": threads,
            "host_cores": os.cpu_count(), "available_processors": avail,
            "pool_rule": f"availableProcessors() = {avail} ({avail_src})"
                         + (f", capped by OMP_NUM_THREADS={env} (this box's CPU share)" if 0 < env < avail else ""),
            "kind": "port",
            "sample": f"{stacks} x {width}x{height}x{depth} stack(s) ({done} cubes) through the restated Java "
                      f"DCT.run + Encoder quantisation, {threads} threads, {t_total:.1f} s"}


def bench_c1(a):
    """BASELINE config 1: the Java CPU Encoder path on one 64x64 8-frame stack (Encoder.java:47-89: the
    DCT's Transform.run over a fixed pool of availableProcessors() threads, one task per cube,
    Transform.java:63-104, then the Math.round quantisation into cube-major order).  The JVM cannot run
    here (no JDK); the restatement (oracle/java_dct3d.c, the same grouping, memoisation and pool) is
    what is timed, so `kind` is "port".  A step = one encode of the stack (DCT.run + quantisation); the
    per-file DCT setup (DCT.initialize + createSums, DCT.java:77-163) is timed once beside it.  No GPU:
    n_gpus 0, no roofline.  The output digest lets a test compare the step's result with the committed
    golden fixture (tests/golden/c1_64x64x8.npz)."""
    import hashlib

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: config 1 IS the CPU reference path, timed as its restatement

    width, height, depth = CONFIGS[a.config][:3]
    syn = importlib.import_module("3ddctvideoencoding_amd.synthetic")
    avail, avail_src = java_available_processors()
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(avail, env) if env > 0 else avail
    fr = syn.frames(width, height, depth, kind=a.kind)
    t0 = time.perf_counter()
    plan = oracle.Plan(8, 8, depth)
    plan_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(a.warmup):
        plan.encode_q(fr, threads=threads)
    # repeats: a step is ~1 ms of work, so every step is timed on its own and the line takes the mean
    times, q = [], None
    t_all = time.perf_counter()
    for _ in range(a.steps):
        t0 = time.perf_counter()
        q = plan.encode_q(fr, threads=threads)
        times.append(time.perf_counter() - t0)
    elapsed = time.perf_counter() - t_all
    cubes = (width // 8) * (height // 8)  # one stack
    ms = sorted(1e3 * t for t in times)
    value = cubes * a.steps / sum(times)
    base = {"value": value, "unit": "cubes/s", "cores": threads, "threads": threads,
            "host_cores": os.cpu_count(), "available_processors": avail,
            "pool_rule": f"availableProcessors() = {avail} ({avail_src})"
                         + (f", capped by OMP_NUM_THREADS={env} (this box's CPU share)" if 0 < env < avail else ""),
            "kind": "port",
            "sample": f"{a.steps} encodes of one {width}x{height}x{depth} stack ({cubes} cubes each) through the "
                      f"restated Java DCT.run + Encoder quantisation, {threads} threads, {sum(times):.3f} s"}
    res = {
        "metric": metric_name("java_cpu", depth, width, height),
        "value": value,
        "unit": "cubes/s",
        "n_gpus": 0,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * sum(times) / a.steps,
        "ms_per_step_median": ms[len(ms) // 2],
        "ms_per_step_min": ms[0],
        "wall_s": elapsed,
        "higher_is_better": True,
        "scaling": None,
        "vs_baseline": None,
        "dtype": "f64",
        "dtype_note": "the Java path's fp64 grouped fold (DCT.java:41-59, Sum.java:41-52), Math.round",
        "data": "synthetic",
        "config": {"workload": f"{width}x{height} grayscale, one {depth}-frame stack, {WHAT['java_cpu']}",
                   "name": a.config, "content": a.kind, "cubes_per_step": cubes, "parallelism": f"{threads} threads"},
        "plan_ms": plan_ms,
        "roofline": None,
        "output_sha256": hashlib.sha256(q.tobytes()).hexdigest(),
        "cpu_baseline": base,
    }
    print(json.dumps(res), flush=True)


def pmc_traffic(config: str, kernel: str, depth: int):
    """HBM bytes per launch of `kernel` from the PMC summary of this config (tools/gpu_pmc.sh ->
    profiles/pmc/<config>.csv): FETCH_SIZE (KB, x2 -- on gfx950 it counts half of a wide coalesced
    stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (KB).  None when no summary was collected."""
    import csv
    path = os.path.join(REPO, "profiles", "pmc", f"{config}.csv")
    if not os.path.exists(path):
        return None, None
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["kernel"]
        if (f"{kernel}<{depth}" in name or (kernel == "encode16_kernel" and f"{kernel}<" in name)):
            vals[r["counter"]] = float(r["avg_per_launch_raw"])
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        return None, None
    return (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0, os.path.relpath(path, REPO)


def job_roofline(per_rank, bytes_per_cube, peak_per_gpu=HBM_PEAK_GBS):
    """The job's roofline for N > 1: every rank's algorithmic bytes of one step, summed, over
    the slowest rank's device time per step, against N x the per-GPU peak -- and the weakest rank's own
    fraction beside it.  per_rank: [{"cubes", "device_ms_per_step", "frac"}, ...] (one entry per rank)."""
    n = len(per_rank)
    job_bytes = sum(r["cubes"] for r in per_rank) * bytes_per_cube
    t_ms = max(r["device_ms_per_step"] for r in per_rank)
    achieved = job_bytes / (t_ms * 1e-3) / 1e9 if t_ms > 0 else 0.0
    return {"achieved": achieved, "peak": n * peak_per_gpu, "frac": achieved / (n * peak_per_gpu),
            "job_bytes_per_step": job_bytes, "max_rank_device_ms_per_step": t_ms,
            "min_rank_frac": min(r["frac"] for r in per_rank)}


def measure_ceiling(ctx, torch, frames, q, reps, geom=None, dec_geom=None):
    """Achievable HBM rates on this device for the path's traffic mix, same buffers, same stream:
    mix = u8 read + int32 NT write (1:4, the encode's algorithmic bytes), copy, write-only, read-only.
    geom = (width, height, stacks, bytes_per_cube) for encode configs: also the encode kernel's own
    traffic without its compute (dct3d_encode_memonly_dev: same loads, LDS staging, NT stores).
    dec_geom = (width, height, stacks, raster_out) for the decode: its memory part and its compute
    part alone (dct3d_decode_diag_dev modes 1 / 2; libdct3d_diag.so)."""
    n_px = frames.numel() // 16 * 16
    out = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    if dec_geom is not None:
        width, height, stacks, raster = dec_geom
        out["decode_memonly_ms"] = timed(lambda: ctx.decode_diag_dev(q, width, height, stacks, raster, 1))
        out["decode_computeonly_ms"] = timed(lambda: ctx.decode_diag_dev(q, width, height, stacks, raster, 2))
    if geom is not None:
        width, height, stacks, bpc = geom
        ctx.encode_memonly_dev(frames, width, height, stacks, q)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ctx.encode_memonly_dev(frames, width, height, stacks, q)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        n_cubes = q.numel() // (bpc // 5)
        out["encode_memonly_ms"] = ms
        out["encode_memonly_GBs"] = n_cubes * bpc / (ms * 1e-3) / 1e9
        if bpc == 5 * 512:  # 8x8x8: the compute part alone (no loads, no stores)
            out["encode_computeonly_ms"] = timed(lambda: ctx.encode_diag_dev(frames, width, height, stacks, q, 2))
    for name, mode, bytes_per_px in (("mix_1r4w", 0, 5), ("copy", 1, 2), ("write", 2, 4), ("write_plain", 5, 4),
                                      ("read", 3, 1)):
        ctx.bandwidth_probe_dev(frames, q, n_px, mode)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ctx.bandwidth_probe_dev(frames, q, n_px, mode)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name + "_GBs"] = n_px * bytes_per_px / (ms * 1e-3) / 1e9
    return out


def xgmi_leg(ctx, torch, dist, sharding, frames, q, n_all, depth, width, height, rank, world, kind):
    """Optional host-of-record distribution, timed apart from the hot path: rank 0 holds the whole job
    (the same synthetic content each rank generated for its own shard: one long video, frame0 = 0),
    scatters every rank's stack range (sharding.shard) over RCCL p2p (xGMI), then gathers the quantised
    cubes back in stack order.  Both directions are verified: the received frames equal the rank's own,
    the gathered cube sums equal the senders'."""
    first, count = sharding.shard(n_all, world, rank)
    stack_px = depth * height * width
    stack_q = (width // 8) * (height // 8) * 64 * depth
    full = None
    if rank == 0:
        full = torch.empty((n_all * depth, height, width), dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic_dev(full, width, height, n_all * depth, frame0=0, kind=kind)
    recv = torch.empty_like(frames)
    torch.cuda.synchronize()

    def timed(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_sc = timed(lambda: sharding.scatter_stacks(full, recv, n_all, stack_px, rank, world))
    ok = torch.tensor([1 if torch.equal(recv, frames) else 0], dtype=torch.int64, device="cuda")
    del full, recv
    gathered = torch.empty((n_all * stack_q,), dtype=torch.int32, device="cuda") if rank == 0 else None
    t_ga = timed(lambda: sharding.gather_stacks(q, gathered, n_all, stack_q, rank, world))
    sums = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(world)]
    dist.all_gather(sums, q[:count * stack_q].sum(dtype=torch.int64).view(1))
    if rank == 0:
        for r in range(world):
            f, c = sharding.shard(n_all, world, r)
            if int(gathered[f * stack_q:(f + c) * stack_q].sum(dtype=torch.int64).item()) != int(sums[r].item()):
                ok.zero_()
    del gathered
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return {"scatter_s": t_sc, "scatter_GBs": n_all * stack_px / t_sc / 1e9,
            "gather_s": t_ga, "gather_GBs": n_all * stack_q * 4 / t_ga / 1e9,
            "bytes_note": "job totals (rank 0's own shard is a local copy)", "verified": bool(ok.item())}


def main():
    a = parse()
    width, height, depth, stacks, direction = CONFIGS[a.config]
    if direction == "java_cpu":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("c1_java_cpu_64x64 is the CPU reference path: run it without torch.distributed")
        return bench_c1(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world != 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    sharding = importlib.import_module("3ddctvideoencoding_amd.sharding")
    first, stacks, job_stacks, scaling = rank_stacks(a.config, a.stacks, a.job_stacks, world, rank)

    import torch

    dist = None
    # DCT3D_BENCH_FORCE_DIST=1: the distributed path (process group, barrier, all-gathers, RCCL) even for a
    # single rank, so that a one-GPU box runs the code the driver's N > 1 runs (tests/test_gpu_bench_flow.py)
    if world > 1 or os.environ.get("DCT3D_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        # one process per GPU over RCCL ("nccl").  DCT3D_BENCH_BACKEND=gloo rehearses the N>1 flow with
        # several ranks on fewer GPUs (ranks are mapped onto the visible devices round-robin).
        backend = os.environ.get("DCT3D_BENCH_BACKEND", "nccl")
        dev_idx = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_idx)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    pkg = importlib.import_module("3ddctvideoencoding_amd")
    ctx = pkg.Context(dev, 8, 8, depth)
    for o in a.opt:
        name, val = o.split("=", 1)
        ctx.set_option(getattr(pkg, "DCT3D_OPT_" + name.upper()), float(val))
    # a dedicated stream: the library, torch's events and torch's allocations all use it (torch's
    # default stream has handle 0, which the C-ABI reads as "use the context's own stream")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    n_cubes = ctx.n_cubes(width, height, stacks)
    cs = 64 * depth
    frames = torch.empty((max(1, stacks) * depth, height, width), dtype=torch.uint8, device="cuda")
    # each rank encodes different content (its own slice of one long synthetic video)
    ctx.fill_synthetic_dev(frames, width, height, stacks * depth, frame0=first * depth, kind=a.kind)
    q = torch.empty((max(1, n_cubes) * cs,), dtype=torch.int32, device="cuda")
    eg_info = {}
    if direction == "decode":
        ctx.encode_stacks_dev(frames, width, height, stacks, q)  # input of the decode = encoder output
        out = torch.empty_like(frames)

        def step():
            ctx.decode_stacks_dev(q, width, height, stacks, out)
    elif direction == "decode_eg":
        eg_cap = n_cubes * cs
        eg_stream = torch.empty(eg_cap // 4, dtype=torch.int32, device="cuda")
        eg_info["bits"] = ctx.encode_eg_dev(frames, width, height, stacks, eg_stream, eg_cap)  # the encoder's stream
        nbytes = (eg_info["bits"] + 7) // 8
        out = torch.empty_like(frames)
        eg_ev = []
        if a.eg_two_step:
            def step():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctx.eg_decode_dev(eg_stream, nbytes, 0, n_cubes, q)  # synchronises (status read back)
                e1.record()
                eg_ev.append((e0, e1))
                ctx.decode_stacks_dev(q, width, height, stacks, out)
        else:  # fused (dct3d_decode_eg_dev): stream -> raster, no int32 intermediate; the step is the whole
            # EG stage, so no per-step events (their packets and the host work would sit in the timed region)
            def step():
                # returns with the verdict, the raster completing on the stream (the timed region ends with a
                # device synchronisation)
                ctx.decode_eg_dev(eg_stream, nbytes, 0, width, height, stacks, out)
    elif direction == "encode_eg" and a.eg_two_step:
        eg_cap = n_cubes * cs  # 8 bits per value: far above what quantised content needs
        eg_out = torch.empty(eg_cap // 4, dtype=torch.int32, device="cuda")
        eg_ev = []

        def step():
            ctx.encode_stacks_dev(frames, width, height, stacks, q)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eg_info["bits"] = ctx.eg_encode_dev(q, n_cubes, eg_out, eg_cap)  # synchronises (total read back)
            e1.record()
            eg_ev.append((e0, e1))
    elif direction == "encode_eg":
        # fused path (dct3d_encode_eg_dev): raster -> stream, no int32 intermediate
        eg_cap = n_cubes * cs
        eg_out = torch.empty(eg_cap // 4, dtype=torch.int32, device="cuda")
        del q
        q = None

        def step():
            eg_info["bits"] = ctx.encode_eg_dev(frames, width, height, stacks, eg_out, eg_cap)  # synchronises
    elif direction in ("forward_f32", "inverse_f32"):
        nby, nbx = height // 8, width // 8
        if direction == "forward_f32":  # readCubes (encoder.c:29-41): u8 raster -> float cube-major
            f_in = (frames.view(stacks, depth, nby, 8, nbx, 8).permute(0, 2, 4, 1, 3, 5)
                    .to(torch.float32).contiguous().view(-1))
        else:  # applyDequantization (decoder.c:48-59) of the encoder's output, float cube-major
            ctx.encode_stacks_dev(frames, width, height, stacks, q)
            kk = torch.arange(cs, device="cuda")
            steps = torch.clamp(5 * (kk % 8 + (kk // 8) % 8 + kk // 64), min=1).to(torch.float32)
            f_in = (q.view(n_cubes, cs).to(torch.float32) * steps).view(-1)
        del q
        q = None
        f_out = torch.empty_like(f_in)
        run = ctx.forward_f32_dev if direction == "forward_f32" else ctx.inverse_f32_dev

        def step():
            run(f_in, n_cubes, f_out)
    else:
        def step():
            ctx.encode_stacks_dev(frames, width, height, stacks, q)
    torch.cuda.synchronize()

    # settle: the GPU's power management needs ~30 ms of sustained load to reach its steady state -- a
    # rocprofv3 trace of back-to-back launches shows kernel durations rising ~15 % over the first ~10
    # launches and decaying back over the next ~50 (profiles/r03/power_transient/); untimed steps for
    # at least --settle-ms of wall time come before the W warmup steps, so the K timed steps measure
    # the steady state whatever W is
    settle_steps, t_settle = 0, time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
        for _ in range(4):
            step()
        settle_steps += 4
        torch.cuda.synchronize()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # the library's per-launch events (kernel_ms) cost ~17 us of device time per step (event packets
    # between the launches); by default they run in a separate pass after the timed region, so the timed
    # steps are back-to-back launches only
    events_timed = a.kernel_events == "timed"
    ctx.set_profiling(events_timed)
    ctx.reset_timers()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # device-side time of the whole timed region on the bench stream (every launch of every step and
    # the gaps between them): the roofline basis, the same interval as `value`'s host clock
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_a.record()
    for _ in range(a.steps):
        step()
    ev_b.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dev_step_ms = ev_a.elapsed_time(ev_b) / a.steps
    if not events_timed:  # the kernel-timing pass: the same steps again, each launch between events
        ctx.set_profiling(True)
        ctx.reset_timers()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    st = ctx.stats()
    ctx.set_profiling(False)
    round_trip = None
    if direction in ("decode", "decode_eg") and stacks:  # the codec's round trip
        d = out.to(torch.int16) - frames.to(torch.int16)
        mse = float((d.to(torch.float64) ** 2).mean())
        round_trip = {"vs": "encoder input frames (lossy: quantisation); bit-exactness against the Java-semantics "
                            "decode is pinned by tests/test_gpu_parity.py",
                      "max_abs_err": int(d.abs().max()), "mean_abs_err": float(d.abs().to(torch.float64).mean()),
                      "psnr_db": (10.0 * math.log10(255.0 ** 2 / mse)) if mse > 0 else None}
    ceiling = None if a.no_ceiling or q is None or not stacks else measure_ceiling(
        ctx, torch, frames, q, max(3, a.steps // 2),
        geom=(width, height, stacks, cs * 5) if direction == "encode" else None,
        dec_geom=(width, height, stacks, torch.empty_like(frames)) if direction == "decode" else None)

    bytes_per_cube = cs * (1 + 4)  # u8 in + int32 out (encode) / int32 in + u8 out (decode)
    if direction in ("forward_f32", "inverse_f32"):
        bytes_per_cube = cs * (4 + 4)  # f32 in + f32 out (4,096 B per cube)
    fused = direction == "encode_eg" and not a.eg_two_step
    if fused:  # u8 in + the cube's share of the coded stream and of the segment bit totals out
        bytes_per_cube = cs + eg_info["bits"] / 8 / max(1, n_cubes) + 4 / 8
    fused_dec = direction == "decode_eg" and not a.eg_two_step
    if fused_dec:  # the cube's share of the stream in, u8 out
        bytes_per_cube = cs + eg_info["bits"] / 8 / max(1, n_cubes)
    kernel_ms = st["kernel_ms_total"] / max(1, st["n_timed"])
    aux_ms = st["aux_ms_total"] / max(1, st["n_timed"])
    alg_bytes = n_cubes * bytes_per_cube
    achieved = alg_bytes / (dev_step_ms * 1e-3) / 1e9 if n_cubes else 0.0       # step basis
    kernel_achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    if ceiling and "encode_memonly_GBs" in ceiling:  # the kernel against its own traffic without compute
        ceiling["kernel_vs_memonly"] = kernel_achieved / ceiling["encode_memonly_GBs"]
        ceiling["step_vs_memonly"] = achieved / ceiling["encode_memonly_GBs"]
    if ceiling and "decode_memonly_ms" in ceiling and kernel_ms > 0:
        ceiling["kernel_vs_memonly"] = ceiling["decode_memonly_ms"] / kernel_ms
    kname = ("decode_eg_kernel" if fused_dec else "decode_kernel") if direction in ("decode", "decode_eg") else (
        "encode_eg_kernel" if fused else ("encode16_kernel" if depth == 8 else "encode_kernel"))
    if direction in ("forward_f32", "inverse_f32"):
        kname = "cube_f32_kernel"
    step_kernels = [kname] + (["eg_compact_kernel"] if fused else [])
    traffic, traffic_src = pmc_traffic(a.config, kname, depth) if not (a.stacks or a.job_stacks) else (None, None)

    # per-rank record (strong scaling: shards differ in size; the job rate is total cubes / max time)
    per_rank = None
    if dist:
        mine = torch.tensor([float(rank), float(stacks), float(n_cubes), dev_step_ms, achieved / HBM_PEAK_GBS],
                            dtype=torch.float64, device="cuda")
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [{"rank": int(r[0]), "stacks": int(r[1]), "cubes": int(r[2]), "device_ms_per_step": float(r[3]),
                     "frac": float(r[4])} for r in (x.tolist() for x in allr)]
    elapsed, total_cubes = sharding.reduce_timing(elapsed, n_cubes, device="cuda")  # max time, summed units
    xgmi = None
    if a.xgmi and dist is not None and direction == "encode" and os.environ.get("DCT3D_BENCH_BACKEND", "nccl") == "nccl":
        xgmi = xgmi_leg(ctx, torch, dist, sharding, frames[:stacks * depth], q, job_stacks or world * stacks,
                        depth, width, height, rank, world, a.kind)

    ms_per_step = elapsed * 1e3 / a.steps
    value = total_cubes * a.steps / elapsed
    unit_name = "8x8x8" if depth == 8 else "8x8x4"
    res = {
        "metric": metric_name(direction, depth, width, height),
        "value": value,
        "unit": "cubes/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "settle_steps": settle_steps,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64" if direction in ("decode", "decode_eg", "forward_f32", "inverse_f32") else "f32",
        "dtype_note": ("fp64 arithmetic throughout" if direction in ("decode", "decode_eg", "forward_f32", "inverse_f32")
                       else "fp32 butterflies certified per coefficient against the fp64 Java value; uncertified "
                            "ones are settled by an fp64 recheck or the exact Java fold, so every output equals "
                            "the fp64 Java result (not a reduced-precision result)"),
        "data": "synthetic",
        "config": {
            "workload": f"{width}x{height} grayscale, {depth}-frame stacks, "
                        f"{WHAT[direction]}"
                        f" ({unit_name} cubes), "
                        + (f"one job of {job_stacks} device-resident stacks split over {world} GPU(s)" if job_stacks
                           else f"{stacks} device-resident stacks per GPU per step"),
            "name": a.config,
            "stacks_per_gpu": stacks if not job_stacks else None,
            "job_stacks": job_stacks,
            "cubes_per_gpu_step": n_cubes,
            "content": a.kind,
            "options": a.opt or None,
            "parallelism": f"dp{world} (stacks sharded, no data-path collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "basis": "algorithmic bytes of one step / device time per step (HIP events around the timed "
                     "region on the bench stream: every launch of the step, " + " + ".join(step_kernels) + ")",
            "traffic": traffic,  # HBM bytes per launch of the main kernel (PMC), compare with algorithmic_bytes
            "traffic_source": traffic_src,
            "algorithmic_bytes": alg_bytes,
            "bytes_per_cube": bytes_per_cube,
            "device_ms_per_step": dev_step_ms,
            "kernel": kname,
            "kernel_ms": kernel_ms,
            "aux_ms": aux_ms,
            "kernel_only_achieved": kernel_achieved,
            "kernel_only_frac": kernel_achieved / HBM_PEAK_GBS,
        },
        "ceiling": ceiling,
        "flagged_units_last_step": st["n_flagged"],
        "rechecked_units_last_step": st.get("n_rechecked", 0),
        "units_per_step": st["n_units"],
        "mcubes_per_s_per_gpu": value / world / 1e6,
        "eg_stage": None if direction not in ("encode_eg", "decode_eg") else {
            "path": ("fused" if fused_dec else "two-step") if direction == "decode_eg" else ("fused" if fused else "two-step"),
            "ms_per_step": (aux_ms if fused else dev_step_ms if fused_dec
                            else sum(x.elapsed_time(y) for x, y in eg_ev[-a.steps:]) / a.steps),
            "bits_per_value": eg_info["bits"] / (max(1, n_cubes) * cs),
            "stream_bytes_per_step": (eg_info["bits"] + 7) // 8},
        "round_trip": round_trip,
        "cpu_baseline": None,
    }
    if per_rank is not None:
        res["per_rank"] = per_rank
        # N > 1: roofline = the job aggregate (all ranks' bytes / the slowest rank's device time / N peaks);
        # rank 0's own numbers stay under roofline.rank0_*
        rf = res["roofline"]
        rf["rank0_achieved"], rf["rank0_frac"] = rf["achieved"], rf["frac"]
        agg = job_roofline(per_rank, bytes_per_cube)
        rf.update(achieved=agg["achieved"], peak=agg["peak"], frac=agg["frac"],
                  min_rank_frac=agg["min_rank_frac"], job_bytes_per_step=agg["job_bytes_per_step"],
                  max_rank_device_ms_per_step=agg["max_rank_device_ms_per_step"],
                  basis="job aggregate: the algorithmic bytes of every rank's step / the slowest rank's device "
                        "time per step / (N x 8 TB/s); rank0_* and per_rank hold the per-rank rates")
    if xgmi is not None:
        res["xgmi"] = xgmi
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(width, height, depth, a.cpu_baseline_seconds, a.kind)
        except Exception as e:  # the baseline is reported, never the target
            res["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
