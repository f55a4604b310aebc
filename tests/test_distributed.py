"""CPU: the N>1 path -- contiguous stack sharding with no data-path collective, gloo world_size 2.

Each rank encodes its own stack range with the Java-semantics oracle (the per-rank work stands in
for the GPU kernel here), the shards are gathered to rank 0 in stack order and must equal the
single-process encode; the timing reduction is max-over-ranks and the units are summed."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist
    import oracle
    pkg = importlib.import_module("3ddctvideoencoding_amd")
    sh = importlib.import_module("3ddctvideoencoding_amd.sharding")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n_stacks = 5
    first, count = sh.shard(n_stacks, world, rank)
    frames = pkg.synthetic.frames(48, 32, count * 8, frame0=first * 8, kind="uniform")
    q = oracle.Plan(8, 8, 8).encode_q(frames, threads=1) if count else np.zeros((0, 8, 8, 8), np.int32)
    t, u = sh.reduce_timing(0.1 * (rank + 1), q.shape[0])
    parts = [None] * world if rank == 0 else None
    dist.gather_object((first, q), parts, dst=0)
    if rank == 0:
        full = np.concatenate([p[1] for p in sorted(parts, key=lambda p: p[0])])
        np.save(os.path.join(out_dir, "full.npy"), full)
        np.save(os.path.join(out_dir, "tu.npy"), np.array([t, u]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges():
    sh = importlib.import_module("3ddctvideoencoding_amd.sharding")
    for n in (0, 1, 7, 64, 65):
        for w in (1, 2, 3, 8):
            rs = [sh.shard(n, w, r) for r in range(w)]
            assert sum(c for _, c in rs) == n
            assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(c for _, c in rs) - min(c for _, c in rs) <= 1
    assert sh.shard(64, 8, 3) == (24, 8)   # config 4: 64 4K stacks over 8 GPUs
    with pytest.raises(ValueError):
        sh.shard(4, 2, 2)


def test_world2_gloo_sharded_encode_equals_single(tmp_path, pkg, plan8):
    mp.spawn(_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    full = np.load(tmp_path / "full.npy")
    frames = pkg.synthetic.frames(48, 32, 40, kind="uniform")
    assert np.array_equal(full, plan8.encode_q(frames))
    t, u = np.load(tmp_path / "tu.npy")
    assert abs(t - 0.2) < 1e-12 and u == full.shape[0]


def test_checksum_order_sensitive():
    sh = importlib.import_module("3ddctvideoencoding_amd.sharding")
    a = np.arange(1000, dtype=np.int32)
    assert sh.checksum(a) != sh.checksum(a[::-1].copy())
    assert sh.checksum(a) == sh.checksum(a.copy())


def _xgmi_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sh = importlib.import_module("3ddctvideoencoding_amd.sharding")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n_stacks, numel = 7, 40          # ragged: shards of 3/2/2 stacks at world 3
    full = torch.arange(n_stacks * numel, dtype=torch.int32) if rank == 0 else None
    first, count = sh.shard(n_stacks, world, rank)
    local = torch.full((max(count, 1) * numel,), -1, dtype=torch.int32)
    sh.scatter_stacks(full, local, n_stacks, numel, rank, world)
    ok = bool(torch.equal(local[:count * numel], torch.arange(first * numel, (first + count) * numel, dtype=torch.int32)))
    # each rank transforms its shard (stand-in for the kernel), rank 0 gathers in stack order
    local[:count * numel] = local[:count * numel] * 3 + rank
    back = torch.zeros(n_stacks * numel, dtype=torch.int32) if rank == 0 else None
    sh.gather_stacks(local, back, n_stacks, numel, rank, world)
    flags = [None] * world if rank == 0 else None
    dist.gather_object(ok, flags, dst=0)
    if rank == 0:
        np.save(os.path.join(out_dir, "back.npy"), back.numpy())
        np.save(os.path.join(out_dir, "ok.npy"), np.array(flags))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_gather_stacks_gloo(tmp_path, world):
    """The optional host-of-record distribution (bench.py --xgmi): p2p scatter of stack ranges from
    rank 0 and the gather back in stack order, with ragged shards."""
    mp.spawn(_xgmi_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    assert np.load(tmp_path / "ok.npy").all()
    back = np.load(tmp_path / "back.npy")
    sh = importlib.import_module("3ddctvideoencoding_amd.sharding")
    exp = np.arange(7 * 40, dtype=np.int32) * 3
    for r in range(world):
        f, c = sh.shard(7, world, r)
        exp[f * 40:(f + c) * 40] += r
    assert np.array_equal(back, exp)


def test_bench_job_split():
    """bench.py's per-rank work: config 4 is ONE job of 64 4K stacks split over the ranks (strong
    scaling, contiguous shards covering the job exactly once); config 2 gives every rank its own 128
    stacks (weak scaling), rank r the r-th slice of one video."""
    sys.path.insert(0, REPO)
    bench = importlib.import_module("bench")
    for world in (1, 2, 4, 8, 3):
        parts = [bench.rank_stacks("c4_encode_4k", None, None, world, r) for r in range(world)]
        assert all(p[2] == 64 and p[3] == "strong" for p in parts)
        assert sum(p[1] for p in parts) == 64
        assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        if 64 % world == 0:
            assert all(p[1] == 64 // world for p in parts)
        w = [bench.rank_stacks("c2_encode_1080p", None, None, world, r) for r in range(world)]
        assert all(p == (r * 128, 128, None, "weak") for r, p in enumerate(w))
    assert bench.rank_stacks("c4_encode_4k", 8, None, 2, 1) == (8, 8, None, "weak")      # --stacks: weak
    assert bench.rank_stacks("c2_encode_1080p", None, 10, 4, 3) == (8, 2, 10, "strong")  # --job-stacks


def _roofline_worker(rank, world, port, out_dir):
    """Each rank's per-step record as bench.py gathers it (all_gather over the process group), then the
    job aggregate bench.py reports for N > 1."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    bench = importlib.import_module("bench")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cubes = [1036800, 1036800, 518400][rank]           # ragged shards, as a 2.5-stack split would be
    ms = [0.50, 0.55, 0.30][rank]
    frac = cubes * 2560 / (ms * 1e-3) / 1e9 / 8000.0
    mine = torch.tensor([float(rank), 8.0, float(cubes), ms, frac], dtype=torch.float64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per_rank = [{"rank": int(r[0]), "stacks": int(r[1]), "cubes": int(r[2]), "device_ms_per_step": float(r[3]),
                 "frac": float(r[4])} for r in (x.tolist() for x in allr)]
    agg = bench.job_roofline(per_rank, 2560)
    if rank == 0:
        np.save(os.path.join(out_dir, "agg.npy"), np.array([agg["achieved"], agg["peak"], agg["frac"],
                                                            agg["min_rank_frac"]]))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_job_roofline_gloo(tmp_path):
    """for N > 1 bench.py reports roofline.frac as the job aggregate -- total
    algorithmic bytes / max-over-ranks device time / (N x 8 TB/s) -- with the weakest rank's own frac
    beside it (min_rank_frac), not rank 0's."""
    mp.spawn(_roofline_worker, args=(3, _port(), str(tmp_path)), nprocs=3, join=True)
    achieved, peak, frac, min_rank = np.load(tmp_path / "agg.npy")
    job = (1036800 * 2 + 518400) * 2560
    assert abs(achieved - job / 0.55e-3 / 1e9) < 1e-6 * achieved
    assert peak == 3 * 8000.0
    assert abs(frac - achieved / 24000.0) < 1e-12
    assert abs(min_rank - 518400 * 2560 / 0.30e-3 / 1e9 / 8000.0) < 1e-12    # the half shard's own rate
    assert frac < min_rank  # the ragged third rank idles while the slowest one finishes
