"""Multi-GPU sharding of the hot path: one process per GPU, contiguous stack ranges,
no data-path collective.  Every 8-frame stack (and every cube in it) is independent for the DCT and
the quantisation (Transform.java:94-100, encoder.c:203), so a job of S stacks on N ranks gives rank r
the stacks [first, first+count).  The only collectives are a barrier around timed regions and tiny
all-reduces (max time, summed unit counts, checksums) -- RCCL ("nccl") on MI355X, gloo on CPU.

The entropy stage (Exp-Golomb + zlib) is stream-sequential (the partial byte and the zlib state carry
across stacks, ExpGolomb.c:112-122) and stays on one host: shards return cube-major int32 that the
owner concatenates in stack order.
"""
from __future__ import annotations


def shard(n_stacks: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced range of stacks for `rank` (the first n % world ranks get one more)."""
    if world <= 0 or not (0 <= rank < world) or n_stacks < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_stacks, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def reduce_timing(elapsed_s: float, units: int, device=None):
    """(max elapsed over ranks, sum of units over ranks); identity when torch.distributed is not
    initialised.  The job rate is units_total / max_elapsed (bench.py contract)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return elapsed_s, units
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    u = torch.tensor([float(units)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), int(u.item())


def checksum(q) -> int:
    """Order-sensitive 64-bit checksum of an int32 cube buffer (numpy or torch): used to all-reduce
    per-shard digests without moving the data."""
    import numpy as np

    if hasattr(q, "detach"):
        q = q.detach().cpu().numpy()
    a = np.ascontiguousarray(q, np.int32).view(np.uint32).astype(np.uint64)
    w = (np.arange(a.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1)
    with np.errstate(over="ignore"):
        return int(np.bitwise_xor.reduce(a * w) if a.size else 0)


# ---- optional host-of-record distribution: timed apart from the hot path ----------
# A job whose frames live on one GPU (rank 0) hands every rank its contiguous stack range and collects
# the quantised cubes back in stack order.  Point-to-point sends over RCCL (xGMI between the GPUs of a
# node; gloo on CPU), posted together with batch_isend_irecv so that rank 0 drives all its links at once.
# Not part of the timed path: the bench's default step has no data-path collective (each rank generates
# its own stacks), `bench.py --xgmi` times these two steps separately.
def _p2p(ops):
    import torch.distributed as dist

    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def scatter_stacks(full, local, n_stacks: int, stack_numel: int, rank: int, world: int) -> None:
    """Rank 0 sends rank r the flat elements of its stacks shard(n_stacks, world, r) from `full` (rank 0
    only; any tensor with n_stacks * stack_numel elements); every rank receives its range into `local`
    (rank 0 copies its own)."""
    import torch.distributed as dist

    first, count = shard(n_stacks, world, rank)
    if local.numel() < count * stack_numel:
        raise ValueError("local buffer too small for this rank's shard")
    ops = []
    if rank == 0:
        flat = full.reshape(-1)
        for r in range(1, world):
            f, c = shard(n_stacks, world, r)
            if c:
                ops.append(dist.P2POp(dist.isend, flat[f * stack_numel:(f + c) * stack_numel], r))
        if count:
            local.reshape(-1)[:count * stack_numel].copy_(flat[first * stack_numel:(first + count) * stack_numel])
    elif count:
        ops.append(dist.P2POp(dist.irecv, local.reshape(-1)[:count * stack_numel], 0))
    _p2p(ops)


def gather_stacks(local, full, n_stacks: int, stack_numel: int, rank: int, world: int) -> None:
    """The inverse of scatter_stacks: rank r sends the first shard-size elements of `local`; rank 0
    receives every range into its place in `full` (stack order)."""
    import torch.distributed as dist

    first, count = shard(n_stacks, world, rank)
    ops = []
    if rank == 0:
        flat = full.reshape(-1)
        for r in range(1, world):
            f, c = shard(n_stacks, world, r)
            if c:
                ops.append(dist.P2POp(dist.irecv, flat[f * stack_numel:(f + c) * stack_numel], r))
        if count:
            flat[first * stack_numel:(first + count) * stack_numel].copy_(local.reshape(-1)[:count * stack_numel])
    elif count:
        ops.append(dist.P2POp(dist.isend, local.reshape(-1)[:count * stack_numel], 0))
    _p2p(ops)
