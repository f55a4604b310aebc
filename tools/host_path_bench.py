"""PCIe-inclusive throughput of the host-pointer entry points, on the GPU box.

Raw link rates first (torch copies, pinned and pageable host memory), then every host API end to end on
S stacks of 1080p x 8 frames with ordinary (pageable) numpy buffers, as a caller of the codec would:
  encode_stacks  u8 raster in -> int32 cubes out      (1 B/px in, 4 B/px out)
  decode_stacks  int32 cubes in -> u8 raster out      (4 B/px in, 1 B/px out)
  encode_eg      u8 raster in -> Exp-Golomb stream    (1 B/px in, ~0.2 B/px out)
  decode_eg      stream in -> u8 raster out           (~0.2 B/px in, 1 B/px out)
These are never bench.py's `value` (that is device-resident); DESIGN.md §5 quotes them.
usage: python tools/host_path_bench.py [--stacks 16] [--reps 3] [--depth 8]  -> one JSON line"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed(fn, reps):
    fn()  # warm-up (allocations, first-touch)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stacks", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module("3ddctvideoencoding_amd")
    W, H, D, S = 1920, 1080, a.depth, a.stacks
    res = {"stacks": S, "width": W, "height": H, "depth": D}

    # raw link: 1 GiB pinned / pageable, both directions
    nbytes = 1 << 30
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    pin = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    pag = torch.from_numpy(np.ones(nbytes, np.uint8))
    for name, host in (("pinned", pin), ("pageable", pag)):
        def h2d():
            dev.copy_(host, non_blocking=False)
            torch.cuda.synchronize()

        def d2h():
            host.copy_(dev, non_blocking=False)
            torch.cuda.synchronize()
        res[f"h2d_{name}_GBs"] = nbytes / timed(h2d, a.reps) / 1e9
        res[f"d2h_{name}_GBs"] = nbytes / timed(d2h, a.reps) / 1e9
    del dev, pin, pag

    ctx = pkg.Context(0, 8, 8, D)
    L = pkg.lib()
    import ctypes
    frames = pkg.synthetic.frames(W, H, S * D, kind="ramp")
    n_cubes = ctx.n_cubes(W, H, S)
    px = frames.size
    # caller-owned, pre-faulted buffers (a codec reuses its buffers; first-touch page faults of a
    # fresh numpy array are not the library's cost)
    q = np.empty(px, np.int32)
    q.fill(0)
    rast = np.empty_like(frames)
    rast.fill(0)
    stream, tb = ctx.encode_eg(frames)
    sbuf = np.frombuffer(stream, np.uint8).copy()
    ptr = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    h = ctx._h
    u64 = ctypes.c_uint64(0)

    def enc():
        assert L.dct3d_encode_stacks(h, ptr(frames), W, H, S, ptr(q), None) == 0

    def dec():
        assert L.dct3d_decode_stacks(h, ptr(q), W, H, S, ptr(rast)) == 0

    def enc_eg():
        assert L.dct3d_encode_eg(h, ptr(frames), W, H, S, 0, 0, ctypes.byref(u64)) == 0
        assert L.dct3d_eg_fetch(h, ptr(sbuf), (u64.value + 7) // 8) == 0

    def dec_eg():
        assert L.dct3d_decode_eg(h, ptr(sbuf), sbuf.size, 0, W, H, S, ptr(rast), ctypes.byref(u64)) == 0

    rows = [("encode_stacks", enc, px * 5), ("decode_stacks", dec, px * 5),
            ("encode_eg", enc_eg, px + len(stream)), ("decode_eg", dec_eg, px + len(stream))]
    for name, fn, moved in rows:
        t = timed(fn, a.reps)
        res[name] = {"ms": t * 1e3, "cubes_per_s": n_cubes / t, "pcie_GBs": moved / t / 1e9}
    enc()
    assert np.array_equal(q.reshape(-1), ctx.encode_stacks(frames).reshape(-1))  # same answer as the API
    res["stream_bytes"] = len(stream)
    ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
