#!/usr/bin/env python3
"""Timeline of one 8x8x8 encode launch (diagnostic, libdct3d_diag.so dct3d_encode_trace_dev): every
wave's start, transform-done and stores-issued times on the 100 MHz clock, and its XCC / CU.  Prints
the launch's shape -- ramp (first completions), steady rate, tail (after the last wave starts), per-XCD
finish times -- and writes the per-microsecond profile to --out.

  python tools/enc_timeline.py --width 3840 --height 2160 --stacks 8 --out gpurun_out/tl_4k8.json
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--stacks", type=int, default=8)
    ap.add_argument("--kind", default="ramp")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module("3ddctvideoencoding_amd")
    torch.cuda.set_device(0)
    ctx = pkg.Context(0, 8, 8, 8)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    w, h, n = a.width, a.height, a.stacks
    frames = torch.empty((n * 8, h, w), dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic_dev(frames, w, h, n * 8, frame0=0, kind=a.kind)
    n_cubes = ctx.n_cubes(w, h, n)
    q = torch.empty(n_cubes * 512, dtype=torch.int32, device="cuda")
    q2 = torch.empty_like(q)
    n_waves = (n_cubes + 3) // 4
    tr = torch.zeros(n_waves * 4, dtype=torch.int64, device="cuda")
    for _ in range(5):
        ctx.encode_stacks_dev(frames, w, h, n, q)
    res = []
    for r in range(a.reps):
        ctx.encode_stacks_dev(frames, w, h, n, q)     # the launch before it, as in the bench's steps
        ctx.encode_trace_dev(frames, w, h, n, q2, tr)
        torch.cuda.synchronize()
        res.append(tr.cpu().numpy().reshape(n_waves, 4).copy())
    assert torch.equal(q, q2), "the traced launch must produce the product's output"
    t = res[-1]
    t0 = t[:, 0].min()
    st, tc, te = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0   # microseconds
    hw = t[:, 3]
    xcc = (hw >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    T = te.max()
    bins = np.arange(0.0, T + 1.0, 1.0)
    active = np.array([((st <= b) & (te > b)).sum() for b in bins])
    done, _ = np.histogram(te, bins=np.append(bins, bins[-1] + 1))
    cubes_per_us = done * 4
    bytes_per_us = cubes_per_us * 2560
    last_start = st.max()
    order = np.sort(te)
    q10, q50, q90 = (order[int(f * (len(order) - 1))] for f in (0.1, 0.5, 0.9))
    steady = (bins > q10) & (bins < q90)
    steady_rate = bytes_per_us[steady].mean() / 1e3 if steady.any() else 0.0  # GB/s = B/us / 1e3
    first_round = st < 1.0
    per_xcc_end = {int(x): float(te[xcc == x].max()) for x in np.unique(xcc)}
    per_xcc_waves = {int(x): int((xcc == x).sum()) for x in np.unique(xcc)}
    summary = {
        "geometry": f"{w}x{h}x8 x {n} stacks, {n_cubes} cubes, {n_waves} waves",
        "launch_us": float(T),
        "ideal_us_at_steady_rate": float(n_cubes * 2560 / (steady_rate * 1e3)) if steady_rate else None,
        "steady_GBs_10_90pct": float(steady_rate),
        "first_completion_us": float(te.min()),
        "completions_10_50_90pct_us": [float(q10), float(q50), float(q90)],
        "last_wave_start_us": float(last_start),
        "tail_after_last_start_us": float(T - last_start),
        "first_round_waves": int(first_round.sum()),
        "first_round_transform_us_median": float(np.median(tc[first_round] - st[first_round])),
        "later_transform_us_median": float(np.median(tc[~first_round] - st[~first_round])),
        "first_round_store_done_us_median": float(np.median(te[first_round])),
        "wave_life_us_median": float(np.median(te - st)),
        "max_active_waves": int(active.max()),
        "per_xcc_end_us": per_xcc_end,
        "per_xcc_waves": per_xcc_waves,
        "launch_us_all_reps": [float((r[:, 2].max() - r[:, 0].min()) / 100.0) for r in res],
    }
    print(json.dumps(summary))
    if a.out:
        json.dump({"summary": summary, "bins_us": bins.tolist(), "active_waves": active.tolist(),
                   "GBs_per_bin": (bytes_per_us / 1e3).tolist()}, open(a.out, "w"))
    ctx.close()


if __name__ == "__main__":
    main()
