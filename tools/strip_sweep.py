"""Traversal sweep of the 8x8x8 encode (the 4K 8-stack shard at 0.68 of the HBM peak against
0.72 for the 1080p batch, both at 0.98-0.99 of their own memory-only twins -- so the read pattern, not
the compute).  The product's waves walk the cubes row-major (runs of 64 consecutive 4-cube slots per XCD,
xcd_tile<64>); the sweep walks them in vertical strips of S cubes (dct3d_encode_strip_dev, libdct3d_diag.so):
memory-only twin (mode 1) and the full encode (mode 0) per S, the product (row-major) beside them,
interleaved over rounds on one box, HIP events on the bench's stream.  One JSON line per geometry.
    python tools/strip_sweep.py [--rounds 3] [--reps 20]"""
import argparse, importlib, json, os, sys, time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("3ddctvideoencoding_amd")
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
GEOMS = [("4k_shard", 3840, 2160, 8, [16, 32, 48, 80, 96, 160, 240]),
         ("1080p_128", 1920, 1080, 128, [16, 48, 80, 240])]
with pkg.Context(0, 8, 8, 8) as ctx:
    ctx.set_stream(stream.cuda_stream)
    for name, w, h, stacks, strips in GEOMS:
        frames = torch.empty(stacks * 8 * h * w, dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic_dev(frames, w, h, stacks * 8, frame0=0, kind="ramp")
        n = ctx.n_cubes(w, h, stacks)
        q = torch.empty(n * 512, dtype=torch.int32, device="cuda")
        ref = torch.empty_like(q)
        ctx.encode_stacks_dev(frames, w, h, stacks, ref)
        variants = [("product", lambda: ctx.encode_stacks_dev(frames, w, h, stacks, q)),
                    ("memonly", lambda: ctx.encode_diag_dev(frames, w, h, stacks, q, 1))]
        for s in strips:
            variants.append((f"strip{s}_mem", lambda s=s: ctx.encode_strip_dev(frames, w, h, stacks, q, 1, s)))
            variants.append((f"strip{s}_enc", lambda s=s: ctx.encode_strip_dev(frames, w, h, stacks, q, 0, s)))
        # the strip encodes write the product's output
        for s in strips:
            ctx.encode_strip_dev(frames, w, h, stacks, q, 0, s)
            torch.cuda.synchronize()
            assert torch.equal(q, ref), f"strip {s}: output differs from the product encode"
        t_end = time.time() + 2.0  # settle (power-management transient)
        while time.time() < t_end:
            ctx.encode_stacks_dev(frames, w, h, stacks, q)
            torch.cuda.synchronize()
        res = {}
        for r in range(a.rounds):
            for label, fn in variants:
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(label, []).append(e0.elapsed_time(e1) / a.reps)
        bytes_step = n * 2560
        out = {"geometry": name, "width": w, "height": h, "stacks": stacks, "cubes": n, "rounds": a.rounds,
               "reps": a.reps, "ms": {k: [round(x, 4) for x in v] for k, v in res.items()},
               "frac_best": {k: round(bytes_step / (min(v) * 1e-3) / 8e12, 4) for k, v in res.items()}}
        print(json.dumps(out), flush=True)
        del frames, q, ref
        torch.cuda.empty_cache()
