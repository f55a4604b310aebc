"""Bandwidth-probe sweep (run on the GPU box): achievable HBM rates per mode and grid size."""
import importlib, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("3ddctvideoencoding_amd")
ctx = pkg.Context(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s); ctx.set_stream(s.cuda_stream)
n = 128 * 1920 * 1080 * 8
src = torch.empty(n, dtype=torch.uint8, device="cuda"); dst = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
ctx.fill_synthetic_dev(src, 1920, 1080, 128 * 8)
res = {}
for mode, name, bpp in ((0, "mix_nt", 5), (1, "copy_nt", 2), (4, "copy_plain", 2), (2, "write_nt", 4), (5, "write_plain", 4), (3, "read", 1)):
    ctx.bandwidth_probe_dev(src, dst, n, mode); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): ctx.bandwidth_probe_dev(src, dst, n, mode)
    e1.record(); torch.cuda.synchronize()
    res[name] = round(n * bpp / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9, 1)
print(os.environ.get("DCT3D_PROBE_GRID", "2048"), json.dumps(res))
