"""Experiment: launch cost of the small kernels (run under rocprofv3 --kernel-trace on the GPU box)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("3ddctvideoencoding_amd")
ctx = pkg.Context(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s); ctx.set_stream(s.cuda_stream)
fr = torch.zeros((8, 8, 64), dtype=torch.uint8, device="cuda")
q = torch.zeros(8 * 8 * 64, dtype=torch.int32, device="cuda")
out = torch.empty_like(fr)
for _ in range(20):                      # tiny decode, tiny encode
    ctx.decode_stacks_dev(q, 64, 8, 1, out)
    ctx.encode_stacks_dev(fr, 64, 8, 1, q)
buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
dst = torch.zeros(4 << 20, dtype=torch.uint8, device="cuda")
for _ in range(20):
    ctx.bandwidth_probe_dev(buf, dst, 16, 3)   # empty-ish probe launch (grid from env)
torch.cuda.synchronize()
print("ok")
