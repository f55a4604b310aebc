"""GPU: every entry point of the boundary on frames whose stacks hold odd cube counts.

The host-pointer entry points pipeline their work in chunks of whole stacks (dct3d_runtime.cpp,
run_pipeline: at most half the stacks per chunk), and the device kernels group cubes by waves (4 or 8
cubes), Exp-Golomb segments (8 cubes) and consumer groups (2,048 values).  A stack of 1, 6, 15 or 153
cubes puts chunk starts, wave groups and segment ends everywhere inside those units.  Expected values:
the oracle's quantised cubes (plan.encode_q: the restated Java DCT.java / Encoder.java), its decode
(plan.decode_q: Decoder.java / InverseDCT.java) and its Exp-Golomb writer (ExpGolombWriter.java), at
sizes it finishes in well under a second.  (Round 6: the host stream decode's chunks could start inside a
consumer group -- test_gpu_eg_fused.py::test_host_decode_eg_chunks_on_groups.)"""
import numpy as np
import pytest

from test_gpu_eg import _expected

pytestmark = pytest.mark.gpu

GEOMS = [(8, 8), (24, 16), (40, 24), (136, 72)]  # 1, 6, 15, 153 cubes per stack


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("w,h", GEOMS)
@pytest.mark.parametrize("stacks", [1, 3, 9])
def test_every_entry_point(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, w, h, stacks):
    import torch
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = pkg.synthetic.frames(w, h, stacks * depth, kind="uniform" if stacks == 3 else "ramp", frame0=w + stacks)
    n = ctx.n_cubes(w, h, stacks)
    q = plan.encode_q(fr).reshape(n, depth, 8, 8)
    raster = plan.decode_q(q, w, h, stacks * depth)
    stream, nbits = _expected(oracle, pkg, q, depth, 0x60, 3)  # continuing a partial byte of 3 bits

    # quantised cubes: host pipeline and device
    assert np.array_equal(ctx.encode_stacks(fr), q)
    dq = torch.zeros(n * ctx.cube_size, dtype=torch.int32, device="cuda")
    ctx.encode_stacks_dev(_dev(fr), w, h, stacks, dq)
    ctx.synchronize()
    assert np.array_equal(dq.cpu().numpy().reshape(q.shape), q)

    # raster from cubes: host pipeline and device
    assert np.array_equal(ctx.decode_stacks(q, w, h, stacks), raster)
    dr = torch.zeros((stacks * depth, h, w), dtype=torch.uint8, device="cuda")
    ctx.decode_stacks_dev(_dev(q), w, h, stacks, dr)
    ctx.synchronize()
    assert np.array_equal(dr.cpu().numpy(), raster)

    # Exp-Golomb stream: fused from frames (host and device), two-step from cubes
    got, tb = ctx.encode_eg(fr, 0x60, 3)
    assert tb == nbits and got == stream
    cap = (len(stream) + 64) // 4 * 4
    out = torch.zeros(cap // 4 + 1, dtype=torch.int32, device="cuda")
    tb = ctx.encode_eg_dev(_dev(fr), w, h, stacks, out, cap, 0x60, 3)
    assert tb == nbits and out.cpu().numpy().view(np.uint8)[: len(stream)].tobytes() == stream
    out.zero_()
    tb = ctx.eg_encode_dev(_dev(q), n, out, cap, 0x60, 3)
    assert tb == nbits and out.cpu().numpy().view(np.uint8)[: len(stream)].tobytes() == stream

    # stream -> raster (host and device) and stream -> cubes, from bit 3
    got, eb = ctx.decode_eg(stream, w, h, stacks, start_bit=3)
    assert eb == nbits and np.array_equal(got, raster)
    words = np.zeros((len(stream) + 7) // 4 * 4, np.uint8)
    words[: len(stream)] = np.frombuffer(stream, np.uint8)
    ds = _dev(words)
    dr.zero_()
    eb = ctx.decode_eg_dev(ds, len(stream), 3, w, h, stacks, dr)
    ctx.synchronize()
    assert eb == nbits and np.array_equal(dr.cpu().numpy(), raster)
    dq.zero_()
    eb = ctx.eg_decode_dev(ds, len(stream), 3, n, dq)
    ctx.synchronize()
    assert eb == nbits and np.array_equal(dq.cpu().numpy().reshape(q.shape), q)
