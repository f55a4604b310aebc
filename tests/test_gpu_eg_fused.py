"""GPU: the fused encode + Exp-Golomb path (dct3d_encode_eg_dev).

The stream must be the reference's (encoder.c:206-274 up to the deflate: DCT + quantisation +
diagonal-slice order + signed order-0 Exp-Golomb, one continuous bitstream carrying the partial byte)
bit for bit.  Expected streams: the oracle's quantised cubes (plan.encode_q, the restated Java
DCT.java / Encoder.java) through the oracle's Exp-Golomb writer at sizes the oracle finishes in
seconds, and the two-step device path (dct3d_encode_stacks_dev + dct3d_eg_encode_dev, both pinned
against the oracle in test_gpu_parity.py / test_gpu_eg.py) at 1080p."""
import numpy as np
import pytest

from conftest import ctx_option
from test_gpu_eg import _expected, _gpu_stream

pytestmark = pytest.mark.gpu


def _fused(ctx, fr, carry_byte=0, carry_bits=0, cap=None):
    import torch
    fr = np.ascontiguousarray(fr, np.uint8)
    F, H, W = fr.shape
    d = torch.from_numpy(fr).cuda()
    cap = cap if cap is not None else (fr.size * 4 + 64) // 4 * 4
    out = torch.zeros(cap // 4 + 1, dtype=torch.int32, device="cuda")
    tb = ctx.encode_eg_dev(d, W, H, F // ctx.bd, out, cap, carry_byte, carry_bits)
    raw = out.cpu().numpy().view(np.uint8)
    return raw[: (tb + 7) // 8].tobytes(), tb, raw


def _content(pkg, kind, w, h, f):
    if kind in ("ramp", "uniform"):
        return pkg.synthetic.frames(w, h, f, kind=kind)
    if kind == "zeros":
        return np.zeros((f, h, w), np.uint8)
    if kind == "full":
        return np.full((f, h, w), 255, np.uint8)
    if kind == "checker":   # extreme AC coefficients (largest codes)
        z, y, x = np.indices((f, h, w))
        return (((x + y + z) & 1) * 255).astype(np.uint8)
    if kind == "corner":    # a large DC and first-order coefficients: group 0's halves > 64 bits
        z, y, x = np.indices((f, h, w))
        return np.where((x % 8) + (y % 8) + (z % 8) < 10, 255, 0).astype(np.uint8)
    if kind == "edge":      # group 0's halves of exactly 64 bits at 8x8x4
        z, y, x = np.indices((f, h, w))
        return np.where((x % 8) + (y % 8) + (z % 4) < 5, 255, 0).astype(np.uint8)
    raise ValueError(kind)


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["ramp", "uniform", "zeros", "full", "checker", "corner", "edge"])
def test_fused_matches_oracle(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, kind):
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = _content(pkg, kind, 64, 64, 2 * depth)
    exp, ebits = _expected(oracle, pkg, plan.encode_q(fr), depth)
    got, tb, raw = _fused(ctx, fr)
    assert tb == ebits
    assert got == exp
    assert not raw[len(got):(tb + 31) // 32 * 4].any()      # zero padding to the word


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("w,h,stacks", [(8, 8, 1), (24, 16, 3), (40, 8, 5), (136, 72, 2)])
def test_fused_ragged_segment_tails(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, w, h, stacks):
    """cube counts that are not a multiple of 8: the last wave codes a partial segment"""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = pkg.synthetic.frames(w, h, stacks * depth, kind="uniform", frame0=w + h)
    exp, ebits = _expected(oracle, pkg, plan.encode_q(fr), depth)
    got, tb, _ = _fused(ctx, fr)
    assert tb == ebits and got == exp


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("w,h,stacks", [(8, 8, 1), (40, 8, 5), (136, 72, 2)])
@pytest.mark.parametrize("carry_bits", [0, 3])
def test_fused_ragged_carry_matches_oracle(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, w, h,
                                           stacks, carry_bits):
    """small and ragged inputs (one segment, a partial last segment) continuing a carried partial byte,
    against the oracle's stream; nothing is written past the stream's last word"""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = pkg.synthetic.frames(w, h, stacks * depth, kind="uniform", frame0=w + carry_bits)
    exp, ebits = _expected(oracle, pkg, plan.encode_q(fr), depth, 0x3C, carry_bits)
    got, tb, raw = _fused(ctx, fr, 0x3C, carry_bits)
    assert tb == ebits and got == exp
    assert not raw[len(got):(tb + 31) // 32 * 4].any()


@pytest.mark.parametrize("carry_bits", range(8))
def test_fused_carry_partial_byte(pkg, oracle, plan8, gpu_ctx8, carry_bits):
    fr = pkg.synthetic.frames(48, 40, 8, kind="uniform", frame0=carry_bits)
    exp, ebits = _expected(oracle, pkg, plan8.encode_q(fr), 8, 0x5A, carry_bits)
    got, tb, _ = _fused(gpu_ctx8, fr, 0x5A, carry_bits)
    assert tb == ebits and got == exp


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["ramp", "uniform"])
def test_fused_1080p_matches_two_step(pkg, gpu_ctx8, gpu_ctx4, depth, kind):
    """1080p, 2 stacks: uncertified coefficients (uniform content, 8x8x4 exact ties) replayed inside
    the fused kernel must give the stand-alone encode kernel's values"""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = pkg.synthetic.frames(1920, 1080, 2 * depth, kind=kind)
    q = ctx.encode_stacks(fr)
    ref, rbits, _ = _gpu_stream(ctx, q)
    got, tb, _ = _fused(ctx, fr)
    assert tb == rbits and got == ref


def test_fused_1080p_matches_oracle(pkg, oracle, plan8, gpu_ctx8):
    fr = pkg.synthetic.frames(1920, 1080, 8, kind="ramp", frame0=3)
    exp, ebits = _expected(oracle, pkg, plan8.encode_q(fr), 8)
    got, tb, _ = _fused(gpu_ctx8, fr)
    assert tb == ebits and got == exp


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["uniform", "checker"])
@pytest.mark.parametrize("carry_bits", [0, 5])
def test_fused_matches_two_step_carry(pkg, gpu_ctx8, gpu_ctx4, depth, kind, carry_bits):
    """the fused path (slots + scan + compaction) and the two-step path (int32 cubes, then the
    stand-alone Exp-Golomb stage) write the same stream at 1080p x 3 stacks (~49k segments) with a
    carried partial byte, on uniform noise and on a checkerboard (long codes everywhere)"""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = _content(pkg, kind, 1920, 1080, 3 * depth) if kind != "uniform" else \
        pkg.synthetic.frames(1920, 1080, 3 * depth, kind="uniform", frame0=11)
    tp, ttp, _ = _fused(ctx, fr, 0xA5, carry_bits)
    ref, rbits, _ = _gpu_stream(ctx, ctx.encode_stacks(fr), 0xA5, carry_bits)
    assert ttp == rbits and tp == ref


def test_fused_capacity(pkg, gpu_ctx8):
    fr = pkg.synthetic.frames(64, 64, 8, kind="uniform")
    _, tb, _ = _fused(gpu_ctx8, fr)
    import torch
    d = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    small = (tb // 32) * 4 - 4          # one word short
    out = torch.full((small // 4 + 4,), 7, dtype=torch.int32, device="cuda")
    with pytest.raises(pkg.Dct3dError) as ei:
        gpu_ctx8.encode_eg_dev(d, 64, 64, 1, out, small)
    assert ei.value.code == pkg.DCT3D_ENOSPC
    o = out.cpu().numpy()
    assert (o == 7).all()                          # nothing written at all
    got, tb2, _ = _fused(gpu_ctx8, fr, cap=(tb + 31) // 32 * 4)   # exactly enough
    assert tb2 == tb


def test_fused_empty_and_errors(pkg, gpu_ctx8):
    import torch
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    assert gpu_ctx8.encode_eg_dev(d, 8, 8, 0, out, 16, 0xF0, 4) == 4
    assert out.cpu().numpy().view(np.uint8)[0] == 0xF0
    with pytest.raises(pkg.Dct3dError):
        gpu_ctx8.encode_eg_dev(d, 12, 8, 1, out, 16)     # width not a multiple of the block width


@pytest.mark.parametrize("depth", [8, 4])
def test_host_encode_eg_is_fused_and_identical(pkg, gpu_ctx8, gpu_ctx4, depth):
    """dct3d_encode_eg (host raster in) now runs the fused path; its stream equals the two-step one"""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = pkg.synthetic.frames(320, 240, 3 * depth, kind="ramp", frame0=11)
    q = ctx.encode_stacks(fr)
    ref, rbits, _ = _gpu_stream(ctx, q, 0x80, 1)
    got, tb = ctx.encode_eg(fr, 0x80, 1)
    assert tb == rbits and got == ref


# ------------------------------------------------------------------------------------------------
# fused stream -> raster decode (dct3d_decode_eg_dev)
# ------------------------------------------------------------------------------------------------
def _stream_dev(data: bytes):
    import torch
    n = (len(data) + 3) // 4 + 1
    buf = np.zeros(n * 4, np.uint8)
    buf[: len(data)] = np.frombuffer(data, np.uint8)
    return torch.from_numpy(buf).cuda()


def _decode_fused(ctx, data: bytes, w, h, stacks, start_bit=0):
    import torch
    d = _stream_dev(data)
    out = torch.empty((stacks * ctx.bd, h, w), dtype=torch.uint8, device="cuda")
    eb = ctx.decode_eg_dev(d, len(data), start_bit, w, h, stacks, out)
    return out.cpu().numpy(), eb


def _decode_two_step(ctx, data: bytes, w, h, stacks, start_bit=0):
    import torch
    d = _stream_dev(data)
    n = ctx.n_cubes(w, h, stacks)
    q = torch.empty(n * ctx.cube_size, dtype=torch.int32, device="cuda")
    eb = ctx.eg_decode_dev(d, len(data), start_bit, n, q)
    out = torch.empty((stacks * ctx.bd, h, w), dtype=torch.uint8, device="cuda")
    ctx.decode_stacks_dev(q, w, h, stacks, out)
    ctx.synchronize()  # *_dev calls are asynchronous on the context stream
    return out.cpu().numpy(), eb


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["ramp", "uniform"])
def test_fused_decode_1080p_matches_two_step(pkg, gpu_ctx8, gpu_ctx4, depth, kind):
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = pkg.synthetic.frames(1920, 1080, 2 * depth, kind=kind, frame0=5)
    data, tb = ctx.encode_eg(fr)
    ref, reb = _decode_two_step(ctx, data, 1920, 1080, 2)
    got, eb = _decode_fused(ctx, data, 1920, 1080, 2)
    assert eb == reb == tb
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("own_stream", [True, False])
def test_fused_encode_back_to_back(pkg, gpu_ctx8, own_stream):
    """dct3d_encode_eg_dev returns once the total is known, the compaction and the stitch still running:
    calls queued back to back (alternating contents and outputs, the last call again into the first
    output) each land their own stream, on the context's own stream and on a shared framework stream"""
    import torch
    fr = [pkg.synthetic.frames(1920, 1080, 2 * 8, kind=k, frame0=f) for k, f in (("ramp", 4), ("uniform", 8))]
    refs = [gpu_ctx8.encode_eg(x) for x in fr]
    ctx = pkg.Context(0, 8, 8, 8)
    try:
        st = None if own_stream else torch.cuda.Stream()
        if st is not None:
            ctx.set_stream(st.cuda_stream)
        ds = [torch.from_numpy(x).cuda() for x in fr]
        cap = fr[0].size * 2
        outs = [torch.zeros(cap // 4, dtype=torch.int32, device="cuda") for _ in range(3)]
        torch.cuda.synchronize()
        with torch.cuda.stream(st) if st is not None else torch.cuda.stream(torch.cuda.current_stream()):
            for k, o in [(0, 0), (1, 1), (0, 2), (1, 0)]:
                assert ctx.encode_eg_dev(ds[k], 1920, 1080, 2, outs[o], cap) == refs[k][1]
            got = [x.cpu().numpy().view(np.uint8) for x in outs]
        for o, k in ((0, 1), (1, 1), (2, 0)):
            assert got[o][: len(refs[k][0])].tobytes() == refs[k][0]
    finally:
        ctx.close()


@pytest.mark.parametrize("own_stream", [True, False])
def test_fused_decode_back_to_back(pkg, gpu_ctx8, own_stream):
    """dct3d_decode_eg_dev returns once the verdict is known, with the consumer still running on the
    stream: calls queued back to back (no synchronisation between them, alternating contents and
    outputs, the last call again into the first output) each land their own raster -- on the context's own
    stream and on a framework stream shared through set_stream"""
    import torch
    fr = [pkg.synthetic.frames(1920, 1080, 2 * 8, kind=k, frame0=f) for k, f in (("ramp", 3), ("uniform", 9))]
    enc = [gpu_ctx8.encode_eg(x) for x in fr]
    refs = [_decode_two_step(gpu_ctx8, d, 1920, 1080, 2)[0] for d, _ in enc]
    ctx = pkg.Context(0, 8, 8, 8)
    try:
        st = None if own_stream else torch.cuda.Stream()
        if st is not None:
            ctx.set_stream(st.cuda_stream)
        ds = [_stream_dev(d) for d, _ in enc]
        outs = [torch.empty((16, 1080, 1920), dtype=torch.uint8, device="cuda") for _ in range(3)]
        torch.cuda.synchronize()
        order = [(0, 0), (1, 1), (0, 2), (1, 0)]  # (content, output): output 0 is written twice
        with torch.cuda.stream(st) if st is not None else torch.cuda.stream(torch.cuda.current_stream()):
            for k, o in order:
                assert ctx.decode_eg_dev(ds[k], len(enc[k][0]), 0, 1920, 1080, 2, outs[o]) == enc[k][1]
            got = [x.cpu().numpy() for x in outs]  # on the decode's stream (st) or the legacy default one
        assert np.array_equal(got[0], refs[1]) and np.array_equal(got[1], refs[1]) and np.array_equal(got[2], refs[0])
    finally:
        ctx.close()


def test_fused_decode_queue_stress(pkg, gpu_ctx8):
    """Many calls queued behind running consumers (the host runs a call ahead of the device): two different
    1080p streams of 16 stacks alternate over 12 calls into 12 outputs -- each call's scan, marks and
    consumer must see only its own stream's values (stale values of the other stream would decode to
    garbage)"""
    import torch
    fr = [pkg.synthetic.frames(1920, 1080, 16 * 8, kind=k, frame0=f) for k, f in (("ramp", 2), ("uniform", 6))]
    enc = [gpu_ctx8.encode_eg(x) for x in fr]
    refs = [_decode_two_step(gpu_ctx8, d, 1920, 1080, 16)[0] for d, _ in enc]
    ds = [_stream_dev(d) for d, _ in enc]
    outs = [torch.empty((128, 1080, 1920), dtype=torch.uint8, device="cuda") for _ in range(12)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        k = i % 2
        assert gpu_ctx8.decode_eg_dev(ds[k], len(enc[k][0]), 0, 1920, 1080, 16, o) == enc[k][1]
    gpu_ctx8.synchronize()
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy(), refs[i % 2]), f"call {i}"


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["ramp", "uniform", "checker", "full"])
def test_fused_decode_matches_oracle(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, kind):
    """stream of the oracle's cubes -> fused decode == the oracle's Java-semantics decode of the cubes"""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = _content(pkg, kind, 64, 48, 2 * depth)
    q = plan.encode_q(fr)
    data, nbits = _expected(oracle, pkg, q, depth, 0xC0, 3)    # starts at bit 3 of a carried byte
    got, eb = _decode_fused(ctx, data, 64, 48, 2, start_bit=3)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, 64, 48, 2 * depth))


def test_fused_decode_whole_cube_replay_from_stream(pkg, gpu_ctx8):
    """a widened certification margin sends cubes to the replay, which re-parses them from the stream"""
    fr = pkg.synthetic.frames(256, 128, 16, kind="uniform", frame0=9)
    data, _ = gpu_ctx8.encode_eg(fr)
    ref, _ = _decode_two_step(gpu_ctx8, data, 256, 128, 2)
    with ctx_option(gpu_ctx8, pkg.DCT3D_OPT_DEC_MARGIN, 0.45):
        got, _ = _decode_fused(gpu_ctx8, data, 256, 128, 2)
        assert gpu_ctx8.stats()["n_flagged"] > 0   # the replay path ran
    assert np.array_equal(got, ref)


def test_fused_decode_truncated_and_corrupt(pkg, gpu_ctx8):
    fr = pkg.synthetic.frames(128, 64, 16, kind="uniform", frame0=2)
    data, _ = gpu_ctx8.encode_eg(fr)
    with pytest.raises(pkg.Dct3dError) as e:
        _decode_fused(gpu_ctx8, data[: len(data) // 2], 128, 64, 2)
    assert e.value.code == pkg.DCT3D_ENODATA
    got, _ = _decode_fused(gpu_ctx8, data[: len(data) // 2 + len(data) // 8], 128, 64, 1)   # one stack is there
    ref, _ = _decode_two_step(gpu_ctx8, data, 128, 64, 1)
    assert np.array_equal(got, ref)
    bad = bytearray(data)
    bad[len(bad) // 3: len(bad) // 3 + 6] = bytes(6)                    # 48 zero bits: no valid code
    with pytest.raises(pkg.Dct3dError) as e:
        _decode_fused(gpu_ctx8, bytes(bad), 128, 64, 2)
    assert e.value.code in (pkg.DCT3D_EINVAL, pkg.DCT3D_ENODATA)


@pytest.mark.parametrize("depth", [8, 4])
def test_fused_decode_dense_long_codes(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth):
    """Streams no encoder of 8-bit frames writes (|q| >= 2^24: 49..61-bit codes everywhere) decode to the
    Java-semantics raster (out-of-range q: whole-cube replay) -- no silently truncated window."""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    rng = np.random.default_rng(11 + depth)
    n = ctx.n_cubes(64, 48, 2)
    q = rng.integers(2**24, 2**30, size=(n, depth, 8, 8)) * rng.choice([-1, 1], size=(n, depth, 8, 8))
    q = q.astype(np.int32)
    q[::3] = rng.integers(-20, 21, size=q[::3].shape)  # ordinary cubes between them
    data, nbits = _expected(oracle, pkg, q, depth)
    got, eb = _decode_fused(ctx, data, 64, 48, 2)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, 64, 48, 2 * depth))


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("with_long", [False, True])
def test_fused_decode_sparse_long_codes(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, with_long):
    """The consumer's parse steps take codes of <= 31 bits unchecked unless the mark pass saw a longer one
    (status[3]): a few 33..41-bit codes (|q| = 2^15 .. 2^20) among ordinary values, in windows that fit
    the LDS, flag the stream and are parsed by the checking steps; |q| = 2^15 - 1 (31 bits, the widest
    code of the unchecked steps) is parsed by either.  Both give the Java-semantics raster."""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    rng = np.random.default_rng(21 + depth + 2 * with_long)
    n = ctx.n_cubes(256, 128, 2)
    q = rng.integers(-20, 21, size=(n, depth, 8, 8))
    q[rng.random(q.shape) < 0.5] = 0
    sgn = rng.choice([-1, 1], size=q.shape)
    edge = rng.random(q.shape) < 0.002
    q[edge] = (2**15 - 1) * sgn[edge]
    if with_long:
        big = rng.random(q.shape) < 0.001
        q[big] = rng.integers(2**15, 2**20, size=int(big.sum())) * sgn[big]
        q[0, 0, 0, 0] = 2**15  # the narrowest long code, 33 bits
    q = q.astype(np.int32)
    data, nbits = _expected(oracle, pkg, q, depth)
    got, eb = _decode_fused(ctx, data, 256, 128, 2)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, 256, 128, 2 * depth))
    qd, eb2 = _eg_decode_q(ctx, data, n)  # the stream -> int32 path (eg_emit_kernel) parses the same way
    assert eb2 == nbits and np.array_equal(qd, q)


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("lo", [15, 19])
def test_fused_decode_long_codes_everywhere_in_window(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, lo):
    """Every value a long code.  lo = 15: 33-bit codes (|q| in [2^15, 2^16)), a consumer group's 2,048
    values span ~67.6 k bits, wider than 2^16 (the 16-bit marks wrap inside the group: mark_offset) and
    still inside the consumer's LDS window -- the flagged (checking) parse steps in the window, marks far
    apart, and the exact replay of every cube (out-of-range coefficients), which re-reads its values from
    the stream at the marks (mark_serial).  lo = 19: 39..41-bit codes, ~82 k bits per group, past the
    window: the parse from global memory at the rebuilt marks."""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    rng = np.random.default_rng(31 + depth + lo)
    n = ctx.n_cubes(64, 48, 2)
    q = rng.integers(2**lo, 2**(lo + 1), size=(n, depth, 8, 8)) * rng.choice([-1, 1], size=(n, depth, 8, 8))
    q = q.astype(np.int32)
    data, nbits = _expected(oracle, pkg, q, depth)
    got, eb = _decode_fused(ctx, data, 64, 48, 2)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, 64, 48, 2 * depth))
    qd, eb2 = _eg_decode_q(ctx, data, n)
    assert eb2 == nbits and np.array_equal(qd, q)


def _eg_decode_q(ctx, data: bytes, n_cubes: int):
    import torch
    d = _stream_dev(data)
    dq = torch.zeros(n_cubes * ctx.cube_size, dtype=torch.int32, device="cuda")
    eb = ctx.eg_decode_dev(d, len(data), 0, n_cubes, dq)
    ctx.synchronize()
    return dq.cpu().numpy().reshape(n_cubes, ctx.bd, 8, 8), eb


@pytest.mark.parametrize("fused", [0, 1])
def test_speculative_front_rerun_on_unresolved_pass0(pkg, oracle, plan8, gpu_ctx8, fused):
    """The stream decode enqueues its front (the resolving sync pass, the scan and the mark pass; or, as
    an option, the fused eg_front_kernel) and the consumer without a host round trip; should pass 0 not resolve, no
    marks are written, the consumer skips itself and the call reruns without speculation.
    DCT3D_OPT_EG_FORCE_RETRY forces that verdict: the three entry points (two-step, fused device, fused
    host) give the same results and errors."""
    fr = pkg.synthetic.frames(128, 64, 24, kind="uniform", frame0=4)
    q = plan8.encode_q(fr)
    data, nbits = _expected(oracle, pkg, q, 8)
    ref_fused, eb0 = _decode_fused(gpu_ctx8, data, 128, 64, 3)
    ref_two, eb1 = _decode_two_step(gpu_ctx8, data, 128, 64, 3)
    ref_host, eb2 = gpu_ctx8.decode_eg(data, 128, 64, 3)
    with ctx_option(gpu_ctx8, pkg.DCT3D_OPT_EG_FORCE_RETRY, 1), ctx_option(gpu_ctx8, pkg.DCT3D_OPT_EG_FUSED_FRONT, fused):
        got_fused, e0 = _decode_fused(gpu_ctx8, data, 128, 64, 3)
        got_two, e1 = _decode_two_step(gpu_ctx8, data, 128, 64, 3)
        got_host, e2 = gpu_ctx8.decode_eg(data, 128, 64, 3)
        with pytest.raises(pkg.Dct3dError) as e:
            _decode_fused(gpu_ctx8, data[: len(data) // 2], 128, 64, 3)
        assert e.value.code == pkg.DCT3D_ENODATA
    assert eb0 == eb1 == e0 == e1 == nbits and eb2 == e2
    expect = plan8.decode_q(q, 128, 64, 24)
    for got in (ref_fused, ref_two, ref_host, got_fused, got_two, got_host):
        assert np.array_equal(got, expect)


@pytest.mark.parametrize("groups", [1, 2, 4, 8])
@pytest.mark.parametrize("depth", [8, 4])
def test_fused_decode_groups_per_wave(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, groups):
    """decode_eg_kernel runs `groups` rounds of 4 consecutive groups (2,048 values each) per block, the
    next group's marks and window words in flight during the current one (DCT3D_OPT_EG_DEC_GROUPS; 0 =
    8).  The same raster for every setting: 1080p uniform content (windows longer than the look-ahead
    words), ragged frames (partial blocks: waves leaving the loop early, per-lane stores), dense long
    codes (windows that do not fit the LDS: the global-memory parse)."""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    cases = [(1920, 1080, 2, "uniform"), (136, 72, 2, "ramp"), (24, 16, 3, "uniform")]
    for w, h, stacks, kind in cases:
        fr = pkg.synthetic.frames(w, h, stacks * depth, kind=kind, frame0=3)
        data, tb = ctx.encode_eg(fr)
        ref, reb = _decode_two_step(ctx, data, w, h, stacks)
        with ctx_option(ctx, pkg.DCT3D_OPT_EG_DEC_GROUPS, groups):
            got, eb = _decode_fused(ctx, data, w, h, stacks)
        assert eb == reb == tb
        assert np.array_equal(got, ref), (w, h, kind)
    rng = np.random.default_rng(5 + depth)
    n = ctx.n_cubes(64, 48, 2)
    q = (rng.integers(2**24, 2**30, size=(n, depth, 8, 8)) * rng.choice([-1, 1], size=(n, depth, 8, 8))).astype(np.int32)
    q[::2] = rng.integers(-9, 10, size=q[::2].shape)
    data, nbits = _expected(oracle, pkg, q, depth)
    with ctx_option(ctx, pkg.DCT3D_OPT_EG_DEC_GROUPS, groups):
        got, eb = _decode_fused(ctx, data, 64, 48, 2)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, 64, 48, 2 * depth))


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("w,h", [(8, 8), (16, 8), (24, 8), (16, 16)])
def test_fused_decode_tiny_frames(pkg, oracle, plan8, plan4, gpu_ctx8, gpu_ctx4, depth, w, h):
    """1 to 4 cubes: one partial consumer group, waves (and look-ahead groups) past the last mark group,
    whose mark_base entry does not exist and must not be read; both consumers."""
    ctx, plan = (gpu_ctx8, plan8) if depth == 8 else (gpu_ctx4, plan4)
    fr = pkg.synthetic.frames(w, h, depth, kind="uniform", frame0=w * h + depth)
    q = plan.encode_q(fr)
    data, nbits = _expected(oracle, pkg, q, depth)
    got, eb = _decode_fused(ctx, data, w, h, 1)
    assert eb == nbits
    assert np.array_equal(got, plan.decode_q(q, w, h, depth))
    n = ctx.n_cubes(w, h, 1)
    qd, eb2 = _eg_decode_q(ctx, data, n)
    assert eb2 == nbits and np.array_equal(qd, q.reshape(n, depth, 8, 8))


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("kind", ["ramp", "uniform"])
def test_fused_front_option_same_results(pkg, gpu_ctx8, gpu_ctx4, depth, kind):
    """DCT3D_OPT_EG_FUSED_FRONT: the one-launch front (eg_front_kernel: resolve, block scan, decoupled
    look-back, marks) gives the three-launch front's raster and end bit at 1080p (~22 k look-back blocks
    per call), through both consumers."""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = pkg.synthetic.frames(1920, 1080, 2 * depth, kind=kind, frame0=7)
    data, tb = ctx.encode_eg(fr)
    ref, reb = _decode_fused(ctx, data, 1920, 1080, 2)
    qref, qeb = _eg_decode_q(ctx, data, ctx.n_cubes(1920, 1080, 2))
    with ctx_option(ctx, pkg.DCT3D_OPT_EG_FUSED_FRONT, 1):
        got, eb = _decode_fused(ctx, data, 1920, 1080, 2)
        qgot, qeb2 = _eg_decode_q(ctx, data, ctx.n_cubes(1920, 1080, 2))
    assert eb == reb == tb == qeb == qeb2
    assert np.array_equal(got, ref) and np.array_equal(qgot, qref)


@pytest.mark.parametrize("depth", [8, 4])
@pytest.mark.parametrize("w,h,stacks", [(136, 72, 3), (24, 16, 5), (8, 8, 9)])
def test_host_decode_eg_chunks_on_groups(pkg, gpu_ctx8, gpu_ctx4, depth, w, h, stacks):
    """The host-pointer stream decode (dct3d_decode_eg) runs the consumer in chunks of stacks; a chunk must
    start on a consumer group (2,048 values): with stacks of 153, 6 or 1 cubes, chunks of a multiple of
    4 / 2 / 4 stacks (8x8x4: 8 / 4 / 8).  Same raster and end bit as the two-step path (round 6: a chunk
    starting inside a group parsed past its window)."""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    fr = pkg.synthetic.frames(w, h, stacks * depth, kind="ramp", frame0=13)
    data, tb = ctx.encode_eg(fr)
    ref, reb = _decode_two_step(ctx, data, w, h, stacks)
    got, eb = ctx.decode_eg(data, w, h, stacks)
    assert eb == reb == tb
    assert np.array_equal(got, ref)
