"""GPU: the device Exp-Golomb stage against the oracle's Java-semantics writer.

The reference stream: every cube's values in diagonal-slice order (CubeUtils.c:5-46), signed order-0
Exp-Golomb (ExpGolomb.c:32-64 == ExpGolombWriter.java:19-49, pinned against the reference's own C
writer in test_oracle.py), MSB first, one continuous bitstream across cubes and stacks (the partial
byte is carried, ExpGolomb.c:112-130).  Bit-exact comparisons only."""
import numpy as np
import pytest

from conftest import ctx_option

pytestmark = pytest.mark.gpu


def _frames(pkg, w, h, f, kind="ramp", frame0=0):
    return pkg.synthetic.frames(w, h, f, kind=kind, frame0=frame0)


def _code_bits(v: np.ndarray) -> int:
    v = v.astype(np.int64)
    code = np.where(v <= 0, -2 * v, 2 * v - 1) + 1
    n = np.floor(np.log2(code.astype(np.float64))).astype(np.int64) + 1
    return int((2 * n - 1).sum())


def _expected(oracle, pkg, q: np.ndarray, depth: int, carry_byte=0, carry_bits=0):
    """(expected stream bytes, total bits) for cube-major q continuing a partial byte."""
    cs = 64 * depth
    vals = q.reshape(-1, cs)[:, pkg.diagonal_order(8, 8, depth)].ravel()
    nbits = _code_bits(vals)
    body = np.unpackbits(np.frombuffer(oracle.eg_write(vals), np.uint8))[:nbits]
    pre = np.unpackbits(np.array([carry_byte], np.uint8))[:carry_bits]
    bits = np.concatenate([pre, body])
    return np.packbits(bits).tobytes(), carry_bits + nbits


def _gpu_stream(ctx, q: np.ndarray, carry_byte=0, carry_bits=0, cap=None):
    import torch
    dq = torch.from_numpy(np.ascontiguousarray(q, np.int32)).cuda()
    n = q.size // ctx.cube_size
    cap = cap if cap is not None else (q.size * 8 + 64) // 4 * 4
    out = torch.zeros(cap // 4 + 1, dtype=torch.int32, device="cuda")
    tb = ctx.eg_encode_dev(dq, n, out, cap, carry_byte, carry_bits)
    raw = out.cpu().numpy().view(np.uint8)
    return raw[: (tb + 7) // 8].tobytes(), tb, raw


@pytest.mark.parametrize("depth,kind", [(8, "ramp"), (8, "uniform"), (4, "ramp")])
def test_eg_encoder_output_matches_oracle(pkg, oracle, gpu_ctx8, gpu_ctx4, depth, kind):
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    q = ctx.encode_stacks(_frames(pkg, 1920, 1080, depth, kind))
    exp, ebits = _expected(oracle, pkg, q, depth)
    got, tb, raw = _gpu_stream(ctx, q)
    assert tb == ebits
    assert got == exp
    assert not raw[len(got):(tb + 31) // 32 * 4].any()      # zero padding to the word


@pytest.mark.parametrize("n_cubes", [1, 3, 4095, 4097, 9000])
def test_eg_random_values_and_chunk_edges(pkg, oracle, gpu_ctx8, n_cubes):
    rng = np.random.default_rng(n_cubes)
    q = rng.integers(-40, 41, size=(n_cubes, 8, 8, 8)).astype(np.int32)
    q[rng.random(q.shape) < 0.6] = 0
    big = rng.random(q.shape) < 0.002
    q[big] = rng.integers(-(2**30) + 1, 2**30, size=int(big.sum()))
    q.reshape(-1)[:4] = [2**30 - 1, -(2**30) + 1, 0, 1]
    if n_cubes > 2:   # cubes whose codes exceed the writer's LDS image (8,160 bits): global-atomic path
        q[1] = rng.integers(2**28, 2**30, size=(8, 8, 8)) * rng.choice([-1, 1], size=(8, 8, 8))
        q[2, :4] = rng.integers(-(2**20), 2**20, size=(4, 8, 8))
    exp, ebits = _expected(oracle, pkg, q, 8)
    got, tb, _ = _gpu_stream(gpu_ctx8, q)
    assert tb == ebits and got == exp


@pytest.mark.parametrize("carry_bits", range(8))
def test_eg_carry_partial_byte(pkg, oracle, gpu_ctx8, carry_bits):
    rng = np.random.default_rng(100 + carry_bits)
    q = rng.integers(-9, 10, size=(37, 8, 8, 8)).astype(np.int32)
    carry_byte = 0xA5
    exp, ebits = _expected(oracle, pkg, q, 8, carry_byte, carry_bits)
    got, tb, _ = _gpu_stream(gpu_ctx8, q, carry_byte, carry_bits)
    assert tb == ebits and got == exp


def test_eg_capacity_and_range_errors(pkg, oracle, gpu_ctx8):
    rng = np.random.default_rng(9)
    q = rng.integers(-300, 300, size=(64, 8, 8, 8)).astype(np.int32)
    _, ebits = _expected(oracle, pkg, q, 8)
    with pytest.raises(pkg.Dct3dError) as e:
        _gpu_stream(gpu_ctx8, q, cap=64)
    assert e.value.code == pkg.DCT3D_ENOSPC
    got, tb, _ = _gpu_stream(gpu_ctx8, q, cap=(ebits + 31) // 32 * 4)   # exactly enough words
    assert tb == ebits and got == _expected(oracle, pkg, q, 8)[0]
    q[3, 1, 2, 3] = 2**30
    with pytest.raises(pkg.Dct3dError) as e:
        _gpu_stream(gpu_ctx8, q)
    assert e.value.code == pkg.DCT3D_EINVAL


@pytest.mark.parametrize("depth", [8, 4])
def test_encode_eg_batches_chain_like_one_stream(pkg, oracle, plan8, plan4, depth):
    """Host raster -> device DCT + quantisation + Exp-Golomb in two batches, the partial byte carried
    from the first to the second: the same stream as one call, and as the oracle's."""
    with pkg.Context(0, 8, 8, depth) as ctx:
        fr = _frames(pkg, 64, 48, depth * 5, "uniform")
        whole, tb_whole = ctx.encode_eg(fr)
        a, tba = ctx.encode_eg(fr[: depth * 2])
        b, tbb = ctx.encode_eg(fr[depth * 2:], carry_byte=a[-1] if tba % 8 else 0, carry_bits=tba % 8)
        chained = a[: tba // 8] + b
        assert tba + tbb - tba % 8 == tb_whole
        assert chained == whole
        q = (plan8 if depth == 8 else plan4).encode_q(fr)
        exp, ebits = _expected(oracle, pkg, q, depth)
        assert tb_whole == ebits and whole == exp


# ------------------------------------------------------------------------------------------------
# decode (expGolomb_readValue / ExpGolombReader.java; Decoder.java:78-96 diagonal placement)
# ------------------------------------------------------------------------------------------------
def _dev_bytes(data: bytes):
    import torch
    pad = (-len(data)) % 4 + 8
    return torch.from_numpy(np.frombuffer(data + bytes(pad), np.uint8).copy()).cuda()


def _eg_decode(ctx, data: bytes, n_cubes: int, start_bit: int = 0):
    import torch
    dq = torch.zeros(n_cubes * ctx.cube_size, dtype=torch.int32, device="cuda")
    eb = ctx.eg_decode_dev(_dev_bytes(data), len(data), start_bit, n_cubes, dq)
    return dq.cpu().numpy().reshape(n_cubes, ctx.bd, 8, 8), eb


@pytest.mark.parametrize("depth,kind", [(8, "ramp"), (8, "uniform"), (4, "ramp")])
def test_eg_decode_round_trip_1080p(pkg, oracle, gpu_ctx8, gpu_ctx4, depth, kind):
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    q = ctx.encode_stacks(_frames(pkg, 1920, 1080, depth, kind))
    data, nbits = _expected(oracle, pkg, q, depth)          # the oracle's (Java writer's) bytes
    got, eb = _eg_decode(ctx, data, q.shape[0])
    assert eb == nbits and np.array_equal(got, q)


@pytest.mark.parametrize("n_cubes", [1, 5, 3000])
def test_eg_decode_large_values_and_start_bits(pkg, oracle, gpu_ctx8, n_cubes):
    rng = np.random.default_rng(7 + n_cubes)
    q = rng.integers(-60, 61, size=(n_cubes, 8, 8, 8)).astype(np.int32)
    q[rng.random(q.shape) < 0.5] = 0
    big = rng.random(q.shape) < 0.01
    q[big] = rng.integers(-(2**30) + 1, 2**30, size=int(big.sum()))      # long codes (up to 61 bits)
    for start_bit in (0, 3, 7):
        data, nbits = _expected(oracle, pkg, q, 8, 0x5A, start_bit)
        got, eb = _eg_decode(gpu_ctx8, data + bytes(9), n_cubes, start_bit)  # trailing bytes are ignored
        assert eb == nbits and np.array_equal(got, q), start_bit


def test_eg_decode_truncated_and_corrupt(pkg, oracle, gpu_ctx8):
    rng = np.random.default_rng(12)
    q = rng.integers(-20, 21, size=(40, 8, 8, 8)).astype(np.int32)
    data, nbits = _expected(oracle, pkg, q, 8)
    with pytest.raises(pkg.Dct3dError) as e:
        _eg_decode(gpu_ctx8, data[: len(data) // 2], 40)
    assert e.value.code == pkg.DCT3D_ENODATA
    got, eb = _eg_decode(gpu_ctx8, data[: len(data) // 2], 15)          # what is there decodes
    assert np.array_equal(got, q[:15])
    bad = bytearray(data)
    bad[len(bad) // 3: len(bad) // 3 + 6] = bytes(6)                    # 48 zero bits: no valid code
    with pytest.raises(pkg.Dct3dError) as e:
        _eg_decode(gpu_ctx8, bytes(bad), 40)
    assert e.value.code in (pkg.DCT3D_EINVAL, pkg.DCT3D_ENODATA)


@pytest.mark.parametrize("depth", [8, 4])
def test_decode_eg_host_path_and_batches(pkg, oracle, plan8, plan4, depth):
    """Host stream -> device entropy decode + dequantise + IDCT, in two batches continuing at the end
    bit of the first: the frames equal the Java-semantics decode of the encoder's coefficients."""
    plan = plan8 if depth == 8 else plan4
    with pkg.Context(0, 8, 8, depth) as ctx:
        fr = _frames(pkg, 64, 48, depth * 5, "uniform")
        stream, tb = ctx.encode_eg(fr)
        a, ea = ctx.decode_eg(stream, 64, 48, 2)
        b, eb = ctx.decode_eg(stream[ea // 8:], 64, 48, 3, start_bit=ea % 8)
        assert ea // 8 * 8 + eb == tb
        q = plan.encode_q(fr)
        assert np.array_equal(np.concatenate([a, b]), plan.decode_q(q, 64, 48, depth * 5))


@pytest.mark.parametrize("confirm", [False, True])
@pytest.mark.parametrize("big_frac", [0.0, 0.02])
def test_eg_decode_resolve_and_confirming_passes(pkg, oracle, gpu_ctx8, confirm, big_frac):
    """Pass 0 with the in-block resolve (each chunk's true parse walked beside its pass-0 parse until
    they meet) and the plain confirming passes (DCT3D_EG_NO_RESOLVE) give the same values.  With long
    codes (|v| up to 2^30: 61-bit codes) some chunks do not meet within the 128-bit walk: their inline
    re-parse runs, and where a chunk's true exit differs from its pass-0 exit the host's confirming
    passes follow."""
    rng = np.random.default_rng(99)
    q = rng.integers(-30, 31, size=(2500, 8, 8, 8)).astype(np.int32)
    q[rng.random(q.shape) < 0.6] = 0
    big = rng.random(q.shape) < big_frac
    q[big] = rng.integers(-(2**30) + 1, 2**30, size=int(big.sum()))
    data, nbits = _expected(oracle, pkg, q, 8)
    with ctx_option(gpu_ctx8, pkg.DCT3D_OPT_EG_NO_RESOLVE, 1 if confirm else 0):
        got, eb = _eg_decode(gpu_ctx8, data, q.shape[0])
    assert eb == nbits and np.array_equal(got, q)


@pytest.mark.parametrize("depth", [8, 4])
def test_eg_decode_dense_long_codes(pkg, oracle, gpu_ctx8, gpu_ctx4, depth):
    """Every value a 49..61-bit code: one consumer wave's 2,048 values span ~120 k bits, more than its
    LDS window holds -- the window must not silently truncate the parse."""
    ctx = gpu_ctx8 if depth == 8 else gpu_ctx4
    rng = np.random.default_rng(7 + depth)
    n = 4096 // (64 * depth) * 3 + 1  # three waves' worth + a ragged cube
    q = rng.integers(2**24, 2**30, size=(n, depth, 8, 8)) * rng.choice([-1, 1], size=(n, depth, 8, 8))
    q = q.astype(np.int32)
    q[0, 0, :2] = 0  # a few short codes among them
    data, nbits = _expected(oracle, pkg, q, depth)
    got, eb = _eg_decode(ctx, data, n)
    assert eb == nbits and np.array_equal(got, q)
