"""CPU: the fused encoder's certify-or-replay scheme, checked through a host emulation of the
kernel's exact fp32 arithmetic (tests/native/emulate_encode.cpp: the same butterfly source as the
kernel, same order, -ffp-contract=off).

  * soundness: every coefficient the emulated kernel does NOT flag already equals the oracle (Java
    semantics); flagged ones are replayed by the exact fold on the device (test_gpu_parity.py);
  * the rigorous per-coefficient bound (dct3d_plan.cpp, Tracked analysis) dominates the observed
    fp32 error on random, extreme and structured inputs;
  * the flag rate stays small (performance, not correctness).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "native", "emulate_encode.cpp")


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    out = tmp_path_factory.mktemp("emu") / "libemu.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-shared", "-fPIC",
                    "-I", os.path.join(REPO, "3ddctvideoencoding_amd", "csrc"), SRC, "-o", str(out)], check=True)
    L = C.CDLL(str(out))
    L.emulate_encode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    return L


def run(emu, pkg, cubes, depth):
    p = pkg.plan_query(8, 8, depth)
    cubes = np.ascontiguousarray(cubes, np.uint8)
    n = cubes.shape[0]
    q = np.empty(cubes.size, np.int32)
    fl = np.empty(cubes.size, np.uint8)
    val = np.empty(cubes.size, np.float32)
    A = np.empty(n, np.float32)
    t = [np.ascontiguousarray(p[k], np.float32) for k in ("enc_rstep", "enc_G", "enc_E")]
    emu.emulate_encode(cubes.ctypes.data, n, depth, t[0].ctypes.data, t[1].ctypes.data, t[2].ctypes.data,
                       p["coef_dc"], q.ctypes.data, fl.ctypes.data, val.ctypes.data, A.ctypes.data)
    shape = (n, depth, 8, 8)
    return q.reshape(shape), fl.reshape(shape).astype(bool), val.reshape(shape), A, p


def _inputs(pkg, depth):
    rng = np.random.default_rng(1234)
    fr_r = pkg.synthetic.frames(256, 128, depth * 2, kind="ramp")
    fr_u = pkg.synthetic.frames(256, 128, depth * 2, kind="uniform")
    z, y, x = np.meshgrid(np.arange(depth * 2), np.arange(64), np.arange(64), indexing="ij")
    extreme = [((x + y + z) % 2) * 255, ((x // 3 + y // 5) % 2) * 255, (x * 29 + y * 7 + z * 3) % 256,
               np.where((x + y) % 16 < 8, 0, 255), np.full_like(x, 255), rng.integers(0, 2, x.shape) * 255]
    return [fr_r, fr_u] + [e.astype(np.uint8) for e in extreme]


@pytest.mark.parametrize("depth", [8, 4])
def test_unflagged_coefficients_equal_oracle(emu, pkg, oracle, plan8, plan4, depth):
    plan = plan8 if depth == 8 else plan4
    tot = fl_tot = 0
    for fr in _inputs(pkg, depth):
        cubes = oracle.to_cubes(fr, 8, 8, depth)
        q, fl, _, _, _ = run(emu, pkg, cubes, depth)
        ref = plan.encode_q(fr)
        bad = (q != ref) & ~fl
        assert not bad.any(), f"{bad.sum()} uncertified mismatches"
        tot += q.size
        fl_tot += fl.sum()
    assert fl_tot / tot < 2e-3


@pytest.mark.parametrize("depth", [8, 4])
def test_bound_dominates_observed_error(emu, pkg, oracle, plan8, plan4, depth):
    plan = plan8 if depth == 8 else plan4
    worst = 0.0
    for fr in _inputs(pkg, depth):
        cubes = oracle.to_cubes(fr, 8, 8, depth)
        _, _, val, A, p = run(emu, pkg, cubes, depth)
        exact = oracle.to_cubes(plan.dct(fr), 8, 8, depth)    # fp64 (error ~1e-12, negligible here)
        K = p["enc_K"].reshape(depth, 8, 8)
        err = np.abs(val.astype(np.float64) - exact)
        err[:, 0, 0, 0] = 0.0                                    # DC: exact integer path, not the fp32 value
        bound = A[:, None, None, None] * K[None] + 1e-9
        assert (err <= bound).all()
        worst = max(worst, float((err / bound).max()))
    assert worst < 1.0


def test_decode_fixed_point_certificate():
    """decode_tile's certificate and byte packing (dct3d_decode_dev.h, kFixMagic): w = v + 1.5 * 2^20 in
    fp64; 'certified' iff mi <= lo(w) <= 2^32 - 1 - mi, mi = ceil(m 2^32 + 1/2) + 1; byte = the low half
    of hi(w) read as a signed 16-bit value, saturated to [0, 255] (v_sat_pk_u8_i16), valid for
    |v| < 2^15.  Claim: when certified, every real value in [v - m, v + m] maps to that byte under
    Java's (byte) clamp(x, 0, 255) of InverseDCT.java:74-80 (floor of the clamped value).  Checked
    exactly (fractions) on random values, values within a few ulps of integers and of the clamp ends,
    values near the 16-bit limits, and several margins m."""
    from fractions import Fraction
    import math
    rng = np.random.default_rng(17)
    base = np.concatenate([rng.uniform(-600, 900, 4000), np.round(rng.uniform(-300, 560, 3000)),
                           rng.uniform(-32700, 32700, 500)])
    vals = [float(v) for v in base]
    for v in list(vals[4000:7000]):
        vals += [math.nextafter(v, math.inf), math.nextafter(v, -math.inf), v + 2.0 ** -30, v - 2.0 ** -30,
                 v + 3e-9, v - 3e-9]
    vals += [0.0, -0.0, 255.0, 256.0, -1e-12, 255.999999999, 254.9999999999, 32767.5, -32767.5, 32000.25]

    def java_byte(x):
        x = min(max(x, Fraction(0)), Fraction(255))
        return math.floor(x)

    def sat8(h16):
        s16 = h16 - 65536 if h16 >= 32768 else h16
        return min(max(s16, 0), 255)

    n_cert = n_flag = 0
    for m in (1e-12, 6.6e-9, 1e-6):
        mi = math.ceil(Fraction(m) * 2 ** 32 + Fraction(1, 2)) + 1
        for v in vals:
            assert abs(v) < 2 ** 15
            w = np.float64(v) + np.float64(1572864.0)
            bits = int(np.array([w]).view(np.uint64)[0])
            hi, lo = bits >> 32, bits & 0xFFFFFFFF
            byte = sat8(hi & 0xFFFF)
            if mi <= lo <= 0xFFFFFFFF - mi:
                n_cert += 1
                fv, fm = Fraction(v), Fraction(m)
                assert java_byte(fv - fm) == byte == java_byte(fv + fm), (v, m)
            else:
                n_flag += 1
    assert n_cert > 0 and n_flag > 0  # both outcomes exercised (most test values sit near integers)


@pytest.fixture(scope="module")
def emu_dec(tmp_path_factory):
    out = tmp_path_factory.mktemp("emud") / "libemud.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-shared", "-fPIC",
                    "-I", os.path.join(REPO, "3ddctvideoencoding_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "emulate_decode.cpp"), "-o", str(out)], check=True)
    L = C.CDLL(str(out))
    L.emulate_decode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    return L


@pytest.mark.parametrize("depth", [8, 4])
def test_decode_bound_dominates_observed_error(emu_dec, pkg, oracle, plan8, plan4, depth):
    """The decode kernel's fp64 values (host emulation, same butterflies, same order) against Java's
    InverseDCT fold (oracle): |v - v_java| <= dec_G * L1 + dec_E with L1 = sum |q * step| over the cube
    (dct3d_plan.cpp, per-input Tracked analysis); both sides clamped to [0, 255], which can only shrink
    the difference.  Also |v| <= L1 * 32000 / dec_l1_max (the 16-bit packing's range argument)."""
    plan = plan8 if depth == 8 else plan4
    p = pkg.plan_query(8, 8, depth)
    W, H, F = 64, 32, depth * 2
    rng = np.random.default_rng(99)
    qs = []
    for fr in _inputs(pkg, depth):
        qs.append(plan.encode_q(np.ascontiguousarray(fr[:F, :H, :W])))
    q = rng.integers(-40, 41, size=qs[0].shape).astype(np.int32)
    q[:, 0, 0, 0] = rng.integers(-300, 6000, size=q.shape[0])
    qs.append(q)
    qs.append(rng.integers(-3, 4, size=qs[0].shape).astype(np.int32) * 50)
    worst = 0.0
    for q in qs:
        q = np.ascontiguousarray(q, np.int32)
        n = q.shape[0]
        v = np.empty(q.size, np.float64)
        l1 = np.empty(n, np.float64)
        emu_dec.emulate_decode(q.ctypes.data, n, depth, v.ctypes.data, l1.ctypes.data)
        v = v.reshape(n, depth, 8, 8)
        java = oracle.to_cubes(plan.idct(oracle.dequantize(q, W, H, F, 8, 8, depth)), 8, 8, depth)
        err = np.abs(np.clip(v, 0.0, 255.0) - java)
        bound = l1[:, None, None, None] * p["dec_G"] + p["dec_E"]
        assert (err <= bound).all()
        worst = max(worst, float((err / bound).max()))
        assert (np.abs(v) <= l1[:, None, None, None] * (32000.0 / p["dec_l1_max"]) * (1 + 1e-6) + 1e-6).all()
    assert worst < 1.0
