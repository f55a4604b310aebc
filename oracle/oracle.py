"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).

ctypes binding of oracle/java_dct3d.c, the plain-C restatement of the reference's Java codec
semantics (dct/DCT.java, dct/InverseDCT.java, Encoder.java:75-89, Decoder.java:78-117,
CubeUtils.java, ExpGolombWriter/Reader.java).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  See java_dct3d.c's header for what pins it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libref_codec.so")

_lib = None


def build(quiet: bool = True) -> None:
    """Compile the oracle (and oracle/_ref when the reference sources are present)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i32, f64 = C.c_void_p, C.c_int, C.c_double
        L.oracle_plan_create.restype = vp
        L.oracle_plan_create.argtypes = [i32, i32, i32]
        L.oracle_plan_create_alt.restype = vp
        L.oracle_plan_create_alt.argtypes = [i32, i32, i32, vp, vp, i32, i32]
        L.oracle_plan_destroy.argtypes = [vp]
        for name in ("oracle_plan_n_mults", "oracle_plan_n_sums", "oracle_plan_treeified"):
            getattr(L, name).restype = i32
            getattr(L, name).argtypes = [vp]
        L.oracle_plan_n_groups.restype = i32
        L.oracle_plan_n_groups.argtypes = [vp, i32]
        L.oracle_plan_group_coef.restype = f64
        L.oracle_plan_group_coef.argtypes = [vp, i32, i32]
        L.oracle_plan_group_of.argtypes = [vp, i32, vp]
        L.oracle_plan_inv_coef.restype = f64
        L.oracle_plan_inv_coef.argtypes = [vp, i32, i32]
        L.oracle_dct_forward.argtypes = [vp, vp, i32, i32, i32, vp, i32]
        L.oracle_dct_inverse.argtypes = [vp, vp, i32, i32, i32, vp, i32]
        L.oracle_quantize.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp]
        L.oracle_dequantize.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp]
        L.oracle_to_bytes.argtypes = [vp, C.c_size_t, vp]
        L.oracle_encode_q.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32]
        L.oracle_decode_q.argtypes = [vp, vp, i32, i32, i32, vp, i32]
        L.oracle_java_round.restype = C.c_int64
        L.oracle_java_round.argtypes = [f64]
        L.oracle_diagonal_slices.restype = i32
        L.oracle_diagonal_slices.argtypes = [i32, i32, i32, vp]
        L.oracle_eg_write.restype = i32
        L.oracle_eg_write.argtypes = [vp, C.c_size_t, vp]
        L.oracle_eg_read.restype = i32
        L.oracle_eg_read.argtypes = [vp, C.c_size_t, C.c_size_t, vp]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


class Plan:
    """DCT.initialize/createSums + InverseDCT.initialize for one cube shape (cw, ch, cd)."""

    def __init__(self, cw: int = 8, ch: int = 8, cd: int = 8, cos_ulp=None, key_flip: int = 0):
        """cos_ulp / key_flip: the Math.cos residual study only (tools/cos_ulp_sensitivity.py) -- an
        alternative plan whose Math.cos is 1 ulp off glibc's at the given arguments ({arg: +-1}), and/or
        whose exactly rational coefficients take the other integer key (java_dct3d.c, cosalt)."""
        self.cw, self.ch, self.cd = cw, ch, cd
        self.cs = cw * ch * cd
        if cos_ulp is None and not key_flip:
            self._p = lib().oracle_plan_create(cw, ch, cd)
        else:
            items = sorted((cos_ulp or {}).items())
            self._args = np.array([a for a, _ in items] or [0.0], np.float64)
            self._delta = np.array([d for _, d in items] or [0], np.int8)
            self._p = lib().oracle_plan_create_alt(cw, ch, cd, _ptr(self._args), _ptr(self._delta), len(items),
                                                   int(key_flip))

    def __del__(self):
        try:
            if self._p:
                lib().oracle_plan_destroy(self._p)
        except Exception:
            pass

    @property
    def n_mults(self) -> int:
        return lib().oracle_plan_n_mults(self._p)

    @property
    def n_sums(self) -> int:
        return lib().oracle_plan_n_sums(self._p)

    @property
    def treeified(self) -> bool:
        return bool(lib().oracle_plan_treeified(self._p))

    def groups(self, k: int):
        """[(coef, members ndarray)] in fold (HashMap iteration) order for coefficient k."""
        ng = lib().oracle_plan_n_groups(self._p, k)
        gof = np.empty(self.cs, np.int16)
        lib().oracle_plan_group_of(self._p, k, _ptr(gof))
        return [(lib().oracle_plan_group_coef(self._p, k, g), np.nonzero(gof == g)[0]) for g in range(ng)]

    def group_of(self, k: int) -> np.ndarray:
        gof = np.empty(self.cs, np.int16)
        lib().oracle_plan_group_of(self._p, k, _ptr(gof))
        return gof

    def inv_coef(self, n: int, k: int) -> float:
        return lib().oracle_plan_inv_coef(self._p, n, k)

    # ---- hot path (Java semantics) ----
    def dct(self, frames: np.ndarray, threads: int | None = None) -> np.ndarray:
        """frames u8 [F, H, W] -> DCT coefficients float64 in raster layout (DCT.run)."""
        frames = np.ascontiguousarray(frames, np.uint8)
        F, H, W = frames.shape
        out = np.empty((F, H, W), np.float64)
        lib().oracle_dct_forward(self._p, _ptr(frames), W, H, F, _ptr(out), threads or default_threads())
        return out

    def encode_q(self, frames: np.ndarray, threads: int | None = None, want_dct: bool = False):
        """frames u8 [F, H, W] -> quantised int32 cube-major [n_cubes, cd, ch, cw] (Encoder.java:75-89)."""
        frames = np.ascontiguousarray(frames, np.uint8)
        F, H, W = frames.shape
        q = np.empty((F // self.cd) * (H // self.ch) * (W // self.cw) * self.cs, np.int32)
        d = np.empty((F, H, W), np.float64) if want_dct else None
        lib().oracle_encode_q(self._p, _ptr(frames), W, H, F, _ptr(q), _ptr(d) if want_dct else None,
                              threads or default_threads())
        q = q.reshape(-1, self.cd, self.ch, self.cw)
        return (q, d) if want_dct else q

    def decode_q(self, q: np.ndarray, W: int, H: int, F: int, threads: int | None = None) -> np.ndarray:
        """quantised int32 cube-major -> u8 frames [F, H, W] (Decoder.java:78-117)."""
        q = np.ascontiguousarray(q, np.int32)
        out = np.empty((F, H, W), np.uint8)
        lib().oracle_decode_q(self._p, _ptr(q), W, H, F, _ptr(out), threads or default_threads())
        return out

    def idct(self, coef_raster: np.ndarray, threads: int | None = None) -> np.ndarray:
        """raster float64 coefficients -> clamped float64 pixels (InverseDCT.run), no byte cast."""
        c = np.ascontiguousarray(coef_raster, np.float64)
        F, H, W = c.shape
        out = np.empty_like(c)
        lib().oracle_dct_inverse(self._p, _ptr(c), W, H, F, _ptr(out), threads or default_threads())
        return out


def quantize(dct_raster: np.ndarray, cw=8, ch=8, cd=8) -> np.ndarray:
    d = np.ascontiguousarray(dct_raster, np.float64)
    F, H, W = d.shape
    q = np.empty(d.size, np.int32)
    lib().oracle_quantize(_ptr(d), W, H, F, cw, ch, cd, _ptr(q))
    return q.reshape(-1, cd, ch, cw)


def dequantize(q: np.ndarray, W: int, H: int, F: int, cw=8, ch=8, cd=8) -> np.ndarray:
    q = np.ascontiguousarray(q, np.int32)
    out = np.empty((F, H, W), np.float64)
    lib().oracle_dequantize(_ptr(q), W, H, F, cw, ch, cd, _ptr(out))
    return out


def java_round(x: float) -> int:
    return lib().oracle_java_round(float(x))


def diagonal_slices(w=8, h=8, d=8) -> np.ndarray:
    out = np.empty((w * h * d, 3), np.int32)
    n = lib().oracle_diagonal_slices(w, h, d, _ptr(out))
    return out[:n]


def eg_write(values: np.ndarray) -> bytes:
    v = np.ascontiguousarray(values, np.int32)
    buf = np.zeros(v.size * 8 + 16, np.uint8)
    pos = lib().oracle_eg_write(_ptr(v), v.size, _ptr(buf))
    return bytes(buf[: pos + 1])  # Encoder.java:116 deflates getBufferPosition() + 1 bytes


def eg_read(data: bytes, n: int) -> np.ndarray:
    b = np.frombuffer(data, np.uint8).copy()
    out = np.empty(n, np.int32)
    r = lib().oracle_eg_read(_ptr(b), b.size, n, _ptr(out))
    if r < 0:
        raise ValueError("truncated Exp-Golomb stream")
    return out


def to_cubes(frames: np.ndarray, cw=8, ch=8, cd=8) -> np.ndarray:
    """u8/any [F, H, W] raster -> cube-major [n_cubes, cd, ch, cw] (encoder.c:29-41 order)."""
    F, H, W = frames.shape
    c = frames.reshape(F // cd, cd, H // ch, ch, W // cw, cw).transpose(0, 2, 4, 1, 3, 5)
    return np.ascontiguousarray(c.reshape(-1, cd, ch, cw))


def from_cubes(cubes: np.ndarray, W: int, H: int, F: int) -> np.ndarray:
    cd, ch, cw = cubes.shape[1:]
    c = cubes.reshape(F // cd, H // ch, W // cw, cd, ch, cw).transpose(0, 3, 1, 4, 2, 5)
    return np.ascontiguousarray(c.reshape(F, H, W))
