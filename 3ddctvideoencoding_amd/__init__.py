"""3ddctvideoencoding_amd -- MI355X-native 3D-DCT hot path of julianopiccoli/3dDCTVideoEncoding.

The product is the C-ABI library ``lib/libdct3d.so`` (HIP kernels for gfx950 + runtime, declared in
``include/dct3d.h``) and the reference-compatible C codec host ``lib/libdct3dcodec.so`` /
``lib/dct3d_codec``.  This module is a thin ctypes binding with the same entry-point names; it has
NO fallback: if the library is missing or no HIP device is present the calls raise.

Since the package name starts with a digit, import it with
``importlib.import_module("3ddctvideoencoding_amd")``.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import synthetic  # noqa: F401  (integer-only generator shared with the device kernel)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libdct3d.so")
DIAG_LIB_PATH = os.path.join(LIB_DIR, "libdct3d_diag.so")  # measurement / test support (include/dct3d_diag.h)
CODEC_LIB_PATH = os.path.join(LIB_DIR, "libdct3dcodec.so")
CLI_PATH = os.path.join(LIB_DIR, "dct3d_codec")
REPO_DIR = os.path.dirname(PKG_DIR)
INCLUDE_DIR = os.path.join(REPO_DIR, "include")

DCT3D_OK, DCT3D_EINVAL, DCT3D_EDEVICE, DCT3D_ENOMEM, DCT3D_EKERNEL, DCT3D_ENOSPC, DCT3D_ENODATA = 0, 1, 2, 3, 4, 5, 6
# test / diagnostic options (include/dct3d.h, Context.set_option)
DCT3D_OPT_DEC_MARGIN, DCT3D_OPT_ENC_NO_RECHECK, DCT3D_OPT_EG_TWO_STEP, DCT3D_OPT_EG_NO_RESOLVE = 2, 3, 5, 6
DCT3D_OPT_EG_FORCE_RETRY = 8
DCT3D_OPT_EG_DEC_GROUPS = 9
DCT3D_OPT_EG_FUSED_FRONT = 10

# Every symbol include/dct3d.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "dct3d_abi_version", "dct3d_strerror", "dct3d_ctx_create", "dct3d_ctx_destroy",
    "dct3d_ctx_set_stream", "dct3d_ctx_info", "dct3d_ctx_set_option", "dct3d_ctx_set_profiling", "dct3d_synchronize", "dct3d_get_stats",
    "dct3d_reset_timers",
    "dct3d_encode_stacks", "dct3d_encode_stacks_dev", "dct3d_decode_stacks", "dct3d_decode_stacks_dev",
    "dct3d_forward_f32", "dct3d_inverse_f32", "dct3d_forward_f32_dev", "dct3d_inverse_f32_dev",
    "dct3d_plan_query",
    "dct3d_eg_encode_dev", "dct3d_encode_eg", "dct3d_eg_fetch", "dct3d_diagonal_order",
    "dct3d_eg_decode_dev", "dct3d_decode_eg", "dct3d_encode_eg_dev", "dct3d_decode_eg_dev",
)
# Every symbol include/dct3d_diag.h declares (libdct3d_diag.so; none of them is in libdct3d.so).
DIAG_SYMBOLS = ("dct3d_fill_synthetic_dev", "dct3d_bandwidth_probe_dev", "dct3d_encode_memonly_dev",
                "dct3d_encode_diag_dev", "dct3d_encode_trace_dev", "dct3d_encode_strip_dev", "dct3d_decode_diag_dev")


class Dct3dError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {strerror(code)} ({code})")
        self.code = code


class PlanInfo(C.Structure):
    _fields_ = [("cube_size", C.c_int), ("n_mults", C.c_int), ("treeified", C.c_int), ("coef_dc", C.c_double),
                ("dec_G", C.c_double), ("dec_E", C.c_double), ("enc_rstep", C.c_float * 32),
                ("enc_G", C.c_float * 32), ("enc_E", C.c_float * 32), ("enc_thr64", C.c_double * 32),
                ("dec_l1_max", C.c_float)]


class Stats(C.Structure):
    _fields_ = [("n_units", C.c_uint64), ("n_flagged", C.c_uint64),
                ("n_timed", C.c_uint64), ("kernel_ms_total", C.c_double), ("aux_ms_total", C.c_double),
                ("n_rechecked", C.c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def lib() -> C.CDLL:
    """Load libdct3d.so (raises if it has not been built: run __graft_entry__.build() / make)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build())")
        # PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7).  If libdct3d.so were
        # loaded first, torch would later load a second HIP runtime and find no GPU; loading torch
        # first lets libdct3d.so bind to the already-loaded runtime (one HIP runtime per process).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, i32, sz, u64, i64 = C.c_void_p, C.c_int, C.c_size_t, C.c_uint64, C.c_int64
        L.dct3d_abi_version.restype = i32
        L.dct3d_strerror.restype = C.c_char_p
        L.dct3d_strerror.argtypes = [i32]
        L.dct3d_ctx_create.argtypes = [i32, i32, i32, i32, C.POINTER(vp)]
        L.dct3d_ctx_destroy.argtypes = [vp]
        L.dct3d_ctx_destroy.restype = None
        L.dct3d_ctx_set_stream.argtypes = [vp, vp]
        L.dct3d_ctx_set_profiling.argtypes = [vp, i32]
        L.dct3d_ctx_set_option.argtypes = [vp, i32, C.c_double]
        L.dct3d_synchronize.argtypes = [vp]
        L.dct3d_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.dct3d_reset_timers.argtypes = [vp]
        for name in ("dct3d_encode_stacks", "dct3d_encode_stacks_dev"):
            getattr(L, name).argtypes = [vp, vp, i32, i32, i32, vp, vp]
        for name in ("dct3d_decode_stacks", "dct3d_decode_stacks_dev"):
            getattr(L, name).argtypes = [vp, vp, i32, i32, i32, vp]
        for name in ("dct3d_forward_f32", "dct3d_inverse_f32", "dct3d_forward_f32_dev", "dct3d_inverse_f32_dev"):
            getattr(L, name).argtypes = [vp, vp, sz, vp]
        L.dct3d_ctx_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(vp)]
        L.dct3d_plan_query.argtypes = [i32, i32, i32, C.POINTER(PlanInfo), vp, vp, vp, vp]
        L.dct3d_eg_encode_dev.argtypes = [vp, vp, u64, C.c_uint8, i32, vp, u64, C.POINTER(u64)]
        L.dct3d_encode_eg.argtypes = [vp, vp, i32, i32, i32, C.c_uint8, i32, C.POINTER(u64)]
        L.dct3d_encode_eg_dev.argtypes = [vp, vp, i32, i32, i32, C.c_uint8, i32, vp, u64, C.POINTER(u64)]
        L.dct3d_eg_fetch.argtypes = [vp, vp, u64]
        L.dct3d_diagonal_order.argtypes = [i32, i32, i32, vp]
        L.dct3d_eg_decode_dev.argtypes = [vp, vp, u64, u64, u64, vp, C.POINTER(u64)]
        L.dct3d_decode_eg.argtypes = [vp, vp, u64, i32, i32, i32, i32, vp, C.POINTER(u64)]
        L.dct3d_decode_eg_dev.argtypes = [vp, vp, u64, u64, i32, i32, i32, vp, C.POINTER(u64)]
        _lib = L
    return _lib


_diag = None


def diag_lib() -> C.CDLL:
    """Load libdct3d_diag.so (bench / test support: synthetic frames, memory-only twins, probes)."""
    global _diag
    if _diag is None:
        lib()  # the product library first (the diag library links against it)
        if not os.path.exists(DIAG_LIB_PATH):
            raise ImportError(f"{DIAG_LIB_PATH} is missing: build it with `make`")
        D = C.CDLL(DIAG_LIB_PATH)
        vp, i32, sz, u64, i64 = C.c_void_p, C.c_int, C.c_size_t, C.c_uint64, C.c_int64
        D.dct3d_fill_synthetic_dev.argtypes = [vp, vp, i32, i32, i32, u64, i64, i32]
        D.dct3d_bandwidth_probe_dev.argtypes = [vp, vp, vp, sz, i32]
        D.dct3d_encode_memonly_dev.argtypes = [vp, vp, i32, i32, i32, vp]
        D.dct3d_encode_diag_dev.argtypes = [vp, vp, i32, i32, i32, vp, i32]
        D.dct3d_encode_strip_dev.argtypes = [vp, vp, i32, i32, i32, vp, i32, i32]
        D.dct3d_encode_trace_dev.argtypes = [vp, vp, i32, i32, i32, vp, i32, vp]
        D.dct3d_decode_diag_dev.argtypes = [vp, vp, i32, i32, i32, vp, i32]
        _diag = D
    return _diag


def strerror(code: int) -> str:
    try:
        return lib().dct3d_strerror(code).decode()
    except Exception:
        return "error"


def _check(rc: int, what: str) -> None:
    if rc != DCT3D_OK:
        raise Dct3dError(rc, what)


def _ptr(a: np.ndarray) -> int:
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data


def _tptr(t) -> int:
    """device pointer of a torch tensor (or an int address)."""
    if isinstance(t, int):
        return t
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return t.data_ptr()


def plan_query(block_w: int = 8, block_h: int = 8, block_d: int = 8) -> dict:
    """Host-side transform plan (no device): Java fold tables + certification tables."""
    cs = block_w * block_h * block_d
    info = PlanInfo()
    ng = np.empty(cs, np.int32)
    coef = np.empty(cs * 64, np.float64)
    gof = np.empty(cs * cs, np.uint8)
    K = np.empty(cs, np.float64)
    _check(lib().dct3d_plan_query(block_w, block_h, block_d, C.byref(info), _ptr(ng), _ptr(coef), _ptr(gof), _ptr(K)),
           "dct3d_plan_query")
    return {"cube_size": info.cube_size, "n_mults": info.n_mults, "treeified": bool(info.treeified),
            "coef_dc": info.coef_dc, "dec_G": info.dec_G, "dec_E": info.dec_E, "dec_l1_max": info.dec_l1_max,
            "enc_rstep": np.array(info.enc_rstep[:]), "enc_G": np.array(info.enc_G[:]),
            "enc_E": np.array(info.enc_E[:]), "enc_thr64": np.array(info.enc_thr64[:]), "ngroups": ng, "coef": coef.reshape(cs, 64),
            "group_of": gof.reshape(cs, cs), "enc_K": K}


def diagonal_order(block_w: int = 8, block_h: int = 8, block_d: int = 8) -> np.ndarray:
    """Diagonal-slice order used by the device Exp-Golomb stage: cube index x + 8y + 64z per stream
    position (CubeUtils.c:5-46)."""
    out = np.empty(block_w * block_h * block_d, np.uint16)
    _check(lib().dct3d_diagonal_order(block_w, block_h, block_d, _ptr(out)), "dct3d_diagonal_order")
    return out


def eg_stream_bytes(total_bits: int) -> int:
    """Bytes holding a stream of total_bits bits (the last one partial)."""
    return (total_bits + 7) // 8


class Context:
    """dct3d_ctx: one per device (the MI355X equivalent of the reference's per-call OpenCL setup,
    encoder.c:147-197).  Block dims are codec.h's DCT_BLOCK_WIDTH/HEIGHT/DEPTH (8x8x8 or 8x8x4)."""

    def __init__(self, device: int = 0, block_w: int = 8, block_h: int = 8, block_d: int = 8):
        h = C.c_void_p()
        _check(lib().dct3d_ctx_create(device, block_w, block_h, block_d, C.byref(h)), "dct3d_ctx_create")
        self._h = h
        self.device, self.bw, self.bh, self.bd = device, block_w, block_h, block_d
        self.cube_size = block_w * block_h * block_d

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().dct3d_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- configuration ----
    def set_stream(self, hip_stream: Optional[int]) -> None:
        """Run on an external hipStream_t.  None or 0 (e.g. torch's default stream, whose handle is 0)
        selects the context's own stream -- use a non-default stream to share one with a framework."""
        _check(lib().dct3d_ctx_set_stream(self._h, hip_stream or None), "dct3d_ctx_set_stream")

    def set_option(self, option: int, value: float) -> None:
        """Test / diagnostic option (DCT3D_OPT_*): changes how later calls reach their (identical)
        results, e.g. to drive a rare path.  0 restores the default."""
        _check(lib().dct3d_ctx_set_option(self._h, option, float(value)), "dct3d_ctx_set_option")

    def set_profiling(self, on: bool) -> None:
        _check(lib().dct3d_ctx_set_profiling(self._h, 1 if on else 0), "dct3d_ctx_set_profiling")

    def synchronize(self) -> None:
        _check(lib().dct3d_synchronize(self._h), "dct3d_synchronize")

    def stats(self) -> dict:
        st = Stats()
        _check(lib().dct3d_get_stats(self._h, C.byref(st)), "dct3d_get_stats")
        return st.as_dict()

    def reset_timers(self) -> None:
        _check(lib().dct3d_reset_timers(self._h), "dct3d_reset_timers")

    def n_cubes(self, width: int, height: int, n_stacks: int) -> int:
        return (width // self.bw) * (height // self.bh) * n_stacks

    # ---- host-pointer (synchronous) entry points ----
    def encode_stacks(self, frames: np.ndarray, want_dct: bool = False):
        """u8 frames [n_stacks*bd, H, W] -> quantised int32 cubes [n_cubes, bd, bh, bw]
        (+ fp64 DCT coefficients in the same layout when want_dct)."""
        frames = np.ascontiguousarray(frames, np.uint8)
        F, H, W = frames.shape
        if F % self.bd:
            raise ValueError("frame count must be a multiple of the block depth")
        n = self.n_cubes(W, H, F // self.bd)
        q = np.empty((n, self.bd, self.bh, self.bw), np.int32)
        d = np.empty((n, self.bd, self.bh, self.bw), np.float64) if want_dct else None
        _check(lib().dct3d_encode_stacks(self._h, _ptr(frames), W, H, F // self.bd, _ptr(q),
                                         _ptr(d) if want_dct else None), "dct3d_encode_stacks")
        return (q, d) if want_dct else q

    def decode_stacks(self, q: np.ndarray, width: int, height: int, n_stacks: int) -> np.ndarray:
        q = np.ascontiguousarray(q, np.int32)
        out = np.empty((n_stacks * self.bd, height, width), np.uint8)
        _check(lib().dct3d_decode_stacks(self._h, _ptr(q), width, height, n_stacks, _ptr(out)),
               "dct3d_decode_stacks")
        return out

    def forward_f32(self, cubes: np.ndarray) -> np.ndarray:
        cubes = np.ascontiguousarray(cubes, np.float32)
        n = cubes.size // self.cube_size
        out = np.empty_like(cubes)
        _check(lib().dct3d_forward_f32(self._h, _ptr(cubes), n, _ptr(out)), "dct3d_forward_f32")
        return out

    def inverse_f32(self, coeffs: np.ndarray) -> np.ndarray:
        coeffs = np.ascontiguousarray(coeffs, np.float32)
        n = coeffs.size // self.cube_size
        out = np.empty_like(coeffs)
        _check(lib().dct3d_inverse_f32(self._h, _ptr(coeffs), n, _ptr(out)), "dct3d_inverse_f32")
        return out

    # ---- device-pointer (asynchronous, ctx stream) entry points ----
    def encode_stacks_dev(self, d_frames, width: int, height: int, n_stacks: int, d_q, d_dct=None) -> None:
        _check(lib().dct3d_encode_stacks_dev(self._h, _tptr(d_frames), width, height, n_stacks, _tptr(d_q),
                                             _tptr(d_dct) if d_dct is not None else None),
               "dct3d_encode_stacks_dev")

    def decode_stacks_dev(self, d_q, width: int, height: int, n_stacks: int, d_frames) -> None:
        _check(lib().dct3d_decode_stacks_dev(self._h, _tptr(d_q), width, height, n_stacks, _tptr(d_frames)),
               "dct3d_decode_stacks_dev")

    def forward_f32_dev(self, d_in, n_cubes: int, d_out) -> None:
        _check(lib().dct3d_forward_f32_dev(self._h, _tptr(d_in), n_cubes, _tptr(d_out)), "dct3d_forward_f32_dev")

    def inverse_f32_dev(self, d_in, n_cubes: int, d_out) -> None:
        _check(lib().dct3d_inverse_f32_dev(self._h, _tptr(d_in), n_cubes, _tptr(d_out)), "dct3d_inverse_f32_dev")

    def bandwidth_probe_dev(self, d_in, d_out, n_px: int, mode: int = 0) -> None:
        _check(diag_lib().dct3d_bandwidth_probe_dev(self._h, _tptr(d_in) if d_in is not None else None,
                                               _tptr(d_out) if d_out is not None else None, n_px, mode),
               "dct3d_bandwidth_probe_dev")

    def encode_memonly_dev(self, d_frames, width: int, height: int, n_stacks: int, d_q) -> None:
        """Diagnostic: the encode's memory traffic without its compute (d_q is NOT a DCT)."""
        _check(diag_lib().dct3d_encode_memonly_dev(self._h, _tptr(d_frames), width, height, n_stacks, _tptr(d_q)),
               "dct3d_encode_memonly_dev")

    def encode_strip_dev(self, d_frames, width: int, height: int, n_stacks: int, d_q, mode: int, strip_w: int) -> None:
        """diagnostic traversal sweep (dct3d_encode_strip_dev): mode 1 memory only, mode 0 the full encode"""
        _check(diag_lib().dct3d_encode_strip_dev(self._h, _tptr(d_frames), width, height, n_stacks, _tptr(d_q), mode,
                                                 strip_w), "dct3d_encode_strip_dev")

    def encode_diag_dev(self, d_frames, width: int, height: int, n_stacks: int, d_q, mode: int) -> None:
        """Diagnostic: the encode's memory part (mode 1) or, 8x8x8, its compute part (mode 2) alone."""
        _check(diag_lib().dct3d_encode_diag_dev(self._h, _tptr(d_frames), width, height, n_stacks, _tptr(d_q), mode),
               "dct3d_encode_diag_dev")

    def encode_trace_dev(self, d_frames, width: int, height: int, n_stacks: int, d_q, d_trace) -> None:
        """Diagnostic: the product encode (8x8x8) with a per-wave timeline in d_trace (uint64, 4 per wave:
        start, transform done, stores issued -- 100 MHz clock -- and XCC_ID << 32 | HW_ID)."""
        _check(diag_lib().dct3d_encode_trace_dev(self._h, _tptr(d_frames), width, height, n_stacks, _tptr(d_q), 3,
                                                 _tptr(d_trace)), "dct3d_encode_trace_dev")

    def decode_diag_dev(self, d_q, width: int, height: int, n_stacks: int, d_frames, mode: int) -> None:
        """Diagnostic: the decode's memory part (mode 1) or compute part (mode 2) alone."""
        _check(diag_lib().dct3d_decode_diag_dev(self._h, _tptr(d_q), width, height, n_stacks, _tptr(d_frames), mode),
               "dct3d_decode_diag_dev")

    # ---- Exp-Golomb stage ----
    def eg_encode_dev(self, d_q, n_cubes: int, d_out, out_cap: int, carry_byte: int = 0, carry_bits: int = 0) -> int:
        """Device Exp-Golomb stream of n_cubes int32 cubes into d_out (4-byte aligned words); returns the
        total bits (carry included).  Raises Dct3dError(DCT3D_ENOSPC) when out_cap is too small."""
        tb = C.c_uint64(0)
        _check(lib().dct3d_eg_encode_dev(self._h, _tptr(d_q), n_cubes, carry_byte, carry_bits, _tptr(d_out), out_cap,
                                         C.byref(tb)), "dct3d_eg_encode_dev")
        return tb.value

    def encode_eg_dev(self, d_frames, width: int, height: int, n_stacks: int, d_out, out_cap: int,
                      carry_byte: int = 0, carry_bits: int = 0) -> int:
        """Fused device path: u8 frames (device) -> Exp-Golomb stream words in d_out, no int32
        intermediate; returns the total bits (carry included).  Dct3dError(DCT3D_ENOSPC) if out_cap is
        too small."""
        tb = C.c_uint64(0)
        _check(lib().dct3d_encode_eg_dev(self._h, _tptr(d_frames), width, height, n_stacks, carry_byte, carry_bits,
                                         _tptr(d_out), out_cap, C.byref(tb)), "dct3d_encode_eg_dev")
        return tb.value

    def encode_eg(self, frames: np.ndarray, carry_byte: int = 0, carry_bits: int = 0) -> tuple[bytes, int]:
        """u8 frames [n_stacks*bd, H, W] -> (Exp-Golomb stream bytes, total bits), computed on the device
        (DCT + quantisation + diagonal order + Exp-Golomb); only the stream crosses PCIe."""
        frames = np.ascontiguousarray(frames, np.uint8)
        F, H, W = frames.shape
        if F % self.bd:
            raise ValueError("frame count must be a multiple of the block depth")
        tb = C.c_uint64(0)
        _check(lib().dct3d_encode_eg(self._h, _ptr(frames), W, H, F // self.bd, carry_byte, carry_bits, C.byref(tb)),
               "dct3d_encode_eg")
        out = np.empty(eg_stream_bytes(tb.value), np.uint8)
        _check(lib().dct3d_eg_fetch(self._h, _ptr(out) if out.size else None, out.size), "dct3d_eg_fetch")
        return out.tobytes(), tb.value

    def eg_decode_dev(self, d_bytes, nbytes: int, start_bit: int, n_cubes: int, d_q) -> int:
        """Device Exp-Golomb stream (4-byte aligned) -> n_cubes cube-major int32 cubes; returns the bit
        after the last value.  Dct3dError(DCT3D_ENODATA) if the stream is too short."""
        eb = C.c_uint64(0)
        _check(lib().dct3d_eg_decode_dev(self._h, _tptr(d_bytes), nbytes, start_bit, n_cubes, _tptr(d_q), C.byref(eb)),
               "dct3d_eg_decode_dev")
        return eb.value

    def decode_eg_dev(self, d_bytes, nbytes: int, start_bit: int, width: int, height: int, n_stacks: int,
                      d_frames) -> int:
        """Fused device path: Exp-Golomb stream (device, 4-byte aligned) -> u8 frames (device), no int32
        intermediate; returns the bit after the last value once the stream's verdict is known -- the frames
        complete asynchronously on the context stream (as decode_stacks_dev; synchronize() or stream order)."""
        eb = C.c_uint64(0)
        _check(lib().dct3d_decode_eg_dev(self._h, _tptr(d_bytes), nbytes, start_bit, width, height, n_stacks,
                                         _tptr(d_frames), C.byref(eb)), "dct3d_decode_eg_dev")
        return eb.value

    def decode_eg(self, stream: bytes, width: int, height: int, n_stacks: int, start_bit: int = 0):
        """Exp-Golomb stream bytes (from bit start_bit, 0..7) -> (u8 frames [n_stacks*bd, H, W], end bit):
        entropy decode + dequantise + IDCT on the device."""
        b = np.frombuffer(stream, np.uint8)
        out = np.empty((n_stacks * self.bd, height, width), np.uint8)
        eb = C.c_uint64(0)
        _check(lib().dct3d_decode_eg(self._h, _ptr(b) if b.size else None, b.size, start_bit, width, height, n_stacks,
                                     _ptr(out), C.byref(eb)), "dct3d_decode_eg")
        return out, eb.value

    def fill_synthetic_dev(self, d_frames, width: int, height: int, n_frames: int,
                           seed: int = synthetic.DEFAULT_SEED, frame0: int = 0, kind: str = "ramp") -> None:
        k = {"ramp": 0, "uniform": 1}[kind]
        _check(diag_lib().dct3d_fill_synthetic_dev(self._h, _tptr(d_frames), width, height, n_frames, seed, frame0, k),
               "dct3d_fill_synthetic_dev")
