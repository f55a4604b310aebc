"""Open-coefficient rate of the 8x8x8 encode's fp32 certificate on the host (tests/native/emulate_encode.cpp:
the kernel's fp32 arithmetic, same butterflies and order), with the per-s tables the kernel uses and with
per-coefficient tables (K_k / step instead of the max over k with the same s).  DESIGN.md §4.
    python tools/cert_bound_study.py [uniform|ramp]"""
import ctypes as C
import importlib
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    sys.path.insert(0, ROOT)
    pkg = importlib.import_module("3ddctvideoencoding_amd")
    so = os.path.join(tempfile.mkdtemp(), "libemu.so")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-shared", "-fPIC", "-I",
                    os.path.join(ROOT, "3ddctvideoencoding_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "emulate_encode.cpp"), "-o", so], check=True)
    L = C.CDLL(so)
    L.emulate_encode.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    kind = sys.argv[1] if len(sys.argv) > 1 else "uniform"
    p = pkg.plan_query(8, 8, 8)
    fr = pkg.synthetic.frames(1024, 512, 16, kind=kind)
    F, H, W = fr.shape
    cubes = np.ascontiguousarray(fr.reshape(F // 8, 8, H // 8, 8, W // 8, 8).transpose(0, 2, 4, 1, 3, 5).reshape(-1, 8, 8, 8))
    n = cubes.shape[0]
    q = np.empty(cubes.size, np.int32)
    fl = np.empty(cubes.size, np.uint8)
    val = np.empty(cubes.size, np.float32)
    A = np.empty(n, np.float32)
    t = [np.ascontiguousarray(p[k], np.float32) for k in ("enc_rstep", "enc_G", "enc_E")]
    L.emulate_encode(cubes.ctypes.data, n, 8, t[0].ctypes.data, t[1].ctypes.data, t[2].ctypes.data, p["coef_dc"],
                     q.ctypes.data, fl.ctypes.data, val.ctypes.data, A.ctypes.data)
    fl = fl.reshape(n, 8, 8, 8).astype(bool)
    val = val.reshape(n, 8, 8, 8).astype(np.float64)
    kz, ky, kx = np.meshgrid(np.arange(8), np.arange(8), np.arange(8), indexing="ij")
    s = kz + ky + kx
    step = np.maximum(1, 5 * s)
    qq = val / step
    frac = np.abs(qq - np.rint(qq))
    Gs, Es = np.array(p["enc_G"], np.float64), np.array(p["enc_E"], np.float64)
    Gk = p["enc_K"].reshape(8, 8, 8) * (1 + 1e-4) / step
    print(f"{kind}: {n} cubes, kernel flag rate {fl.mean():.3e}")
    for name, G in (("per-s tables (kernel)", Gs[s]), ("per-coefficient tables", Gk)):
        open_ = frac >= 0.5 - (A[:, None, None, None] * G[None] + Es[s][None])
        open_[:, 0, 0, 0] = False
        print(f"  {name}: open rate {open_.mean():.3e}, waves (4 cubes) with an open coefficient "
              f"{open_.reshape(-1, 4 * 512).any(1).mean():.3f}")


if __name__ == "__main__":
    main()
