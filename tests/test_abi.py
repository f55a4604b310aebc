"""CPU: the C-ABI library loads, exports every symbol include/dct3d.h declares, and validates its
arguments without a device (no compute calls here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    return sorted(set(re.findall(r"\b([a-zA-Z_][a-zA-Z0-9_]*)\s*\(", src)) -
                  {"if", "sizeof", "defined", "extern", "while", "for", "return"})


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_dct3d_header_symbols_exported(pkg):
    names = _declared("dct3d.h")
    exp = _exported(pkg.LIB_PATH)
    missing = [n for n in names if n not in exp]
    assert not missing, missing
    assert set(pkg.ABI_SYMBOLS) <= set(names)


def test_diag_header_symbols_exported_by_diag_lib_only(pkg):
    """include/dct3d_diag.h (measurement / test support) is exported by libdct3d_diag.so and by
    nothing in the product library."""
    names = _declared("dct3d_diag.h")
    exp = _exported(pkg.DIAG_LIB_PATH)
    assert not [n for n in names if n not in exp]
    assert set(pkg.DIAG_SYMBOLS) == set(names)
    assert not set(names) & _exported(pkg.LIB_PATH)


@pytest.mark.parametrize("header", ["codec.h", "cube_utils.h", "exp_golomb.h", "cube_io.h"])
def test_codec_header_symbols_exported(pkg, header):
    names = _declared(header)
    exp = _exported(pkg.CODEC_LIB_PATH)
    missing = [n for n in names if n not in exp]
    assert not missing, missing


def test_library_loads_and_reports_version(pkg):
    import re
    hdr = open(os.path.join(REPO, "include", "dct3d.h")).read()
    assert pkg.lib().dct3d_abi_version() == int(re.search(r"#define DCT3D_ABI_VERSION (\d+)", hdr).group(1))
    assert pkg.strerror(0) == "ok" and pkg.strerror(1) == "invalid argument"
    assert pkg.strerror(pkg.DCT3D_ENOSPC) == "output buffer too small"


def test_diagonal_order_matches_oracle(pkg, oracle):
    """The device Exp-Golomb stage's order table == the oracle's CubeUtils restatement (itself pinned
    against the reference's cubeUtils_diagonalSlices in test_oracle.py)."""
    for d in (8, 4):
        pos = oracle.diagonal_slices(8, 8, d)
        assert np.array_equal(pkg.diagonal_order(8, 8, d), pos[:, 0] + 8 * pos[:, 1] + 64 * pos[:, 2])
    with pytest.raises(pkg.Dct3dError):
        pkg.diagonal_order(8, 8, 5)


def test_argument_validation_without_device(pkg):
    L = pkg.lib()
    h = C.c_void_p()
    assert L.dct3d_ctx_create(0, 8, 8, 8, None) == pkg.DCT3D_EINVAL
    # no GPU in this container: a device error, never a crash or a silent CPU fallback
    rc = L.dct3d_ctx_create(0, 8, 8, 8, C.byref(h))
    assert rc in (pkg.DCT3D_OK, pkg.DCT3D_EDEVICE)
    if rc == pkg.DCT3D_OK:
        L.dct3d_ctx_destroy(h)
    for fn in ("dct3d_synchronize", "dct3d_reset_timers"):
        assert getattr(L, fn)(None) == pkg.DCT3D_EINVAL
    assert L.dct3d_encode_stacks(None, None, 64, 64, 1, None, None) == pkg.DCT3D_EINVAL
    assert L.dct3d_decode_stacks_dev(None, None, 64, 64, 1, None) == pkg.DCT3D_EINVAL
    assert L.dct3d_forward_f32(None, None, 1, None) == pkg.DCT3D_EINVAL
    L.dct3d_ctx_destroy(None)  # no-op


def test_cli_usage_without_device(pkg):
    r = subprocess.run([pkg.CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 0 and "Usage" in r.stdout
    r = subprocess.run([pkg.CLI_PATH, "encode", "/nonexistent", "/tmp/x.bin", "64", "64", "8"],
                       capture_output=True, text=True)
    assert r.returncode == 1
