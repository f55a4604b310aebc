"""CPU: the corpora of tests/test_gpu_eg_fused.py::test_fused_matches_oracle reach every branch of the fused
encode's grouped Exp-Golomb emission (csrc/dct3d_kernels.hip, encode_eg_kernel): lane (cube, part) codes
stream positions part * cs/8 .. in groups of 8 codes (group 0, the DC's, as two halves of 4), a group
concatenated into one 64-bit append when its widths sum to W < 64 (group 0: both halves < 64) and
appended code by code otherwise; an append emits 0, 1 or 2 words.  The widths are computed here from the
oracle's quantised cubes (the restated Java encode) in the kernel's partition, so the GPU test's
bit-exact comparison covers: the fast path including appends of 32 <= W < 64 bits (two words from one
append when the lane has pending bits), the code-by-code path, and its boundary W = 64 (a sum of four or
eight odd widths is even: 63 cannot occur)."""
import numpy as np
import pytest


def _content(pkg, kind, w, h, f):
    if kind in ("ramp", "uniform"):
        return pkg.synthetic.frames(w, h, f, kind=kind)
    z, y, x = np.indices((f, h, w))
    if kind == "corner":    # a large DC and first-order coefficients
        return np.where((x % 8) + (y % 8) + (z % 8) < 10, 255, 0).astype(np.uint8)
    if kind == "edge":      # group 0's halves of exactly 64 bits at 8x8x4
        return np.where((x % 8) + (y % 8) + (z % 4) < 5, 255, 0).astype(np.uint8)
    return (((x + y + z) & 1) * 255).astype(np.uint8)   # checker: the largest AC codes


def _append_widths(pkg, plan, fr, depth):
    """Bits per append of the kernel's grouping: [cube, part, append] (append 0 / 1 = group 0's halves,
    then groups 1 ..)."""
    cs = 64 * depth
    q = plan.encode_q(fr).reshape(-1, cs)
    v = q[:, pkg.diagonal_order(8, 8, depth).astype(np.int64)]          # stream order per cube
    code = np.where(v > 0, 2 * v, 1 - 2 * v).astype(np.int64)           # ExpGolomb.c:32-64
    width = 2 * (np.floor(np.log2(code)).astype(np.int64) + 1) - 1
    w = width.reshape(-1, 8, cs // 64, 8)                                # [cube, part, group, code]
    return np.concatenate([w[:, :, :1, :4].sum(3), w[:, :, :1, 4:].sum(3), w[:, :, 1:].sum(3)], axis=2)


@pytest.mark.parametrize("depth", [8, 4])
def test_fused_corpora_cover_emission_branches(pkg, plan8, plan4, depth):
    plan = plan8 if depth == 8 else plan4
    W = np.concatenate([_append_widths(pkg, plan, _content(pkg, k, 64, 64, 2 * depth), depth).ravel()
                        for k in ("ramp", "uniform", "checker", "corner", "edge")])
    assert (W % 2 == 0).all()
    assert (W < 32).sum() > 0                      # fast path, at most one word out
    assert ((W >= 32) & (W < 64)).sum() > 100      # fast path, two words out when bits are pending
    assert (W == 64).sum() > 0                     # the boundary: code by code
    assert (W > 64).sum() > 100                    # code by code (the corner's DC halves)
