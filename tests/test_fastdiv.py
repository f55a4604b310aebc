"""CPU: the kernels' address-map division (FastDiv, dct3d_kernels.h; fast_div in dct3d_runtime.cpp):
floor(n * m / 2^s) with s = 31 + ceil(log2 d), m = ceil(2^s / d) equals n // d for every n < 2^31.
Restated here from the two source lines; checked at every kind of boundary (multiples of d and their
neighbours, the top of the range) for the geometries' divisors and random ones."""
import numpy as np


def fast_div(d):
    l = 0
    while (1 << l) < d:
        l += 1
    s = 31 + l
    return ((1 << s) + d - 1) // d, s


def test_fastdiv_matches_integer_division():
    rng = np.random.default_rng(3)
    divisors = {1, 2, 3, 5, 7, 8, 60, 135, 240, 480, 1024, 32400, 129600, 2**16 + 1}
    divisors |= set(rng.integers(1, 2**20, size=100).tolist())
    for d in sorted(divisors):
        m, s = fast_div(d)
        assert m < 2**32
        k = rng.integers(0, (2**31 - 1) // d + 1, size=300).astype(np.uint64)
        n = np.concatenate([np.arange(0, 3 * d + 3, dtype=np.uint64)[:2000], k * d, k * d + (d - 1),
                            np.array([2**31 - 1], np.uint64)])
        n = n[n < 2**31]
        # n * m < 2^63: exact in uint64
        assert np.array_equal((n * np.uint64(m)) >> np.uint64(s), n // np.uint64(d)), d
