"""Integer-only deterministic synthetic grayscale frames (host side).

Bit-identical to the device generator ``dct3d_fill_synthetic_dev`` (csrc/dct3d_kernels.hip,
synth_kernel).  For global pixel index idx = ((frame0 + f) * height + y) * width + x:
  "ramp"    : clamp(128 + ((3x + 5y + 7(frame0+f)) & 63) - 32 + (splitmix64(seed ^ idx) & 15), 0, 255)
  "uniform" : splitmix64(seed ^ idx) & 255
The ramp+noise content (values 96..174, smooth gradients plus 4-bit noise) stands in for
grayscale screen captures (README.md:24); "uniform" is the high-entropy stress case.
"""
from __future__ import annotations

import numpy as np

DEFAULT_SEED = 0x3DDC7


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def frames(width: int, height: int, n_frames: int, seed: int = DEFAULT_SEED, frame0: int = 0,
           kind: str = "ramp") -> np.ndarray:
    """u8 frames [n_frames, height, width]."""
    plane = width * height
    out = np.empty((n_frames, height, width), np.uint8)
    y, x = np.meshgrid(np.arange(height, dtype=np.int64), np.arange(width, dtype=np.int64), indexing="ij")
    for f in range(n_frames):
        gf = frame0 + f
        idx = np.arange(gf * plane, (gf + 1) * plane, dtype=np.uint64).reshape(height, width)
        h = splitmix64(np.uint64(seed) ^ idx)
        if kind == "uniform":
            out[f] = (h & np.uint64(255)).astype(np.uint8)
        elif kind == "ramp":
            v = 128 + ((3 * x + 5 * y + 7 * gf) & 63) - 32 + (h & np.uint64(15)).astype(np.int64)
            out[f] = np.clip(v, 0, 255).astype(np.uint8)
        else:
            raise ValueError(kind)
    return out
