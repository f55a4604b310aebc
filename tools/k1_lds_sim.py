"""LDS bank conflicts of K1's code staging (encode_eg_kernel<8>, dct3d_kernels.hip), simulated by the bank
rules of MI355X_MICROARCH.md §LDS:
  * the staging stores: ds_write_b128, lane groups of 8 contiguous lanes = one cube's 8 faces (lane (c, kz)
    writes row ky of face kz), bank = (a/4) mod 32: 8 rows in one 4-bank group = 7 extra cycles per group;
  * the emission's code reads: ds_read_u16 (as b32: 2 groups of 32 lanes, bank = (a/4) mod 32, identical
    dwords broadcast), lane (cp, part) reading stream position part*64 + i of cube cp at step i.
Layouts: `plain` row ky of face kz at kz*128 + ky*16 (rounds 4-5), `rot` at kz*128 + ((ky + kz) mod 8)*16
(round 6).  Cubes 1,056 B apart.  CPU only.
    python tools/k1_lds_sim.py"""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module('3ddctvideoencoding_amd')

CUBE_B = 1056


def layout(kind):
    """byte offset of code k = (kz*8 + ky)*8 + kx within a cube"""
    k = np.arange(512)
    kz, ky, kx = k >> 6, (k >> 3) & 7, k & 7
    slot = ky if kind == 'plain' else (ky + kz) & 7
    return kz * 128 + slot * 16 + kx * 2


def read_extra(off, diag):
    tot = 0
    for i in range(64):
        for g in (0, 1):
            banks = {}
            for lane in range(32 * g, 32 * g + 32):
                cp, part = lane >> 3, lane & 7
                dw = (cp * CUBE_B + off[diag[part * 64 + i]]) // 4
                banks.setdefault(dw % 32, set()).add(dw)
            tot += max(len(v) for v in banks.values()) - 1
    return tot / 64


def write_extra(off):
    tot = 0
    for ky in range(8):
        for c in range(8):  # one lane group = cube c, kz = 0..7
            groups = {}
            for kz in range(8):
                a = c * CUBE_B + off[(kz * 8 + ky) * 8]
                groups.setdefault((a // 16) % 8, set()).add(a)
            tot += max(len(v) for v in groups.values()) - 1
    return tot / 8


def main():
    diag = pkg.diagonal_order(8, 8, 8).astype(np.int64)
    for kind in ('plain', 'rot'):
        off = layout(kind)
        print(f"{kind:6s} code reads: {read_extra(off, diag):.2f} extra cycles per ds_read_u16; "
              f"staging stores: {write_extra(off):.1f} extra cycles per ds_write_b128")


if __name__ == '__main__':
    main()
