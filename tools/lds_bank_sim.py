"""LDS bank conflicts of the stream decode's parse passes, simulated.

The sync and mark passes (csrc/dct3d_eg.hip) parse one 512-bit chunk per thread out of the block's LDS
window; lane t of a wave starts at window word 16 t.  Every lean step reads one window word (the refill
word `s[c.nx]`), all lanes of the wave at the same step (SIMT), so a ds_read_b32 of that step has the
lanes' word indices nx_t(k).  This replays the lean loops of both passes bit for bit (lean_step /
lean_step2, 32-bit arithmetic) on the oracle-written stream of a slice of the bench content and counts,
per ds_read_b32, the extra LDS cycles of the bank rule in MI355X_MICROARCH.md §LDS (two groups of 32
lanes, bank = dword address mod 32, identical addresses broadcast, N distinct addresses on one bank =
N - 1 extra cycles), under several window layouts:

  linear   word i at dword i                      (rounds 1-4)
  pad17    word i at i + (i >> 4)                 (one spare dword after every chunk)
  trans    word i at (i & 15) * S + (i >> 4)      (chunk-transposed, S = 288 = 9 * 32: the bank of a
                                                   word is its chunk mod 32, whatever its offset)

CPU only; the oracle writes the stream (test infrastructure).
Usage: python tools/lds_bank_sim.py [ramp|uniform] [rows]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'oracle'))
import importlib  # noqa: E402

pkg = importlib.import_module('3ddctvideoencoding_amd')
import oracle  # noqa: E402

M32 = 0xFFFFFFFF
S_T = 288


def clz32(x):
    x &= M32
    return 32 - x.bit_length()


LAYOUTS = {
    'linear': lambda i: i,
    'pad17': lambda i: i + (i >> 4),
    'trans': lambda i: (i & 15) * S_T + (i >> 4),
}


class Lane:
    """Lean state of dct3d_eg.hip: bits [pos, pos + avail) left-aligned in hi:lo, pre = word nx."""

    def __init__(self, win, p):
        self.s = win
        k = p >> 5
        sh = p & 31
        buf = ((win[k] << 32) | win[k + 1]) << sh
        buf &= (1 << 64) - 1
        self.hi, self.lo = buf >> 32, buf & M32
        self.avail = 64 - sh
        self.nx = k + 2
        self.pre = win[self.nx]
        self.reads = [k, k + 1, k + 2]  # the seek's reads (three ds_read_b32)

    def pos(self):
        return self.nx * 32 - self.avail

    def step(self, bounded=False, cap=31, room=32):
        cap_bit = (0x80000000 >> min(room, 31)) if bounded else (0x80000000 >> cap)
        n1 = clz32((~self.hi & M32) | cap_bit)
        b = (((self.hi << 32) | self.lo) << n1) & ((1 << 64) - 1)
        self.avail -= n1
        has = self.avail != 0 and (b >> 63) == 0 and (not bounded or n1 < room)
        hi, lo = b >> 32, b & M32
        if self.avail < 32:
            a = self.avail
            rh = hi | (self.pre >> (a & 31))
            rl = ((self.pre << (32 - a)) & M32) if a else 0
            hi, lo = rh, rl
            self.avail += 32
            self.nx += 1
        self.pre = self.s[self.nx]
        read = self.nx
        zz = clz32(hi)
        bad = has and zz >= 16
        take = has and zz < 16
        w = 2 * zz + 1 if take else 0
        b = (((hi << 32) | lo) << w) & ((1 << 64) - 1)
        self.hi, self.lo = b >> 32, b & M32
        self.avail -= w
        return n1 + (1 if take else 0), bad, read

    def step2(self, cap=31):
        n, bad, read = self.step(False, cap)
        z2 = clz32(self.hi | 1)
        w2 = 2 * z2 + 1
        if not bad and z2 < 16 and w2 <= self.avail:
            b = (((self.hi << 32) | self.lo) << w2) & ((1 << 64) - 1)
            self.hi, self.lo = b >> 32, b & M32
            self.avail -= w2
            n += 1
        return n, bad, read


def lane_reads(win, start, stop, cap):
    """the sequence of word indices the lean loops read (first loop, then the bounded loop)"""
    ln = Lane(win, start)
    first = list(ln.reads)
    loop1, loop2 = [], []
    fast_stop = stop - 128
    bad = False
    while not bad and ln.pos() < fast_stop:
        _, bad, r = ln.step2(cap)
        loop1.append(r)
    while not bad and ln.pos() < stop:
        _, bad, r = ln.step(True, cap, stop - ln.pos())
        loop2.append(r)
    return first, loop1, loop2


def extra_cycles(addrs):
    """extra LDS cycles of one ds_read_b32: addrs[lane] (None: inactive), groups of 32 lanes"""
    tot = 0
    for g in (0, 32):
        banks = {}
        for a in addrs[g:g + 32]:
            if a is not None:
                banks.setdefault(a % 32, set()).add(a)
        if banks:
            tot += max(len(v) for v in banks.values()) - 1
    return tot


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else 'ramp'
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    fr = np.ascontiguousarray(pkg.synthetic.frames(1920, 1080, 8, kind=kind)[:, :rows, :])
    plan = oracle.Plan(8, 8, 8)
    q = plan.encode_q(fr)
    vals = q.reshape(-1, 512)[:, pkg.diagonal_order(8, 8, 8)].ravel().astype(np.int32)
    data = oracle.eg_write(vals)
    words = np.frombuffer(data + b'\0' * (-len(data) % 4), '>u4').astype(np.int64).tolist()
    code = np.where(vals <= 0, -2 * vals.astype(np.int64), 2 * vals.astype(np.int64) - 1) + 1
    L = 2 * np.floor(np.log2(code.astype(np.float64))).astype(np.int64) + 1
    bounds = np.concatenate([[0], np.cumsum(L)])
    nbits = int(bounds[-1])
    print(f'{kind}: {vals.size} values, {nbits / vals.size:.3f} bits/value')
    n_chunks = nbits // 512 - 2
    waves = n_chunks // 64
    res = {}
    for lay, f in LAYOUTS.items():
        res[lay] = {'sync': [0, 0], 'mark': [0, 0]}
    for w in range(waves):
        for pas in ('sync', 'mark'):
            seqs = []
            for l in range(64):
                t = w * 64 + l
                win = words[t * 16:t * 16 + 16 * 3] + [0] * 8  # the lane's chunk and slack, offset 0
                # window-relative: the chunk starts at word 0 of `win`; the layouts take the word's
                # block-window index 16 * (l + 64 * (w % 4)) + i
                if pas == 'sync':
                    st = 0
                    cap = 31
                else:
                    st = int(bounds[np.searchsorted(bounds, t * 512)]) - t * 512
                    cap = 30
                first, a, b = lane_reads(win, st, 512, cap)
                base = 16 * (l + 64 * (w % 4))
                seqs.append(([base + i for i in first], [base + i for i in a], [base + i for i in b]))
            for lay, f in LAYOUTS.items():
                ins = ext = 0
                for part in range(3):
                    n = max(len(s[part]) for s in seqs)
                    for k in range(n):
                        addrs = [f(s[part][k]) if k < len(s[part]) else None for s in seqs]
                        ext += extra_cycles(addrs)
                        ins += 1
                res[lay][pas][0] += ins
                res[lay][pas][1] += ext
    print(f'{waves} waves of 64 chunks; per parse-read ds_read_b32 instruction, extra LDS cycles:')
    for lay in LAYOUTS:
        print(f"  {lay:7s} sync {res[lay]['sync'][1] / res[lay]['sync'][0]:.2f}   mark {res[lay]['mark'][1] / res[lay]['mark'][0]:.2f}"
              f"   ({res[lay]['sync'][0] / waves:.1f} / {res[lay]['mark'][0] / waves:.1f} reads per wave)")
    # the staging stores: thread i of the block writes window word i + 256 b (ds_write_b32)
    for lay, f in LAYOUTS.items():
        ext = sum(extra_cycles([f(i + 256 * b) for i in range(g, g + 64)]) for b in range(17) for g in (0, 64, 128, 192))
        print(f'  staging stores, {lay}: {ext / (17 * 4):.2f} extra cycles per ds_write_b32')


if __name__ == '__main__':
    main()
