"""fdlibm 5.3's cos, restated in Python doubles (the JVM cosine behind the exact-tie
residual).

Java's StrictMath.cos is specified as fdlibm's algorithm (java.lang.StrictMath's class comment; JDK 8
links fdlibm 5.3's C, later JDKs carry a Java port, FdLibm.java, of the same code), and HotSpot's
SharedRuntime::dcos -- the Math.cos of the interpreter and of JIT builds without a platform libm
intrinsic -- is the same fdlibm source.  The restated routines follow the published algorithm:

  s_cos.c           cos(x): |x| <= pi/4 -> __kernel_cos(x, 0); else n = __ieee754_rem_pio2(x, y) and,
                    by n mod 4, +-__kernel_cos(y0, y1) or +-__kernel_sin(y0, y1, 1)
  e_rem_pio2.c      x - n pi/2 as y0 + y1: |x| < 3pi/4 with the 33 + 53-bit pi/2 (n = 1); medium
                    |x| <= 2^19 pi/2 by Cody-Waite with up to three pieces of pi/2
  k_cos.c, k_sin.c  the minimax polynomials on [-pi/4, pi/4]

Python floats are IEEE binary64 with round-to-nearest and no contraction, so evaluating fdlibm's
expressions in its order reproduces its bits.  Every constant is built from its hex words (as fdlibm
writes them in comments) and checked against its decimal form at import.  Only the paths the DCT plans
reach are restated (|x| < 2^19 pi/2; the large-argument __kernel_rem_pio2 path raises).

CPU only, measurement/test support (tests/test_fdlibm_cos.py); nothing in the product imports it."""
import math
import struct


def _hw(x):
    """fdlibm's __HI(x): the high 32-bit word, as a signed int"""
    return struct.unpack('<q', struct.pack('<d', x))[0] >> 32


def _from_words(hi, lo):
    return struct.unpack('<d', struct.pack('<Q', ((hi & 0xFFFFFFFF) << 32) | (lo & 0xFFFFFFFF)))[0]


def _with_hi(hi, lo=0):
    return _from_words(hi, lo)


def _const(hi, lo, dec):
    v = _from_words(hi, lo)
    assert v == float(dec), (hex(hi), hex(lo), dec, v)
    return v


# k_cos.c
C1 = _const(0x3FA55555, 0x5555554C, '4.16666666666666019037e-02')
C2 = _const(0xBF56C16C, 0x16C15177, '-1.38888888888741095749e-03')
C3 = _const(0x3EFA01A0, 0x19CB1590, '2.48015872894767294178e-05')
C4 = _const(0xBE927E4F, 0x809C52AD, '-2.75573143513906633035e-07')
C5 = _const(0x3E21EE9E, 0xBDB4B1C4, '2.08757232129817482790e-09')
C6 = _const(0xBDA8FAE9, 0xBE8838D4, '-1.13596475577881948265e-11')
# k_sin.c
S1 = _const(0xBFC55555, 0x55555549, '-1.66666666666666324348e-01')
S2 = _const(0x3F811111, 0x1110F8A6, '8.33333333332248946124e-03')
S3 = _const(0xBF2A01A0, 0x19C161D5, '-1.98412698298579493134e-04')
S4 = _const(0x3EC71DE3, 0x57B1FE7D, '2.75573137070700676789e-06')
S5 = _const(0xBE5AE5E6, 0x8A2B9CEB, '-2.50507602534068634195e-08')
S6 = _const(0x3DE5D93A, 0x5ACFD57C, '1.58969099521155010221e-10')
# e_rem_pio2.c
INVPIO2 = _const(0x3FE45F30, 0x6DC9C883, '6.36619772367581382433e-01')
PIO2_1 = _const(0x3FF921FB, 0x54400000, '1.57079632673412561417e+00')
PIO2_1T = _const(0x3DD0B461, 0x1A626331, '6.07710050650619224932e-11')
PIO2_2 = _const(0x3DD0B461, 0x1A600000, '6.07710050630396597660e-11')
PIO2_2T = _const(0x3BA3198A, 0x2E037073, '2.02226624879595063154e-21')
PIO2_3 = _const(0x3BA3198A, 0x2E000000, '2.02226624871116645580e-21')
PIO2_3T = _const(0x397B839A, 0x252049C1, '8.47842766036889956997e-32')
# high words of n * pi/2, n = 1 .. 32 (the quick no-cancellation check)
NPIO2_HW = [
    0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C,
    0x4025FDBB, 0x402921FB, 0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C,
    0x40346B9C, 0x4035FDBB, 0x40378FDB, 0x403921FB, 0x403AB41B, 0x403C463A,
    0x403DD85A, 0x403F6A7A, 0x40407E4C, 0x4041475C, 0x4042106C, 0x4042D97C,
    0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB, 0x4046C6CB, 0x40478FDB,
    0x404858EB, 0x404921FB,
]
for _n, _h in enumerate(NPIO2_HW, 1):  # each entry is the high word of n * pi/2
    assert _hw(_n * (math.pi / 2)) == _h, (_n, hex(_h))


def kernel_cos(x, y):
    """k_cos.c: cos(x + y) for |x| <= pi/4, y the tail of x"""
    ix = _hw(x) & 0x7FFFFFFF
    if ix < 0x3E400000 and int(x) == 0:  # |x| < 2^-27
        return 1.0
    z = x * x
    r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))))
    if ix < 0x3FD33333:  # |x| < 0.3
        return 1.0 - (0.5 * z - (z * r - x * y))
    qx = 0.28125 if ix > 0x3FE90000 else _with_hi(ix - 0x00200000, 0)  # x > 0.78125, else x / 4
    hz = 0.5 * z - qx
    a = 1.0 - qx
    return a - (hz - (z * r - x * y))


def kernel_sin(x, y, iy):
    """k_sin.c: sin(x + y) for |x| <= pi/4 (iy = 0: y is zero)"""
    ix = _hw(x) & 0x7FFFFFFF
    if ix < 0x3E400000 and int(x) == 0:
        return x
    z = x * x
    v = z * x
    r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))
    if iy == 0:
        return x + v * (S1 + z * r)
    return x - ((z * (0.5 * y - v * r) - y) - v * S1)


def rem_pio2(x):
    """e_rem_pio2.c for |x| <= 2^19 pi/2: (n, y0, y1) with x - n pi/2 = y0 + y1"""
    hx = _hw(x)
    ix = hx & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return 0, x, 0.0
    if ix < 0x4002D97C:  # |x| < 3pi/4: n = +-1
        if hx > 0:
            z = x - PIO2_1
            if ix != 0x3FF921FB:
                y0 = z - PIO2_1T
                y1 = (z - y0) - PIO2_1T
            else:  # near pi/2: 33 + 33 + 53-bit pi/2
                z -= PIO2_2
                y0 = z - PIO2_2T
                y1 = (z - y0) - PIO2_2T
            return 1, y0, y1
        z = x + PIO2_1
        if ix != 0x3FF921FB:
            y0 = z + PIO2_1T
            y1 = (z - y0) + PIO2_1T
        else:
            z += PIO2_2
            y0 = z + PIO2_2T
            y1 = (z - y0) + PIO2_2T
        return -1, y0, y1
    if ix <= 0x413921FB:  # medium: |x| ~<= 2^19 pi/2
        t = abs(x)
        n = int(t * INVPIO2 + 0.5)
        fn = float(n)
        r = t - fn * PIO2_1
        w = fn * PIO2_1T  # first round, good to 85 bits
        if n < 32 and ix != NPIO2_HW[n - 1]:
            y0 = r - w  # quick check: no cancellation
        else:
            j = ix >> 20
            y0 = r - w
            i = j - ((_hw(y0) >> 20) & 0x7FF)
            if i > 16:  # second iteration, good to 118 bits
                t = r
                w = fn * PIO2_2
                r = t - w
                w = fn * PIO2_2T - ((t - r) - w)
                y0 = r - w
                i = j - ((_hw(y0) >> 20) & 0x7FF)
                if i > 49:  # third iteration, 151 bits
                    t = r
                    w = fn * PIO2_3
                    r = t - w
                    w = fn * PIO2_3T - ((t - r) - w)
                    y0 = r - w
        y1 = (r - y0) - w
        if hx < 0:
            return -n, -y0, -y1
        return n, y0, y1
    raise NotImplementedError('large arguments (__kernel_rem_pio2) are not reached by the DCT plans')


def cos(x):
    """s_cos.c"""
    ix = _hw(x) & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return kernel_cos(x, 0.0)
    if ix >= 0x7FF00000:
        return x - x
    n, y0, y1 = rem_pio2(x)
    q = n & 3
    if q == 0:
        return kernel_cos(y0, y1)
    if q == 1:
        return -kernel_sin(y0, y1, 1)
    if q == 2:
        return -kernel_cos(y0, y1)
    return kernel_sin(y0, y1, 1)


def plan_args(n):
    """every argument DCT.initialize / InverseDCT.initialize pass to Math.cos on an axis of length n
    (DCT.java:83-112, InverseDCT.java:110-124): (Math.PI / (float) n) * (m + 0.5f) * k, left to right"""
    import numpy as np
    f32 = lambda v: float(np.float32(v))
    p = math.pi / f32(n)
    return {(m, k): p * f32(m + 0.5) * k for m in range(n) for k in range(n)}


if __name__ == '__main__':
    for n in (8, 4):
        diff = [(mk, a) for mk, a in plan_args(n).items() if cos(a) != math.cos(a)]
        print(f'{n}-point axis: {len(plan_args(n))} arguments, fdlibm != glibc at {len(diff)}')
