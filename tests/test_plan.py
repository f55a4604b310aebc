"""CPU: the product's transform plan (csrc/dct3d_plan.cpp, via dct3d_plan_query) against the
oracle's independent restatement of DCT.initialize / InverseDCT.initialize, and sanity of the
certification tables the fused kernels use."""
import numpy as np
import pytest


@pytest.mark.parametrize("depth", [8, 4])
def test_plan_matches_oracle_grouping(pkg, plan8, plan4, depth):
    oplan = plan8 if depth == 8 else plan4
    p = pkg.plan_query(8, 8, depth)
    cs = 64 * depth
    assert p["cube_size"] == cs
    assert p["n_mults"] == oplan.n_mults
    assert not p["treeified"]
    for k in range(cs):
        groups = oplan.groups(k)
        assert p["ngroups"][k] == len(groups), k
        # same fold order, same coefficient bits, same membership
        assert np.array_equal(p["coef"][k, : len(groups)], np.array([c for c, _ in groups])), k
        gof = oplan.group_of(k)
        assert np.array_equal(p["group_of"][k].astype(np.int16), gof), k
    assert p["coef_dc"] == groups[0][0] if False else p["coef_dc"] == oplan.groups(0)[0][0]


def test_certification_tables_sane(pkg):
    for depth in (8, 4):
        p = pkg.plan_query(8, 8, depth)
        smax = 7 + 7 + depth - 1
        assert np.isinf(p["enc_E"][0]) and p["enc_G"][0] == 0       # DC never flagged (exact path)
        for s in range(1, smax + 1):
            step = 5 * s
            assert p["enc_rstep"][s] == np.float32(1.0 / step)
            assert 0 < p["enc_G"][s] < 1e-4 and 1e-7 < p["enc_E"][s] < 1e-6
        # the bound per coefficient is small relative to a quantisation step for all s
        assert (p["enc_K"] * 255 < 0.01).all()
        assert 0 < p["dec_G"] < 1e-10


def test_invalid_block_dims(pkg):
    with pytest.raises(pkg.Dct3dError):
        pkg.plan_query(8, 8, 5)
    with pytest.raises(pkg.Dct3dError):
        pkg.plan_query(4, 4, 4)


def test_second_certificate_bound(pkg, oracle, plan8):
    """The 8x8x8 second certificate (e16_recheck64): an fp64 evaluation v64 of every coefficient from
    the cube's bytes and the fp64 basis lies within E64 = (0.5 - thr64[s]) / 2 of Java's fold value
    (DCT.java:44-52, the oracle) in units of the step, on uniform noise and extreme patterns -- and so
    every coefficient it settles (|q64 - rint(q64)| < thr64) rounds to Java's Math.round.  numpy's
    evaluation order differs from the kernel's; the bound (dct3d_plan.cpp) covers any order with at
    most ~24 roundings per term, and the observed error is checked against it with room to spare."""
    p = pkg.plan_query(8, 8, 8)
    thr = p["enc_thr64"]
    assert thr[0] == 0.5
    e64 = (0.5 - thr[1:22]) / 2
    assert (e64 > 0).all() and (e64 < 1e-9).all()
    B = np.array([[(np.sqrt(0.125) if k == 0 else 0.5) * np.cos(np.pi * (2 * n + 1) * k / 16) for n in range(8)]
                  for k in range(8)])
    rng = np.random.default_rng(5)
    z, y, x = np.meshgrid(np.arange(16), np.arange(64), np.arange(64), indexing="ij")
    contents = [rng.integers(0, 256, size=(16, 64, 64)).astype(np.uint8),
                (((x + y + z) % 2) * 255).astype(np.uint8), np.where(z % 8 < 4, 0, 255).astype(np.uint8)]
    s = (np.arange(8)[:, None, None] + np.arange(8)[None, :, None] + np.arange(8)[None, None, :])
    step = np.maximum(1, 5 * s)
    worst = 0.0
    for fr in contents:
        q, d = plan8.encode_q(fr, want_dct=True)
        cubes = oracle.to_cubes(fr).astype(np.float64)             # [n, z, y, x]
        v64 = np.einsum("nzyx,cz,by,ax->ncba", cubes, B, B, B)     # [n, kz, ky, kx]
        java = oracle.to_cubes(d)                                  # Java's fp64 DCT values, cube-major
        err = np.abs(v64 - java) / step
        bound = np.where(s == 0, np.inf, np.concatenate([[np.inf], e64, [np.inf] * 10])[s])
        assert (err <= bound).all()
        worst = max(worst, float((err / bound)[:, s > 0].max()))
        q64 = v64 / step
        settled = (np.abs(q64 - np.rint(q64)) < thr[s]) & (s > 0)
        assert np.array_equal(np.rint(q64)[settled].astype(np.int32), q[settled])
    assert worst < 0.25  # observed ~0.05


def _java_hashmap_fold_order(cw, ch, cd, k0, k1, k2):
    """Closed-form Java 8 HashMap<Long, Multiplication> iteration order for output coefficient
    (k0, k1, k2) of DCT.initialize (DCT.java:93-133), written independently of the planner's
    insert/resize emulation (csrc/dct3d_plan.cpp JavaLongMap) and of the oracle's:
      * the coefficient expression, left to right as javac evaluates it (DCT.java:119), with the
        Transform.java:20-21 constants; the key (long)(c * 1E9), zero keys dropped (DCT.java:122-123);
      * HashMap iteration = bins in index order, each bin's list in insertion order (a resize splits
        a bin into lo/hi lists that keep their relative order, so this holds at the final capacity);
        bin = spread(Long.hashCode(key)) & (cap - 1), spread(h) = h ^ (h >>> 16);
      * final capacity: 16 doubled while size > 0.75 cap (putVal's threshold), valid only if no bin
        ever holds more than TREEIFY_THRESHOLD = 8 nodes (a 9th would resize below 64 or treeify),
        checked for the keys each capacity holds (the first 0.75 cap + 1 inserted).
    Returns the group coefficients in fold order and the fold index of every input n (-1: dropped)."""
    import math
    dim = math.sqrt(math.pow(2.0, 3.0))
    inv_sqrt2 = 1.0 / math.sqrt(2.0)
    f32 = lambda v: float(np.float32(v))
    scale = dim / math.sqrt(cw * ch * cd)
    pw, ph, pd = math.pi / f32(cw), math.pi / f32(ch), math.pi / f32(cd)
    c0 = inv_sqrt2 if k0 == 0 else 1.0
    c1 = inv_sqrt2 if k1 == 0 else 1.0
    c2 = inv_sqrt2 if k2 == 0 else 1.0
    first = {}          # key -> (insertion rank, coefficient)
    key_of = []
    for n0 in range(cd):
        for n1 in range(ch):
            for n2 in range(cw):
                c = scale * c0 * c1 * c2 * math.cos(pd * f32(n0 + 0.5) * k0) * math.cos(ph * f32(n1 + 0.5) * k1) \
                    * math.cos(pw * f32(n2 + 0.5) * k2)
                key = int(c * 1e9)                       # (long) truncates toward zero
                key_of.append(key)
                if key != 0 and key not in first:
                    first[key] = (len(first), c)

    def bin_of(key, cap):
        v = key & 0xFFFFFFFFFFFFFFFF
        h = (v ^ (v >> 32)) & 0xFFFFFFFF                 # Long.hashCode
        return (h ^ (h >> 16)) & (cap - 1)               # HashMap.hash, then index

    cap = 16
    while len(first) > 0.75 * cap:
        cap *= 2
    keys = sorted(first, key=lambda kk: first[kk][0])   # insertion order
    c_ = 16
    while c_ <= cap:                                     # no bin of 9 at any capacity on the way
        held = keys[: int(0.75 * c_) + 1]
        counts = np.bincount([bin_of(kk, c_) for kk in held], minlength=c_)
        assert counts.max() <= 8, (k0, k1, k2, c_)
        c_ *= 2
    order = sorted(first, key=lambda kk: (bin_of(kk, cap), first[kk][0]))
    pos = {kk: i for i, kk in enumerate(order)}
    coefs = np.array([first[kk][1] for kk in order])
    gof = np.array([pos[kk] if kk != 0 else -1 for kk in key_of])
    return coefs, gof


@pytest.mark.parametrize("depth", [8, 4])
def test_hashmap_fold_order_closed_form(pkg, plan8, plan4, depth):
    """the Java fold order decides the quantised value at exact ties (8x8x4: the
    4-point k = 2 row is +-1/2; 8x8x8: e.g. k = (0, 2, 2), tests/test_gpu_parity.py).  The closed form
    above must give, for every output coefficient, the same group coefficients in the same order and
    the same membership as the product's planner (dct3d_plan_query) and the oracle."""
    p = pkg.plan_query(8, 8, depth)
    oplan = plan8 if depth == 8 else plan4
    cs = 64 * depth
    for k in range(cs):
        k0, k1, k2 = k // 64, (k // 8) % 8, k % 8
        coefs, gof = _java_hashmap_fold_order(8, 8, depth, k0, k1, k2)
        ng = len(coefs)
        assert p["ngroups"][k] == ng, k
        assert np.array_equal(p["coef"][k, :ng], coefs), k          # bit-identical, same order
        assert np.array_equal(np.where(p["group_of"][k] == 0xFF, -1, p["group_of"][k].astype(np.int64)), gof), k
        assert np.array_equal(np.array([c for c, _ in oplan.groups(k)]), coefs), k


def _cos_args(n):
    """Every argument DCT.initialize / InverseDCT.initialize pass to Math.cos for one axis of length n
    (DCT.java:104-112, InverseDCT.java:110-124): (Math.PI / (float) n) * (m + 0.5f) * k, left to right."""
    import math
    f32 = lambda v: float(np.float32(v))
    p = math.pi / f32(n)
    return {(m, k): p * f32(m + 0.5) * k for m in range(n) for k in range(n)}


def test_libm_cos_correctly_rounded_at_plan_arguments():
    """VERDICT r2 #6 (Math.cos residual): Java's Math.cos is specified only to 1 ulp, the planner, the
    oracle and this interpreter use glibc cos.  At every argument the Java plan evaluates (8-point and
    4-point axes), glibc returns the correctly rounded cosine (mpmath at 60 digits), so the planner's
    coefficient bits equal those of any Java whose Math.cos is correctly rounded there."""
    import math
    import mpmath
    mpmath.mp.dps = 60
    for n in (8, 4):
        for (m, k), a in _cos_args(n).items():
            exact = mpmath.cos(mpmath.mpf(a))          # the double a, exactly, then cos to 60 digits
            got = math.cos(a)
            # correctly rounded: |exact - cos(a)| <= half an ulp of cos(a)
            assert abs(exact - mpmath.mpf(got)) <= mpmath.mpf(math.ulp(got)) / 2, (n, m, k, a)


def _plan_coefficients(depth):
    """Every DCT.initialize coefficient (DCT.java:104-112) as [k0, k1, k2, n0, n1, n2] float64, the
    product evaluated left to right as javac does, with glibc cos, plus the number of non-trivial
    cosine factors (k != 0: cos(0) = 1 exactly in any libm) of each."""
    import math
    cd = depth
    scale = math.sqrt(math.pow(2.0, 3.0)) / math.sqrt(64 * cd)
    inv_sqrt2 = 1.0 / math.sqrt(2.0)
    ax = {n: _cos_args(n) for n in (8, 4)}
    cosd = np.array([[math.cos(ax[cd][(m, k)]) for m in range(cd)] for k in range(cd)])   # [k][n]
    cosh = np.array([[math.cos(ax[8][(m, k)]) for m in range(8)] for k in range(8)])
    cvec = lambda n: np.array([inv_sqrt2] + [1.0] * (n - 1))
    c = scale * cvec(cd)[:, None, None, None, None, None]
    c = c * cvec(8)[None, :, None, None, None, None]
    c = c * cvec(8)[None, None, :, None, None, None]
    c = c * cosd[:, None, None, :, None, None]
    c = c * cosh[None, :, None, None, :, None]
    c = c * cosh[None, None, :, None, None, :]
    nt = ((np.arange(cd) != 0)[:, None, None] + (np.arange(8) != 0)[None, :, None]
          + (np.arange(8) != 0)[None, None, :]).astype(int)
    return c, np.broadcast_to(nt[:, :, :, None, None, None], c.shape)


@pytest.mark.parametrize("depth", [8, 4])
def test_grouping_keys_stable_under_cos_ulp(depth):
    """how far the Java grouping depends on Math.cos's last bit.  A cosine 1 ulp off the
    correctly rounded one moves a coefficient by at most ~3 ulp (plus re-roundings of the product); the
    group key is (long)(c * 1E9) (DCT.java:115).
      * Every coefficient whose exact real value times 1E9 is NOT an integer keeps its key under any
        relative move of 2^-44 (~200x the largest 1-ulp effect).
      * The others are the rational coefficients: c = +-1/32 or +-1/16 exactly (e.g. k = (0, 2, 2) at
        8^3: 1/8 * 1/sqrt2 * cos(pi/8) cos(3pi/8) = 1/32; 8x8x4's k0 = 2 row is +-sqrt2/2).  Their fp64
        values straddle the integer key (31249999.99999999 -> 31249999, 31250000.0 -> 31250000), so their
        keys -- hence the groups and the HashMap fold order of those k -- are decided by the cosine bits.
        For them the plan equals Java's iff Math.cos is correctly rounded at their arguments, which is what
        glibc returns (test_libm_cos_correctly_rounded_at_plan_arguments).  The residual is therefore
        exactly: "a JVM whose Math.cos is not correctly rounded at one of these arguments"."""
    import mpmath
    mpmath.mp.dps = 40
    c, nt = _plan_coefficients(depth)
    x = c * 1e9
    eps = 2.0 ** -44
    moved = (np.trunc(x * (1 - eps)) != np.trunc(x * (1 + eps))) & (nt > 0)
    # every key that can move belongs to a coefficient whose exact value * 1E9 is an integer
    kk = np.argwhere(moved)
    exact_rational = {}
    for k0, k1, k2, n0, n1, n2 in kk:
        key = (int(k0), int(k1), int(k2), int(n0), int(n1), int(n2))
        cd = depth
        e = (mpmath.sqrt(8) / mpmath.sqrt(64 * cd)
             * (1 / mpmath.sqrt(2) if k0 == 0 else 1) * (1 / mpmath.sqrt(2) if k1 == 0 else 1)
             * (1 / mpmath.sqrt(2) if k2 == 0 else 1)
             * mpmath.cos(mpmath.pi / cd * (n0 + mpmath.mpf(1) / 2) * k0)
             * mpmath.cos(mpmath.pi / 8 * (n1 + mpmath.mpf(1) / 2) * k1)
             * mpmath.cos(mpmath.pi / 8 * (n2 + mpmath.mpf(1) / 2) * k2)) * 10 ** 9
        assert abs(e - mpmath.nint(e)) < mpmath.mpf(10) ** -20, key
        exact_rational[key[:3]] = exact_rational.get(key[:3], 0) + 1
    # the sensitive outputs: 24 at 8^3 (kz, ky, kx in {0, 2, 6} patterns), 39 at 8x8x4
    assert len(exact_rational) == {8: 24, 4: 39}[depth], len(exact_rational)
    # all other keys sit far from an integer boundary
    nz = (np.abs(x) >= 1.0) & ~moved & (nt > 0)
    frac = np.abs(x[nz] - np.round(x[nz])) / np.abs(x[nz])
    assert frac.min() > eps, frac.min()
