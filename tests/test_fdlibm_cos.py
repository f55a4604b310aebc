"""CPU: the exact-tie residual against the JVM cosine that StrictMath specifies.

tools/fdlibm_cos.py restates fdlibm 5.3's cos (s_cos.c, e_rem_pio2.c, k_cos.c, k_sin.c): Java's
StrictMath.cos, and HotSpot's SharedRuntime::dcos (the Math.cos of the interpreter and of builds without a
platform libm intrinsic).  DCT.initialize / InverseDCT.initialize (DCT.java:83-112, InverseDCT.java:110-124)
take Math.cos at 64 arguments per 8-point axis and 16 per 4-point axis.  Found here:

  * fdlibm returns glibc's (correctly rounded) bits at every argument but two distinct ones of the
    8-point axis -- (pi/8) * 2.5 * 7 = (pi/8) * 3.5 * 5 and (pi/8) * 7.5 * 3 -- where it is 1 ulp above;
  * the plan built with those two cosines (the oracle's alternative-plan hook, java_dct3d.c cosalt)
    changes no quantised output and no decoded byte of any committed corpus: 0 of 1.66e8 / 4.98e7
    outputs at 8x8x8 / 8x8x4 (the whole-corpus run, `python tools/cos_ulp_sensitivity.py --fdlibm`:
    profiles/r05/fdlibm_residual.json; here the whole 64x64 fixtures, every cube re-run).

So a JVM whose Math.cos is fdlibm's reproduces the oracle (and the GPU) exactly on every corpus; the counted
residual of tests/test_cos_residual.py (<= 4.1e-5 at 8x8x4) covers only JVMs with another Math.cos (e.g. a
platform intrinsic that is not correctly rounded at one of the plan's arguments)."""
import json
import math
import os
import random
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import fdlibm_cos  # noqa: E402  (asserts every constant against its hex words at import)
import cos_ulp_sensitivity as study  # noqa: E402


def test_fdlibm_restatement_within_one_ulp():
    """fdlibm documents |error| < 1 ulp; a wrong constant or a misordered expression breaks that badly"""
    import mpmath
    mpmath.mp.dps = 50
    rng = random.Random(5)
    worst = 0.0
    for _ in range(4000):
        x = rng.uniform(-25.0, 25.0)
        c = fdlibm_cos.cos(x)
        err = abs(mpmath.mpf(c) - mpmath.cos(mpmath.mpf(x))) / mpmath.mpf(math.ulp(c))
        worst = max(worst, float(err))
    assert worst < 1.0, worst
    # reduction paths: |x| <= pi/4, n = +-1 (|x| < 3 pi / 4), medium, and near multiples of pi/2
    for x in (0.0, 1e-9, 0.3, 0.78, 1.0, 2.0, -2.0, math.pi / 2, 3 * math.pi / 2, 10 * math.pi / 2, 20.6):
        assert abs(fdlibm_cos.cos(x) - math.cos(x)) <= math.ulp(math.cos(x)), x


def test_fdlibm_vs_glibc_at_plan_arguments():
    diff = {}
    for n in (8, 4):
        for (m, k), a in fdlibm_cos.plan_args(n).items():
            f, g = fdlibm_cos.cos(a), math.cos(a)
            if f != g:
                assert f == math.nextafter(g, math.inf), (n, m, k)  # one ulp above
                diff[(n, m, k)] = a
    assert sorted(diff) == [(8, 2, 7), (8, 3, 5), (8, 7, 3)], diff
    assert len(set(diff.values())) == 2  # 2.5 * 7 = 3.5 * 5: one argument
    assert study.fdlibm_cos_ulp() == {a: 1 for a in diff.values()}


@pytest.mark.parametrize("depth", [8, 4])
def test_fdlibm_plan_changes_no_output_on_fixtures(oracle, depth):
    """the whole 64x64 corpora (encode and decode) under the fdlibm plan: identical to the glibc plan"""
    base = oracle.Plan(8, 8, depth)
    alt = oracle.Plan(8, 8, depth, cos_ulp=study.fdlibm_cos_ulp())
    for name, fr in study.corpora(depth, quick=True):
        c = study.Corpus(name, fr, base)
        assert c.run(alt, full=True)[:2] == (0, 0), name


def test_fdlibm_whole_corpus_record():
    r = json.load(open(os.path.join(REPO, "profiles", "r05", "fdlibm_residual.json")))
    assert r["depth8"]["total_coefficients"] == 165953536 and r["depth8"]["changed_encode"] == 0
    assert r["depth4"]["total_coefficients"] == 49799168 and r["depth4"]["changed_encode"] == 0
    assert r["depth8"]["changed_decode"] == 0 and r["depth4"]["changed_decode"] == 0
