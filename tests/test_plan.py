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
