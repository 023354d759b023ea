"""CPU: numerically hard LPs (tests/golden/robust_lps.json, HiGHS optima) and the
scaling the solver applies by default (elp_control.scaling = geometric +
equilibrate, lp_solve's default lp.control(scaling = ...), R/class.R:262).

Without scaling, some badly scaled LPs end "optimal" at a wrong vertex (the
absolute 1e-9 tolerances meet entries spanning 1e-8 .. 1e8); with it every
fixture matches HiGHS."""
import numpy as np
import pytest

from conftest import load_robust_lps

ROBUST = load_robust_lps()


def _args(r):
    return r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"]


@pytest.mark.parametrize("rule", [1, 0], ids=["devex", "dantzig"])
@pytest.mark.parametrize("rec", ROBUST, ids=[r["name"] for r in ROBUST])
def test_robust_lps_vs_highs(rec, rule):
    from oracle import solve_dense
    o = solve_dense(*_args(rec), price_rule=rule)
    assert o.status == 0
    assert abs(o.objval - rec["objective"]) <= 1e-9 * max(1.0, abs(rec["objective"]))


@pytest.mark.parametrize("rec", ROBUST, ids=[r["name"] for r in ROBUST])
def test_robust_lps_csc_order(rec):
    from oracle import solve_dense
    o = solve_dense(*_args(rec), price_mode=1)
    assert o.status == 0
    assert abs(o.objval - rec["objective"]) <= 1e-9 * max(1.0, abs(rec["objective"]))


def test_scale_factors_properties():
    from oracle import scale_factors
    for rec in ROBUST:
        A = rec["A"]
        rho, gam = scale_factors(A)
        S = np.abs(A) * np.exp2(rho)[:, None] * np.exp2(gam)[None, :]
        nz = A != 0
        colmax = np.where(nz, S, 0).max(axis=0)
        used = nz.any(axis=0)
        # equilibrate: every nonempty column's largest scaled entry in [1/2, 1)
        assert ((colmax[used] >= 0.5) & (colmax[used] < 1.0)).all(), rec["name"]
        assert (gam[~used] == 0).all()
        # geometric mode alone is a fixed point of one more row + column pass
        r2, g2 = scale_factors(A, 4)
        S2 = np.abs(A) * np.exp2(r2)[:, None] * np.exp2(g2)[None, :]
        e = np.where(nz, np.floor(np.log2(np.where(nz, S2, 1.0))), 0).astype(int)
        for i in np.nonzero(nz.any(axis=1))[0]:
            row = e[i, nz[i]]
            assert -((row.min() + row.max()) // 2) == 0 or abs(row.min() + row.max()) <= 1
    # a matrix spanning 1e-8 .. 1e8 comes out within a few binades of 1
    rec = next(r for r in ROBUST if r["name"] == "badly_scaled_4")
    rho, gam = scale_factors(rec["A"])
    S = np.abs(rec["A"]) * np.exp2(rho)[:, None] * np.exp2(gam)[None, :]
    nzv = S[rec["A"] != 0]
    assert nzv.max() < 1.0 and nzv.min() > 1e-8
    raw = np.abs(rec["A"][rec["A"] != 0])
    assert raw.max() / raw.min() > 1e10


def test_scaling_is_exact_and_transparent():
    """Scaled and unscaled solves of a well-scaled LP reach the same optimum;
    x and y come back in the user's units (powers of two: unscaling is exact)."""
    from oracle import generate_dense, solve_dense
    A, b, c = generate_dense(4, 120, 500)
    dirs = np.ones(120, np.int32)
    a = solve_dense(A, dirs, b, c, maximize=True, scaling=0)
    s = solve_dense(A, dirs, b, c, maximize=True)
    assert a.status == s.status == 0
    np.testing.assert_array_equal(a.basis, s.basis)
    assert abs(a.objval - s.objval) <= 1e-12 * abs(a.objval)
    np.testing.assert_allclose(s.x, a.x, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(s.y, a.y, rtol=1e-10, atol=1e-12)
    assert abs(b @ s.y - s.objval) <= 1e-10 * abs(s.objval)  # duals in user units
