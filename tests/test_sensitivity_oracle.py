"""CPU: the oracle's sensitivity report (R/class.R:613-646 semantics, textbook
ranging -- lp_solve itself is absent, parity with it is unpinned) on a textbook
LP with published ranges, and by brute force: inside a reported range the
optimal basis does not change, just outside it does."""
import numpy as np
import pytest

from conftest import load_sparse_lps


def _solve(A, dirs, b, c, lo=None, up=None, mx=True, **kw):
    from oracle import solve_dense
    return solve_dense(A, dirs, b, c, lo, up, mx, **kw)


def test_wyndor_textbook_ranges():
    """Hillier & Lieberman's Wyndor Glass LP: max 3x1 + 5x2, x1 <= 4, 2x2 <= 12,
    3x1 + 2x2 <= 18; duals (0, 1.5, 1), 0 <= c1 <= 7.5, c2 >= 2,
    b1 >= 2, 6 <= b2 <= 18, 12 <= b3 <= 24."""
    A = np.array([[1, 0], [0, 2], [3, 2.0]])
    r = _solve(A, [1, 1, 1], [4, 12, 18], [3, 5], sens=True)
    s = r.sens
    np.testing.assert_allclose(s["duals"][:3], [0, 1.5, 1], atol=1e-12)
    np.testing.assert_allclose(s["objfrom"], [0, 2], atol=1e-12)
    np.testing.assert_allclose(s["objtill"], [7.5, 1e30])
    np.testing.assert_allclose(s["dualsfrom"][:3], [2, 6, 12])
    np.testing.assert_allclose(s["dualstill"][:3], [1e30, 18, 24])


def _random_lp(seed, m=12, n=20):
    rng = np.random.default_rng(seed)
    A = rng.uniform(0, 1, (m, n))
    b = rng.uniform(2, 5, m)
    c = rng.uniform(0.5, 2, n)
    return A, np.ones(m, np.int32), b, c


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_objective_ranges_keep_basis(seed):
    A, d, b, c = _random_lp(seed)
    r = _solve(A, d, b, c, sens=True)
    for j in range(len(c)):
        lo, hi = r.sens["objfrom"][j], r.sens["objtill"][j]
        for t in (0.25, 0.75):
            if lo > -1e29 and hi < 1e29:
                cj = lo + t * (hi - lo)
            elif lo > -1e29:
                cj = lo + t * (1 + abs(lo))
            else:
                cj = hi - t * (1 + abs(hi))
            c2 = c.copy()
            c2[j] = cj
            assert np.array_equal(_solve(A, d, b, c2).basis, r.basis), (j, lo, hi, cj)
        if hi < 1e29:  # just beyond the upper limit the basis is no longer optimal
            c2 = c.copy()
            c2[j] = hi + 1e-3 * (1 + abs(hi))
            assert not np.array_equal(_solve(A, d, b, c2).basis, r.basis)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_rhs_ranges_keep_basis(seed):
    A, d, b, c = _random_lp(seed)
    r = _solve(A, d, b, c, sens=True)
    m = len(b)
    for i in range(m):
        lo, hi = r.sens["dualsfrom"][i], r.sens["dualstill"][i]
        lo_f = lo if lo > -1e29 else b[i] - 1.0
        hi_f = hi if hi < 1e29 else b[i] + 1.0
        for t in (0.2, 0.8):
            b2 = b.copy()
            b2[i] = lo_f + t * (hi_f - lo_f)
            r2 = _solve(A, d, b2, c, sens=True)
            # same basis, same duals
            assert np.array_equal(r2.basis, r.basis), (i, lo, hi, b2[i])
            np.testing.assert_allclose(r2.sens["duals"][:m], r.sens["duals"][:m], atol=1e-9)


def test_min_sense_and_bounds():
    """min problem with boxed and free columns and >= / == rows: every reported
    objective range keeps the basis (both interior points)."""
    rng = np.random.default_rng(7)
    m, n = 8, 14
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 1, n)
    dirs = np.array([2, 2, 3, 1, 1, 2, 1, 1], np.int32)
    b = A @ x0 + np.where(dirs == 1, 0.5, np.where(dirs == 2, -0.5, 0.0))
    lo = np.zeros(n)
    up = np.full(n, 2.0)
    c = rng.uniform(-1, 1, n)
    r = _solve(A, dirs, b, c, lo, up, False, sens=True)
    assert r.status == 0
    for j in range(n):
        lo_j, hi_j = r.sens["objfrom"][j], r.sens["objtill"][j]
        lo_f = lo_j if lo_j > -1e29 else c[j] - 1.0
        hi_f = hi_j if hi_j < 1e29 else c[j] + 1.0
        c2 = c.copy()
        c2[j] = 0.5 * (lo_f + hi_f)
        assert np.array_equal(_solve(A, dirs, b, c2, lo, up, False).basis, r.basis)


def test_sparse_fixture_sensitivity_column_order():
    from oracle import solve_dense
    rec = next(r for r in load_sparse_lps() if r["name"] == "packing_s2_60x200")
    r = solve_dense(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                    rec["maximize"], sens=True, price_mode=1)
    assert r.status == 0 and r.sens is not None
    # basic columns have a two-sided range containing c_j
    basic = [j for j in r.basis if j < len(rec["obj"])]
    for j in basic:
        assert r.sens["objfrom"][j] <= rec["obj"][j] <= r.sens["objtill"][j]
