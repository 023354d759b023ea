"""Pin the CPU oracle (oracle/) to the reference's known answers and to the
HiGHS fixtures, before it is trusted as the checker for the HIP path.

Reference anchors: tests/testthat/test-DOP.R:53, tests/testthat/test-unbounded.R:8-9,
README.md:14-38, vignettes (see tests/golden/make_golden.py for each source line).
"""
import numpy as np
import pytest

from conftest import feasible, load_dense_lps, load_generator_vectors, load_known_answers
from oracle import generate_dense, solve_dense

KNOWN = load_known_answers()
DENSE = load_dense_lps()


@pytest.mark.parametrize("rule", [1, 0], ids=["devex", "dantzig"])
@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answer(rec, rule):
    r = solve_dense(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                    rec["maximize"], price_rule=rule)
    exp = rec["expected"]
    assert r.status == exp["status"]
    if r.status == 3:
        # lp_solve reports 1e30; R/utils.R:172-176 turns it into +-Inf.
        assert r.objval == exp["objective"]
        if "x" in exp:
            np.testing.assert_array_equal(r.x, exp["x"])
        return
    if r.status != 0:
        return
    assert feasible(rec["A"], rec["dir"], rec["rhs"], r.x, rec["lo"], rec["up"])
    obj = exp["objective"]
    assert abs(r.objval - obj) <= 1e-9 * max(1.0, abs(obj))
    if "objective_value" in exp:
        assert abs(r.objval + rec["objective_add"] - exp["objective_value"]) <= 1e-9 * abs(obj)
    if "x" in exp:
        np.testing.assert_allclose(r.x, exp["x"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("rec", [d for d in DENSE if d["m"] <= 500],
                         ids=[f"s{d['seed']}_{d['m']}x{d['n']}" for d in DENSE if d["m"] <= 500])
@pytest.mark.parametrize("rule", [1, 0], ids=["devex", "dantzig"])
def test_dense_vs_highs(rec, rule):
    m, n = rec["m"], rec["n"]
    A, b, c = generate_dense(rec["seed"], m, n)
    r = solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, price_rule=rule)
    assert r.status == 0
    assert abs(r.objval - rec["objective"]) <= 1e-8 * abs(rec["objective"])
    x = np.zeros(n)
    for j, v in rec["x_nonzero"].items():
        x[int(j)] = v
    np.testing.assert_allclose(r.x, x, rtol=1e-8, atol=1e-8 * np.abs(x).max())
    assert rec["nondegenerate"]
    np.testing.assert_array_equal(r.basis, rec["basis"])  # bit-exact basis indices


def test_generator_known_vectors():
    for rec in load_generator_vectors():
        seed, m, n = rec["seed"], rec["m"], rec["n"]
        for i, j, hx in rec["A"]:
            A, _, _ = generate_dense(seed, m, n, col0=j, ncols=1)
            assert A[i, 0] == float.fromhex(hx)
        _, b, c = generate_dense(seed, m, n, col0=0, ncols=0, want_A=False)
        for i, hx in rec["b"]:
            assert b[i] == float.fromhex(hx)
        for j, hx in rec["c"]:
            _, _, cj = generate_dense(seed, m, n, col0=j, ncols=1, want_A=False)
            assert cj[0] == float.fromhex(hx)


def test_iteration_cap_reports_suboptimal():
    A, b, c = generate_dense(1, 50, 200)
    r = solve_dense(A, np.ones(50, np.int32), b, c, maximize=True, max_iter=3)
    assert r.status == 1 and r.stats["iterations"] == 3


def test_refactor_period_does_not_change_optimum():
    A, b, c = generate_dense(2, 200, 800)
    r1 = solve_dense(A, np.ones(200, np.int32), b, c, maximize=True, refactor_period=7)
    r2 = solve_dense(A, np.ones(200, np.int32), b, c, maximize=True, refactor_period=1000)
    assert r1.status == r2.status == 0
    np.testing.assert_array_equal(r1.basis, r2.basis)
    assert abs(r1.objval - r2.objval) <= 1e-10 * abs(r1.objval)


def test_trace_records_pivots():
    A, b, c = generate_dense(3, 50, 200)
    r = solve_dense(A, np.ones(50, np.int32), b, c, maximize=True, trace_cap=10000)
    assert r.trace.shape == (r.stats["iterations"], 2)
    assert np.all(r.trace[:, 0] >= 0)


def test_gauss_jordan_refactor_mode_same_optimum():
    A, b, c = generate_dense(4, 200, 800)
    r0 = solve_dense(A, np.ones(200, np.int32), b, c, maximize=True, refactor_period=10)
    r1 = solve_dense(A, np.ones(200, np.int32), b, c, maximize=True, refactor_period=10,
                     refactor_mode=1)
    assert r0.stats["gj_refactors"] == 0 and r1.stats["gj_refactors"] == r1.stats["refactors"] > 0
    np.testing.assert_array_equal(r0.basis, r1.basis)
    assert abs(r0.objval - r1.objval) <= 1e-11 * abs(r0.objval)


def test_general_lps_vs_highs():
    """Random general-form LPs (phase 1, free/boxed columns, <=/>=/== rows)
    against SciPy-HiGHS (build container only)."""
    pytest.importorskip("scipy")
    from golden.make_golden import highs
    rng = np.random.default_rng(7)
    for trial in range(8):
        m, n = 20 + 5 * trial, 40 + 9 * trial
        A = rng.uniform(-1, 1, (m, n))
        x0 = rng.uniform(0, 2, n)
        dirs = rng.integers(1, 4, m).astype(np.int32)
        rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
        lo = np.where(rng.random(n) < 0.3, -3.0, 0.0)
        up = np.where(rng.random(n) < 0.5, 5.0, np.inf)
        obj = rng.uniform(-1, 1, n)
        mx = bool(trial % 2)
        r = solve_dense(A, dirs, rhs, obj, lo, up, mx)
        h = highs(A, dirs, rhs, obj, lo, up, mx)
        assert r.status == {0: 0, 2: 2, 3: 3}[h.status]
        if r.status == 0:
            hv = -h.fun if mx else h.fun
            assert abs(r.objval - hv) <= 1e-8 * max(1, abs(hv))
