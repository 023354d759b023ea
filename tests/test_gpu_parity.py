"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden fixtures.  Integer outputs (status, basis, pivot trace) must be
identical; with the shared reduction-order contract the objective
and x are expected bit-identical too, and are asserted within 1e-12 relative
(north_star requires 1e-8)."""
import numpy as np
import pytest

from conftest import feasible, load_dense_lps, load_known_answers

pytestmark = pytest.mark.gpu

KNOWN = load_known_answers()
DENSE = load_dense_lps()


def _cmp(g, o, rel=1e-12):
    assert g.status == o.status
    if hasattr(o, "stats") and "gj_refactors" in o.stats:
        assert g.stats["gj_refactors"] == o.stats["gj_refactors"]
        assert g.stats["max_inv_resid"] == o.stats["max_inv_resid"]  # same E, bit for bit
        assert g.stats["refactors"] >= o.stats["refactors"]
    if g.status in (0, 1):
        assert abs(g.objval - o.objval) <= rel * max(1.0, abs(o.objval))
        np.testing.assert_allclose(g.x, o.x, rtol=rel, atol=rel * max(1.0, np.abs(o.x).max()))
        np.testing.assert_array_equal(g.basis, o.basis)
    if g.status == 3:
        assert g.objval == o.objval
        np.testing.assert_array_equal(g.x, o.x)


@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answers_gpu(gpu, rec):
    from oracle import solve_dense as orc
    g = gpu.solve_dense(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                        rec["maximize"], trace=100000)
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            trace_cap=100000)
    exp = rec["expected"]
    assert g.status == exp["status"], (g.status, g.stats)
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)
    if g.status == 0:
        assert feasible(rec["A"], rec["dir"], rec["rhs"], g.x, rec["lo"], rec["up"])
        if "objective" in exp:
            assert abs(g.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))
        if "objective_value" in exp:
            assert abs(g.objval + rec["objective_add"] - exp["objective_value"]) <= 1e-9 * abs(
                exp["objective_value"])
    if g.status == 3:
        assert gpu.large_to_infinity([g.objval])[0] == (np.inf if rec["maximize"] else -np.inf)


@pytest.mark.parametrize("rec", DENSE, ids=[f"s{d['seed']}_{d['m']}x{d['n']}" for d in DENSE])
def test_dense_fixtures_gpu(gpu, rec):
    from oracle import generate_dense, solve_dense as orc
    m, n = rec["m"], rec["n"]
    A, b, c = generate_dense(rec["seed"], m, n)
    g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=200000)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=200000)
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)
    assert g.stats["iterations"] == o.stats["iterations"]
    # HiGHS fixture: objective to 1e-8, basis bit-exact
    assert abs(g.objval - rec["objective"]) <= 1e-8 * abs(rec["objective"])
    np.testing.assert_array_equal(g.basis, rec["basis"])


def test_device_generator_matches_oracle(gpu):
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 300, 1200, 11
    with gpu.Problem(m, n) as p:
        p.set_trace(100000)
        p.load_generated(seed)
        st = p.solve()
        g = p.solution(st)
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)


def test_iterate_in_chunks_equals_solve(gpu):
    from oracle import generate_dense
    m, n = 200, 800
    A, b, c = generate_dense(5, m, n)
    ref = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=100000)
    with gpu.Problem(m, n, sync_every=7) as p:
        p.set_trace(100000)
        p.load_dense(A, np.ones(m, np.int32), b, c, maximize=True)
        st = 1
        steps = 0
        while st == 1:
            st = p.iterate(13)
            steps += 1
        g = p.solution(st)
    assert steps > 3
    _cmp(g, ref, rel=0.0)
    np.testing.assert_array_equal(g.trace, ref.trace)


@pytest.mark.parametrize("period,mode", [(1, 0), (5, 0), (37, 0), (5, 1), (37, 1)])
def test_refactor_period_parity(gpu, period, mode):
    """Newton-Schulz refactor (mode 0) and forced Gauss-Jordan (mode 1)."""
    from oracle import generate_dense, solve_dense as orc
    m, n = 120, 500
    A, b, c = generate_dense(9, m, n)
    g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=100000,
                        refactor_period=period, refactor_mode=mode)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000,
            refactor_period=period, refactor_mode=mode)
    assert o.stats["gj_refactors"] == (o.stats["refactors"] if mode else 0)
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)


def test_iteration_cap(gpu):
    from oracle import generate_dense
    A, b, c = generate_dense(1, 50, 200)
    g = gpu.solve_dense(A, np.ones(50, np.int32), b, c, maximize=True, max_iter=3)
    assert g.status == 1 and g.stats["iterations"] == 3


def test_mixed_general_lp_vs_oracle(gpu):
    """Random general-form LPs: free / boxed columns, <=, >=, == rows (phase 1)."""
    from oracle import solve_dense as orc
    rng = np.random.default_rng(123)
    for trial in range(6):
        m, n = 30 + 7 * trial, 60 + 11 * trial
        A = rng.uniform(-1, 1, (m, n))
        x0 = rng.uniform(0, 2, n)
        dirs = rng.integers(1, 4, m).astype(np.int32)
        rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
        if trial % 2 == 0:  # boxed: optimal after phase 1, with bound flips
            lo = np.where(rng.random(n) < 0.3, -3.0, 0.0)
            up = np.full(n, 5.0)
        else:  # free / half-open columns: exercises the unbounded exit
            lo = np.where(rng.random(n) < 0.2, -np.inf, 0.0)
            up = np.where(rng.random(n) < 0.3, 5.0, np.inf)
        obj = rng.uniform(-1, 1, n)
        g = gpu.solve_dense(A, dirs, rhs, obj, lo, up, maximize=bool(trial % 2), trace=100000)
        o = orc(A, dirs, rhs, obj, lo, up, bool(trial % 2), trace_cap=100000)
        _cmp(g, o)
        np.testing.assert_array_equal(g.trace, o.trace)


def _equality_lp(m, n, seed):
    rng = np.random.default_rng(seed)
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 4, n)
    rhs = A @ x0
    obj = rng.uniform(-1, 1, n)
    return A, np.full(m, 3, np.int32), rhs, obj, np.zeros(n), np.full(n, 5.0)


def test_large_bump_vs_oracle(gpu):
    """All-equality LP: the bump grows past 256 (two bump tiles, |Y| >= 256
    pricing chunks of 32+ rows) -- the regime of the 5000x50000 benchmark."""
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up = _equality_lp(420, 700, 3)
    g = gpu.solve_dense(A, dirs, rhs, obj, lo, up, False, trace=200000)
    o = orc(A, dirs, rhs, obj, lo, up, False, trace_cap=200000)
    assert o.stats["bump_dim"] > 256, o.stats
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)


def test_ar_growth_during_solve(gpu, monkeypatch):
    """The Y-row copy AR starts at 8 rows and is grown at polls while |Y| rises."""
    from oracle import generate_dense, solve_dense as orc
    monkeypatch.setenv("ELP_AR_INIT_ROWS", "8")
    m, n = 300, 1200
    A, b, c = generate_dense(21, m, n)
    g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=100000, sync_every=5)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    assert o.stats["y_rows"] > 16
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)


def test_bump_past_1024_vs_oracle(gpu):
    """Diagonally dominant LP whose optimal basis is all structural: the bump
    grows by one per pivot to k = 1050, past the register-resident limits of
    the latency kernels (B^-1 rows and bump FTRAN by lane-strided chains past
    512, the ratio test's row loops and two-pass A[lrow, S] gather past 1024,
    alpha_S staged in LDS for FTRAN-z)."""
    from oracle import solve_dense as orc
    m = n = 1050
    rng = np.random.default_rng(7)
    A = np.eye(m) + rng.uniform(0, 1.0 / m, (m, n))
    b = rng.uniform(1, 2, m)
    c = rng.uniform(1, 2, n)
    dirs = np.ones(m, np.int32)
    g = gpu.solve_dense(A, dirs, b, c, maximize=True, trace=100000)
    o = orc(A, dirs, b, c, maximize=True, trace_cap=100000)
    assert o.stats["bump_dim"] > 1024, o.stats
    _cmp(g, o)
    np.testing.assert_array_equal(g.trace, o.trace)
