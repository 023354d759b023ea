"""The basis representation of the CSC path: the explicit bump
inverse with buffers grown with k (O(m k + k^2) device memory) solves the
Netlib-scale feasible-start LP to the HiGHS optimum, its capacity growth keeps
the oracle's pivot path bit for bit, and ELP_BASIS_LU -- the r03-r04 sparse-LU
engine, measured 150x slower than the bump inverse and removed in r05
 -- is refused loudly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_kkt_feasible_20000x100000_optimum(gpu):
    """VERDICT r02 #6 at "Netlib scale": 20 000 x 100 000, 5 nonzeros per column,
    the feasible-start LP (8 160 pivots in the oracle, k = 2 000 at the end) to
    the constructed optimum and the HiGHS objective within 1e-8."""
    import easylp_amd
    from conftest import load_sparse_lu
    from easylp_amd.synth import sparse_kkt
    fx = {f["name"]: f for f in load_sparse_lu()}["kkt_feasible_20000x100000"]
    m, n = fx["m"], fx["n"]
    cp, ri, v, b, c, u, obj = sparse_kkt(fx["seed"], m, n, fx["k"], feasible_start=True)
    assert obj == fx["objective"]
    dirs, lo = np.ones(m, np.int32), np.zeros(n)
    with easylp_amd.Problem(m, n) as p:
        p.load_csc(cp, ri, v, dirs, b, c, lo, u, maximize=True)
        st = p.solve()
        g = p.solution(st)
    assert st == 0 and g.stats["basis"] == 1
    # the refactor policy (oracle refactor()): the one refactor
    # whose residual reaches 1.3e-3 takes two Newton-Schulz corrections, not a
    # k = 3 452 Gauss-Jordan rebuild
    assert g.stats["gj_refactors"] == 0 and 1e-6 < g.stats["max_inv_resid"] <= 1e-2
    assert abs(g.objval - fx["highs_objective"]) <= 1e-8 * abs(fx["highs_objective"])
    assert abs(g.objval - obj) <= 1e-8 * abs(obj)
    print("kkt feasible 20000x100000 (inverse): %d iterations, %.2f s, k %d" % (
        g.stats["iterations"], g.stats["seconds_total"], g.stats["bump_dim"]))


def test_bump_capacity_growth(gpu, monkeypatch):
    """The explicit inverse's buffers start at ELP_KCAP_INIT positions and double
    at polls while k grows: the pivot path stays the oracle's, bit for bit."""
    from oracle import generate_dense, solve_dense as orc
    import easylp_amd
    monkeypatch.setenv("ELP_KCAP_INIT", "3")
    m, n, seed = 300, 1201, 11
    A, b, c = generate_dense(seed, m, n)
    g = easylp_amd.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=200000)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=200000)
    assert g.stats["bump_dim"] > 3
    np.testing.assert_array_equal(g.trace, o.trace)
    assert g.objval == o.objval


def test_sparse_lu_basis_refused(gpu):
    import easylp_amd
    from easylp_amd._lib import ElpError
    A = np.array([[1.0, 2.0], [3.0, 1.0]])
    args = (A, np.ones(2, np.int32), np.ones(2), np.ones(2))
    for solve in (easylp_amd.solve_sparse, easylp_amd.solve_dense):
        with pytest.raises(ElpError, match="sparse-LU engine was removed"):
            solve(*args, basis=2)
