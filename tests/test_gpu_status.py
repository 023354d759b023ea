"""GPU: the solver's failure exits reach the caller with lp_solve's numbering
(R/class.R:279-295): 5 "numerical failure encountered" from a refactor that
finds the basis singular (elp_control.tol_singular, the oracle's rule too) and
7 "timeout" from elp_control.time_limit (lp.control(timeout = ...), R/class.R:262)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_numerical_failure_status_matches_oracle(gpu):
    from oracle import generate_dense, solve_dense as orc
    m, n = 300, 1200
    A, b, c = generate_dense(5, m, n)
    dirs = np.ones(m, np.int32)
    ctl = dict(refactor_mode=1, refactor_period=20, tol_singular=1e300)
    g = gpu.solve_dense(A, dirs, b, c, maximize=True, trace=100, **ctl)
    o = orc(A, dirs, b, c, maximize=True, trace_cap=100, **ctl)
    assert o.status == 5 and g.status == 5
    assert g.status_text == "numerical failure encountered"
    assert g.stats["iterations"] == o.stats["iterations"] == 20
    np.testing.assert_array_equal(g.trace, o.trace)
    # the default threshold solves the same LP
    assert gpu.solve_dense(A, dirs, b, c, maximize=True, refactor_mode=1).status == 0


def test_timeout_status(gpu):
    from easylp_amd import Problem
    with Problem(2000, 20000, time_limit=0.002) as p:
        p.load_generated(3)
        st = p.solve()
        s = p.stats()
        sol = p.solution(st)
    assert st == 7 and sol.status_text == "timeout"
    assert 0 < s["iterations"] < 2000
    assert np.all(np.isfinite(sol.x)) and np.all(sol.x >= 0)
    with Problem(2000, 20000) as p:  # no limit: solved
        p.load_generated(3)
        assert p.solve() == 0
        assert p.stats()["iterations"] > s["iterations"]
