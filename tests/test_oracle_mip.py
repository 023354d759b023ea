"""CPU: the oracle's branch and bound (oracle/elp_oracle.c orc_solve_mip) on
the reference's own MIP tests (test-investments.R:44-45, test-students.R:40,
test-cyingair.R:27-28) and on random knapsacks against SciPy-HiGHS milp."""
import numpy as np
import pytest

from conftest import load_mip_known_answers

MIP = load_mip_known_answers()


@pytest.mark.parametrize("rec", MIP, ids=[r["name"] for r in MIP])
def test_reference_mips(rec):
    from oracle import solve_mip
    o = solve_mip(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                  rec["maximize"], rec["is_int"])
    exp = rec["expected"]
    assert o.status == exp["status"]
    assert abs(o.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))
    if "objective_value" in exp:  # objective_add applied outside the solver (R/class.R:596)
        assert o.objval + rec["objective_add"] == exp["objective_value"]
    if "x" in exp:
        np.testing.assert_allclose(o.x, exp["x"], atol=1e-9)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_random_knapsack_vs_highs(seed):
    from scipy.optimize import Bounds, LinearConstraint, milp
    from oracle import solve_mip
    rng = np.random.default_rng(seed)
    m, n = 3, 12
    A = rng.integers(1, 20, (m, n)).astype(float)
    b = A.sum(axis=1) * 0.4
    c = rng.integers(1, 30, n).astype(float)
    up = rng.integers(1, 4, n).astype(float)
    is_int = np.ones(n, np.int32)
    is_int[::4] = 0  # some continuous columns
    o = solve_mip(A, np.ones(m, np.int32), b, c, np.zeros(n), up, True, is_int)
    r = milp(-c, constraints=LinearConstraint(A, -np.inf, b), integrality=is_int,
             bounds=Bounds(np.zeros(n), up))
    assert o.status == 0 and r.status == 0
    assert abs(o.objval + r.fun) <= 1e-7 * max(1.0, abs(r.fun))


def test_infeasible_and_node_limit():
    from oracle import solve_mip
    # 2x = 1 with x integer: LP feasible, MIP infeasible
    o = solve_mip(np.array([[2.0]]), [3], [1.0], [1.0], [0.0], [5.0], False, [1])
    assert o.status == 2
    rec = next(r for r in MIP if r["name"] == "cyingair")
    o = solve_mip(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                  rec["maximize"], rec["is_int"], max_nodes=5)
    assert o.status == 1 and o.stats["nodes"] == 5


def test_iteration_budget_bounds_the_whole_tree():
    """ctl.max_iter caps the LP iterations of the whole branch and bound (not each
    node): the search stops when a node hits it; with an incumbent the result is
    sub-optimal (1), without one the failed node's status (1)."""
    from oracle import solve_mip
    rec = next(r for r in MIP if r["name"] == "students")
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            rec["is_int"])
    full = solve_mip(*args)
    assert full.status == 0 and full.stats["nodes"] > 1
    total = full.stats["lp_iterations"]
    # a budget inside the first node: no incumbent, the node's status
    o = solve_mip(*args, max_iter=3)
    assert o.status == 1 and o.stats["lp_iterations"] <= 3 and o.stats["nodes"] == 1
    # a budget that runs out later in the tree: never more iterations than allowed
    for cap in (total // 2, total - 1):
        o = solve_mip(*args, max_iter=cap)
        assert o.status == 1
        assert o.stats["lp_iterations"] <= cap
    # a budget above the total changes nothing
    o = solve_mip(*args, max_iter=total + 10)
    assert o.status == 0 and o.objval == full.objval and o.stats["nodes"] == full.stats["nodes"]
