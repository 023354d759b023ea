"""GPU branch and bound (elp_set_int + elp_solve): the reference's MIP tests
through the C ABI, dense and CSC.  The LP relaxations are bit-identical to the
oracle's, so the GPU must explore the oracle's tree node for node (same node
count) and return the same incumbent."""
import numpy as np
import pytest

from conftest import load_mip_known_answers

pytestmark = pytest.mark.gpu

MIP = load_mip_known_answers()


@pytest.mark.parametrize("path", ["dense", "csc"])
@pytest.mark.parametrize("rec", MIP, ids=[r["name"] for r in MIP])
def test_reference_mips_gpu(gpu, rec, path):
    from oracle import solve_mip
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    solve = gpu.solve_dense if path == "dense" else gpu.solve_sparse
    g = solve(*args, is_int=rec["is_int"], **({"basis": 1} if path == "csc" else {}))
    o = solve_mip(*args, rec["is_int"], price_mode=1 if path == "csc" else 0)
    exp = rec["expected"]
    assert g.status == o.status == exp["status"]
    assert g.objval == o.objval
    np.testing.assert_array_equal(g.x, o.x)
    assert g.stats["mip_nodes"] == o.stats["nodes"]
    assert g.stats["mip_lp_iterations"] == o.stats["lp_iterations"]
    assert abs(g.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))
    if "x" in exp:
        np.testing.assert_allclose(g.x, exp["x"], atol=1e-9)


def test_mip_refuses_sensitivity_and_infeasible(gpu):
    """R/class.R:615-618: "not optimal" is checked first, then integer columns."""
    from easylp_amd import Problem
    from easylp_amd._lib import ElpError
    with Problem(1, 1) as p:
        p.load_dense(np.array([[2.0]]), [3], [1.0], [1.0], [0.0], [5.0])
        p.set_int([1])
        assert p.solve() == 2
        with pytest.raises(ElpError, match="not optimal"):
            p.sensitivity()
    with Problem(1, 1) as p:
        p.load_dense(np.array([[2.0]]), [1], [3.0], [1.0], [0.0], [5.0], maximize=True)
        p.set_int([1])
        assert p.solve() == 0
        assert p.solution(0).x[0] == 1.0
        with pytest.raises(ElpError, match="integer/binary"):
            p.sensitivity()


def test_mps_with_integer_markers(gpu, tmp_path):
    from easylp_amd.mps import solve_mps
    f = tmp_path / "k.mps"
    f.write_text("""NAME KNAP
OBJSENSE
    MAX
ROWS
 N obj
 L cap
COLUMNS
    MARKER 'MARKER' 'INTORG'
    a obj 10 cap 5
    b obj 13 cap 6
    c obj 7 cap 4
    MARKER 'MARKER' 'INTEND'
RHS
    rhs cap 10
BOUNDS
 UP bnd a 1
 UP bnd b 1
 UP bnd c 1
ENDATA
""")
    p, g = solve_mps(str(f))
    assert g.status == 0 and g.objval == 20.0  # b + c
    np.testing.assert_array_equal(g.x, [0, 1, 1])


@pytest.mark.parametrize("name", ["students", "cyingair", "investments"])
def test_mip_iteration_budget_matches_oracle(gpu, name):
    """max_iter bounds the whole tree on the GPU as in the oracle: same status,
    node count, LP iterations and incumbent for budgets that end the search at
    different depths."""
    from oracle import solve_mip
    rec = next(r for r in MIP if r["name"] == name)
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    total = solve_mip(*args, rec["is_int"]).stats["lp_iterations"]
    for cap in sorted({1, 3, max(1, total // 3), max(1, total // 2), max(1, total - 1), total + 5}):
        o = solve_mip(*args, rec["is_int"], max_iter=cap)
        g = gpu.solve_dense(*args, is_int=rec["is_int"], max_iter=cap)
        assert (g.status, g.stats["mip_nodes"], g.stats["mip_lp_iterations"]) == (
            o.status, o.stats["nodes"], o.stats["lp_iterations"]), cap
        assert o.stats["lp_iterations"] <= cap
        if o.status in (0, 1) and g.status in (0, 1) and o.objval != 0.0:
            assert g.objval == o.objval


def test_mip_time_limit_bounds_the_whole_tree(gpu):
    """time_limit counts from the start of the branch and bound: a tree that
    needs many nodes stops with 1 (incumbent) or 7 (none) instead of running on."""
    import time
    rng = np.random.default_rng(7)
    m, n = 30, 60
    A = rng.integers(1, 40, (m, n)).astype(float)
    b = A.sum(axis=1) * 0.37
    c = rng.integers(1, 60, n).astype(float)
    t0 = time.time()
    g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, np.zeros(n), np.full(n, 3.0), True,
                        is_int=np.ones(n, np.int32), time_limit=0.05)
    el = time.time() - t0
    assert g.status in (1, 7)
    assert el < 5.0
