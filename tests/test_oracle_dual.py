"""CPU: the oracle's dual simplex phase 1 (lp_solve's default SIMPLEX_DUAL_PRIMAL,
reached through R/class.R:262 lp.control and :276 solve; orc_control.simplex =
6) on every fixture whose slack basis is infeasible: the same outcome and
optimum as HiGHS (and as the primal phase 1 on artificials), a feasible x
(R/class.R:533-540's criterion), and the Netlib-shaped KKT LP solved in a
number of pivots close to HiGHS's own dual simplex (the bound-flipping ratio
test; the primal walk needs ~45x as many)."""
import json
import os

import numpy as np
import pytest

from conftest import feasible, load_known_answers, load_robust_lps
from fuzz_lps import fuzz_mip, fuzz_set

HERE = os.path.dirname(os.path.abspath(__file__))
FUZZ = fuzz_set(120)
KNOWN = load_known_answers()
ROBUST = load_robust_lps()


def _args(r):
    return r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"]


def _agree(p, d, rec):
    assert d.status == p.status, (d.status, p.status)
    if d.status == 0:
        assert abs(d.objval - p.objval) <= 1e-7 * max(1.0, abs(p.objval)), (d.objval, p.objval)
        assert feasible(rec["A"], rec["dir"], rec["rhs"], d.x, rec["lo"], rec["up"], tol=1e-7)


@pytest.mark.parametrize("price_mode", [0, 1], ids=["dense", "csc"])
@pytest.mark.parametrize("rec", FUZZ, ids=[f"f{r['seed']}_{r['m']}x{r['n']}_{r['kind'][:3]}_s{r['style']}"
                                           for r in FUZZ])
def test_dual_fuzz_matches_primal(rec, price_mode):
    from oracle import solve_dense as orc
    p = orc(*_args(rec), simplex=5, price_mode=price_mode)
    d = orc(*_args(rec), simplex=6, price_mode=price_mode)
    _agree(p, d, rec)
    if rec["kind"] == "infeasible":
        assert d.status == 2


@pytest.mark.parametrize("rule", [1, 0], ids=["devex", "dantzig"])
@pytest.mark.parametrize("rec", KNOWN + ROBUST, ids=[r["name"] for r in KNOWN + ROBUST])
def test_dual_known_and_robust(rec, rule):
    from oracle import solve_dense as orc
    d = orc(*_args(rec), simplex=6, price_rule=rule)
    exp = rec.get("expected", {"status": 0, "objective": rec.get("objective")})
    assert d.status == exp["status"]
    if d.status == 0:
        assert abs(d.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))


def test_dual_runs_where_the_slack_basis_is_infeasible():
    """The dual phase runs exactly when the slack basis is infeasible; a
    feasible start walks the primal path unchanged (same trace as simplex 5)."""
    from oracle import generate_dense, solve_dense as orc
    used = 0
    for rec in FUZZ:
        d = orc(*_args(rec), simplex=6)
        used += d.stats["dual_iterations"] > 0
    assert used >= 60
    A, b, c = generate_dense(3, 60, 200)
    one = np.ones(60, np.int32)
    p = orc(A, one, b, c, maximize=True, simplex=5, trace_cap=10000)
    d = orc(A, one, b, c, maximize=True, simplex=6, trace_cap=10000)
    assert d.stats["dual_iterations"] == 0
    np.testing.assert_array_equal(p.trace, d.trace)


def test_dual_kkt_2000x10000_near_highs():
    """tests/golden/sparse_lu.json kkt_2000x10000 (phase-1 start, one column in
    ten at its upper bound in the optimum): the HiGHS-pinned optimum in a pivot
    count within 1.5x of HiGHS's dual simplex -- bound flips carry the columns
    that end at u (the primal path needs 20 616 pivots)."""
    from easylp_amd.synth import dense_of, sparse_kkt
    from oracle import solve_dense as orc
    fx = {f["name"]: f for f in json.load(open(os.path.join(HERE, "golden", "sparse_lu.json")))}
    k = fx["kkt_2000x10000"]
    cp, ri, v, b, c, u, obj = sparse_kkt(k["seed"], k["m"], k["n"], k["k"])
    A = dense_of(cp, ri, v, k["m"], k["n"])
    d = orc(A, np.ones(k["m"], np.int32), b, c, np.zeros(k["n"]), u, True, simplex=6, price_mode=1)
    assert d.status == 0
    assert abs(d.objval - k["highs_objective"]) <= 1e-9 * abs(k["highs_objective"])
    assert d.stats["dual_iterations"] > 0 and d.stats["bound_flips"] > 0
    assert d.stats["iterations"] <= 1.5 * k["highs_iterations"]


MIPS = [fuzz_mip(s) for s in range(40)]


def test_warm_mip_vs_highs_and_cold():
    """under SIMPLEX_DUAL_PRIMAL every branch-and-bound node LP
    after the first continues from the basis of the node solved last (warm_core:
    the dual simplex repairs the changed bounds).  Same MIP optimum as the cold
    primal tree and as HiGHS's MILP, on the 40 fuzz MIPs and the reference's
    three MIP tests, with far fewer LP iterations over the trees."""
    from conftest import load_mip_known_answers
    from oracle import solve_mip
    from test_fuzz_oracle import _highs_milp
    cold = warm = 0
    recs = MIPS + load_mip_known_answers()
    for rec in recs:
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        a = solve_mip(*args, rec["is_int"], simplex=5)
        b = solve_mip(*args, rec["is_int"], simplex=6)
        assert a.status == b.status, (a.status, b.status)
        if b.status == 0:
            assert abs(a.objval - b.objval) <= 1e-7 * max(1.0, abs(a.objval))
            assert feasible(rec["A"], rec["dir"], rec["rhs"], b.x, rec["lo"], rec["up"], tol=1e-7)
        if "kind" in rec:
            hs, hobj = _highs_milp(rec)
            if hs == 0:
                assert b.status == 0 and abs(b.objval - hobj) <= 1e-7 * max(1.0, abs(hobj))
        cold += a.stats["lp_iterations"]
        warm += b.stats["lp_iterations"]
    assert warm < 0.5 * cold, (warm, cold)
