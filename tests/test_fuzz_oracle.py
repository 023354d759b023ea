"""The oracle on the seeded fuzz LPs (tests/fuzz_lps.py) against SciPy's HiGHS,
an independent solver: the same outcome (optimal / infeasible / unbounded),
the same optimum to 1e-7 relative, and a returned x that satisfies every row
and bound (R/class.R:533-540's 2e-8 criterion).  Infeasible-by-construction
LPs must come back status 2 (R/class.R:282 "unfeasible")."""
import numpy as np
import pytest

from conftest import feasible
from fuzz_lps import fuzz_mip, fuzz_set

FUZZ = fuzz_set(120)
HIGHS_STATUS = {0: 0, 2: 2, 3: 3}  # linprog status -> elp status


def _highs(rec):
    from scipy.optimize import linprog
    A, d, b = rec["A"], rec["dir"], rec["rhs"]
    sgn = -1.0 if rec["maximize"] else 1.0
    ub_rows = [(A[i], b[i]) for i in range(rec["m"]) if d[i] == 1]
    ub_rows += [(-A[i], -b[i]) for i in range(rec["m"]) if d[i] == 2]
    eq = [i for i in range(rec["m"]) if d[i] == 3]
    kw = {}
    if ub_rows:
        kw["A_ub"] = np.array([r for r, _ in ub_rows])
        kw["b_ub"] = np.array([v for _, v in ub_rows])
    if eq:
        kw["A_eq"] = A[eq]
        kw["b_eq"] = b[eq]
    bounds = [(None if not np.isfinite(lo) else lo, None if not np.isfinite(up) else up)
              for lo, up in zip(rec["lo"], rec["up"])]
    r = linprog(sgn * rec["obj"], bounds=bounds, method="highs", options={"presolve": False}, **kw)
    if r.status == 4:  # HiGHS' own numerical trouble (badly scaled rows): once more with presolve
        r = linprog(sgn * rec["obj"], bounds=bounds, method="highs", **kw)
    return r.status, (sgn * r.fun if r.status == 0 else None)


@pytest.mark.parametrize("rec", FUZZ, ids=[f"f{r['seed']}_{r['m']}x{r['n']}_{r['kind'][:3]}_s{r['style']}"
                                           for r in FUZZ])
def test_oracle_vs_highs(rec):
    from oracle import solve_dense as orc
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    hs, hobj = _highs(rec)
    assert hs in HIGHS_STATUS or hs == 4, hs
    if hs in HIGHS_STATUS:  # (4: HiGHS gave up; the construction still decides below)
        assert o.status == HIGHS_STATUS[hs], (o.status, hs)
    if rec["kind"] == "infeasible":
        assert o.status == 2
    if rec["kind"] == "feasible":
        assert o.status in (0, 3)
    if o.status == 0 and hs == 0:
        assert abs(o.objval - hobj) <= 1e-7 * max(1.0, abs(hobj)), (o.objval, hobj)
    if o.status == 0:
        assert feasible(rec["A"], rec["dir"], rec["rhs"], o.x, rec["lo"], rec["up"], tol=1e-7)


def test_fuzz_set_covers_every_outcome():
    from oracle import solve_dense as orc
    seen = set()
    for rec in FUZZ:
        o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        seen.add(o.status)
    assert {0, 2, 3} <= seen, seen
    assert {r["style"] for r in FUZZ} == {0, 1, 2, 3}
    assert any(r["m"] == 0 for r in FUZZ) and any(r["n"] == 1 for r in FUZZ)


MIPS = [fuzz_mip(s) for s in range(40)]


def _highs_milp(rec):
    from scipy.optimize import Bounds, LinearConstraint, milp
    A, d, b = rec["A"], rec["dir"], rec["rhs"]
    lo_r = np.where(d == 1, -np.inf, b)
    up_r = np.where(d == 2, np.inf, b)
    sgn = -1.0 if rec["maximize"] else 1.0
    r = milp(sgn * rec["obj"], constraints=[LinearConstraint(A, lo_r, up_r)],
             integrality=rec["is_int"], bounds=Bounds(rec["lo"], rec["up"]))
    return r.status, (sgn * r.fun if r.status == 0 else None)


@pytest.mark.parametrize("rec", MIPS, ids=[f"mip{r['seed']}_{r['m']}x{r['n']}_{r['kind'][:3]}" for r in MIPS])
def test_oracle_mip_vs_highs(rec):
    """Branch and bound over the oracle's LPs (orc_solve_mip, the rules of
    lp_solve's defaults: DESIGN.md section 11) against HiGHS' MILP optimum."""
    from oracle import solve_mip
    o = solve_mip(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
                  rec["is_int"])
    hs, hobj = _highs_milp(rec)
    if rec["kind"] == "infeasible":
        assert o.status == 2 and hs == 2, (o.status, hs)
        return
    assert hs == 0 and o.status == 0, (o.status, hs)
    assert abs(o.objval - hobj) <= 1e-7 * max(1.0, abs(hobj)), (o.objval, hobj)
    xi = o.x[rec["is_int"] == 1]
    assert np.all(np.abs(xi - np.round(xi)) <= 1e-7)
    assert feasible(rec["A"], rec["dir"], rec["rhs"], o.x, rec["lo"], rec["up"], tol=1e-7)
