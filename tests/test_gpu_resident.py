"""The resident small-LP solver (easylp_amd/csrc/elp_resident.hip, DESIGN.md
14): one wave runs the whole simplex loop of an LP whose state fits in LDS, in
one launch.  Its arithmetic is the oracle's (oracle/elp_oracle.c run_phase,
run_dual, basis_change, refactor), so every trace must be the oracle's bit for
bit -- and the multi-workgroup pipeline's, which these tests run beside it
(elp_control.resident = 2).  Covered: the reference's known answers (dense and
CSC, both simplex types, both pricing rules), the robust and small sparse
fixtures, the fuzz LPs, Klee-Minty, MIP trees with warm-started nodes, the
elp_iterate budget, the time limit, sensitivity from a resident basis, and the
whole pipeline parity suite again with the resident solver off (a child
process with ELP_RESIDENT=0: the default routes small LPs to the resident
solver, so the in-process suite tests it and the child tests the pipeline)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import (feasible, load_known_answers, load_mip_known_answers, load_robust_lps,
                      load_sparse_lps)
from fuzz_lps import fuzz_set

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KNOWN = load_known_answers()
ROBUST = load_robust_lps()
SPARSE = load_sparse_lps()
MIP = load_mip_known_answers()
FUZZ = fuzz_set(120)


def _same(g, o):
    assert g.status == o.status, (g.status, o.status)
    np.testing.assert_array_equal(g.trace, o.trace)
    if g.status in (0, 1):
        np.testing.assert_array_equal(g.basis, o.basis)
        assert abs(g.objval - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
        if len(o.x):
            np.testing.assert_allclose(g.x, o.x, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(o.x).max()))
    if g.status == 3:
        assert g.objval == o.objval
        np.testing.assert_array_equal(g.x, o.x)


def _args(rec):
    return (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])


def _pair(gpu, rec, sparse=False, gctl=None, octl=None, expect_resident=True):
    """resident (1) and pipeline (2) against the oracle; returns both"""
    from oracle import solve_dense as orc
    gctl = dict(gctl or {})
    octl = dict(octl or {})
    solve = gpu.solve_sparse if sparse else gpu.solve_dense
    if sparse:
        gctl.setdefault("basis", 1)
        octl["price_mode"] = 1
    o = orc(*_args(rec), trace_cap=200000, **octl)
    out = []
    for res in (1, 2):
        g = solve(*_args(rec), trace=200000, resident=res, **gctl)
        ran = g.stats["resident"] == 1
        if res == 2:
            assert not ran
        elif expect_resident and rec["A"].shape[0] >= 1 and not np.any(np.asarray(rec["lo"]) > np.asarray(rec["up"])):
            assert ran, "the resident solver did not run"  # (lower > upper: decided at the load)
        _same(g, o)
        out.append(g)
    return out


@pytest.mark.parametrize("simplex", [6, 5], ids=["dual_primal", "primal_primal"])
@pytest.mark.parametrize("rule", [1, 0], ids=["devex", "dantzig"])
@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answers_resident(gpu, rec, rule, simplex):
    ctl = {"pricing": rule, "simplex": simplex}
    octl = {"price_rule": rule, "simplex": simplex}
    g, _ = _pair(gpu, rec, gctl=ctl, octl=octl)
    assert g.status == rec["expected"]["status"]
    if g.status == 0:
        assert feasible(rec["A"], rec["dir"], rec["rhs"], g.x, rec["lo"], rec["up"])
    _pair(gpu, rec, sparse=True, gctl=ctl, octl=octl)


@pytest.mark.parametrize("rec", ROBUST, ids=[r["name"] for r in ROBUST])
def test_robust_resident(gpu, rec):
    g, _ = _pair(gpu, rec)
    assert g.status == 0
    assert abs(g.objval - rec["objective"]) <= 1e-9 * max(1.0, abs(rec["objective"]))
    _pair(gpu, rec, gctl={"scaling": 0, "refactor_mode": 1, "refactor_period": 7},
          octl={"scaling": 0, "refactor_mode": 1, "refactor_period": 7})


@pytest.mark.parametrize("rec", SPARSE, ids=[r["name"] for r in SPARSE])
def test_sparse_fixtures_resident(gpu, rec):
    """CSC fixtures: the small ones run resident, the larger ones fall back to
    the pipeline (their state does not fit in LDS) -- same bits either way."""
    _pair(gpu, rec, sparse=True, expect_resident=rec["m"] * rec["n"] <= 40 * 100)


def test_fuzz_resident(gpu):
    seen, ran = set(), 0
    for rec in FUZZ:
        rid = f"f{rec['seed']}_{rec['m']}x{rec['n']}"
        try:
            for sparse in (False, True):
                g, _ = _pair(gpu, rec, sparse=sparse, expect_resident=False,
                             gctl={"pricing": rec["seed"] % 2, "refactor_period": 5 + rec["seed"] % 40},
                             octl={"price_rule": rec["seed"] % 2, "refactor_period": 5 + rec["seed"] % 40})
                seen.add(g.status)
                ran += g.stats["resident"]
        except Exception as e:  # name the LP
            raise AssertionError(f"{rid}: {type(e).__name__}: {e}") from None
    assert {0, 2, 3} <= seen
    assert ran >= len(FUZZ)  # (most fuzz LPs fit; the larger ones take the pipeline)


@pytest.mark.parametrize("rule", [0, 1], ids=["dantzig", "devex"])
@pytest.mark.parametrize("path", ["dense", "csc"])
def test_klee_minty_resident(gpu, rule, path):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_sparse import klee_minty
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up, mx = klee_minty(12)
    Ad = A.toarray()
    solve = gpu.solve_sparse if path == "csc" else gpu.solve_dense
    kw = {"basis": 1} if path == "csc" else {}
    g = solve(A if path == "csc" else Ad, dirs, rhs, obj, lo, up, mx, trace=10000, pricing=rule, scaling=0,
              resident=1, **kw)
    o = orc(Ad, dirs, rhs, obj, lo, up, mx, trace_cap=10000, price_rule=rule, scaling=0,
            price_mode=1 if path == "csc" else 0)
    assert g.stats["resident"] == 1 and g.stats["resident_launches"] == 1
    _same(g, o)
    assert g.objval == 5.0 ** 12
    if rule == 0:
        assert g.stats["iterations"] == 2 ** 12 - 1
        assert g.stats["refactors"] == o.stats["refactors"]


@pytest.mark.parametrize("path", ["dense", "csc"])
@pytest.mark.parametrize("rec", MIP, ids=[r["name"] for r in MIP])
def test_reference_mips_resident(gpu, rec, path):
    """Branch and bound: every node LP (warm-started from the last node's basis,
    which the resident solver wrote back) runs resident when it fits; the tree
    is the oracle's node for node."""
    from oracle import solve_mip
    solve = gpu.solve_dense if path == "dense" else gpu.solve_sparse
    o = solve_mip(*_args(rec), rec["is_int"], price_mode=1 if path == "csc" else 0)
    for res in (1, 2):
        g = solve(*_args(rec), is_int=rec["is_int"], resident=res, **({"basis": 1} if path == "csc" else {}))
        assert g.status == o.status == rec["expected"]["status"]
        assert g.objval == o.objval
        np.testing.assert_array_equal(g.x, o.x)
        assert g.stats["mip_nodes"] == o.stats["nodes"]
        assert g.stats["mip_lp_iterations"] == o.stats["lp_iterations"]


def test_iterate_budget_resident(gpu):
    """elp_iterate stops the resident loop at the budget and resumes it from
    the written-back state: the same trace as one solve and as the oracle."""
    from easylp_amd import Problem
    from oracle import solve_dense as orc
    rec = next(r for r in KNOWN if r["name"] == "dop")
    o = orc(*_args(rec), trace_cap=10000)
    with Problem(rec["A"].shape[0], rec["A"].shape[1], resident=1) as p:
        p.set_trace(10000)
        p.load_dense(*_args(rec))
        st = 1
        for _ in range(200):
            st = p.iterate(2)
            if st != 1:
                break
        sol = p.solution(st)
        assert p.stats()["resident_launches"] >= 2
    _same(sol, o)


def test_time_limit_resident(gpu):
    """A Klee-Minty cube of 2^18 - 1 Dantzig pivots under a 5 ms time limit:
    the resident loop stops at a loop top with lp_solve's TIMEOUT (7)."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_sparse import klee_minty
    A, dirs, rhs, obj, lo, up, mx = klee_minty(18)
    g = gpu.solve_dense(A.toarray(), dirs, rhs, obj, lo, up, mx, pricing=0, scaling=0, resident=1,
                        time_limit=0.005)
    assert g.status == 7
    assert 0 < g.stats["iterations"] < 2 ** 18 - 1


@pytest.mark.parametrize("rec", [r for r in KNOWN if r["name"] in ("dop", "transport", "modified_simple", "brass")],
                         ids=lambda r: r["name"])
def test_sensitivity_after_resident(gpu, rec):
    """The sensitivity report reads the basis the resident solver wrote back
    (Minv, MinvT, AS, the lists): bit-equal to the pipeline's report, and the
    oracle's to 1e-9 (the MFMA accumulation order differs)."""
    from oracle import solve_dense as orc
    from test_gpu_sensitivity import _check
    o = orc(*_args(rec), sens=True)
    reps = []
    for res in (1, 2):
        g = gpu.solve_dense(*_args(rec), sensitivity=True, resident=res)
        assert g.stats["resident"] == (1 if res == 1 else 0)
        _check(g, o)
        reps.append(g.sens)
    for key in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
        np.testing.assert_array_equal(reps[0][key], reps[1][key])


def test_pipeline_suite_with_resident_off():
    """The parity suites again in a child process with ELP_RESIDENT=0: every
    small LP through the multi-workgroup pipeline."""
    env = dict(os.environ, ELP_RESIDENT="0")
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
           os.path.join(HERE, "test_gpu_parity.py"), os.path.join(HERE, "test_gpu_csc.py"),
           os.path.join(HERE, "test_gpu_dual.py"), os.path.join(HERE, "test_gpu_fuzz.py"),
           os.path.join(HERE, "test_gpu_mip.py"), os.path.join(HERE, "test_gpu_pricing.py"),
           os.path.join(HERE, "test_gpu_status.py"), os.path.join(HERE, "test_gpu_scaling.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=os.path.dirname(HERE))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert " passed" in r.stdout
