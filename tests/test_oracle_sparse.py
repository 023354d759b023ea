"""CPU: the oracle's CSC pricing order (price_mode 1, the order of the HIP CSC
path) against the HiGHS optima of tests/golden/sparse_lps.json, and the dense
known answers through the same order."""
import numpy as np
import pytest

from conftest import feasible, load_known_answers, load_sparse_lps

SPARSE = load_sparse_lps()
KNOWN = load_known_answers()


@pytest.mark.parametrize("rec", SPARSE, ids=[r["name"] for r in SPARSE])
def test_sparse_vs_highs(rec):
    from oracle import solve_dense as orc
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            price_mode=1)
    exp = rec["expected"]
    assert o.status == exp["status"]
    assert abs(o.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))
    assert feasible(rec["A"], rec["dir"], rec["rhs"], o.x, rec["lo"], rec["up"])


@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answers_column_order(rec):
    from oracle import solve_dense as orc
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            price_mode=1)
    exp = rec["expected"]
    assert o.status == exp["status"]
    if o.status == 0 and "objective" in exp:
        assert abs(o.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))


@pytest.mark.parametrize("n", [4, 7, 10])
def test_klee_minty_exponential_path(n):
    """Unscaled, Dantzig's rule walks all 2^n vertices of the Klee-Minty cube
    and Devex weights take a short path; the default scaling (geometric +
    equilibrate) breaks the construction, and every variant reaches 5^n."""
    from oracle import solve_dense as orc
    rec = next(r for r in SPARSE if r["name"] == f"klee_minty_{n}")
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], True)
    o = orc(*args, price_mode=1, price_rule=0, scaling=0)
    assert o.status == 0 and o.objval == 5.0 ** n
    assert o.stats["iterations"] == 2 ** n - 1
    v = orc(*args, price_mode=1, scaling=0)
    assert v.status == 0 and v.objval == 5.0 ** n
    assert v.stats["iterations"] <= 6 * n  # 9, 21, 51 for n = 4, 7, 10
    for rule in (0, 1):
        sc = orc(*args, price_mode=1, price_rule=rule)
        assert sc.status == 0 and abs(sc.objval - 5.0 ** n) <= 1e-12 * 5.0 ** n
