"""GPU parity of both pricing rules (elp_control.pricing): Devex reference
weights (the default, lp_solve's default pricer) and Dantzig, against the
oracle with the same rule (price_rule).  The Devex weights are state carried
between pricing passes (previous reduced costs, weights, the last pivot's
d_q / w_q / leaving variable) on both sides, so identical pivot traces also
pin the weight arithmetic."""
import numpy as np
import pytest

from conftest import load_sparse_lps

pytestmark = pytest.mark.gpu

RULES = [(0, "dantzig"), (1, "devex")]


def _same(g, o):
    assert g.status == o.status
    np.testing.assert_array_equal(g.trace, o.trace)
    if g.status == 0:
        assert abs(g.objval - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
        np.testing.assert_array_equal(g.basis, o.basis)


def _general_lp(seed, m, n, boxed):
    rng = np.random.default_rng(seed)
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 2, n)
    dirs = rng.integers(1, 4, m).astype(np.int32)
    rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
    if boxed:
        lo = np.where(rng.random(n) < 0.3, -3.0, 0.0)
        up = np.full(n, 5.0)
    else:
        lo = np.where(rng.random(n) < 0.2, -np.inf, 0.0)
        up = np.where(rng.random(n) < 0.3, 5.0, np.inf)
    return A, dirs, rhs, rng.uniform(-1, 1, n), lo, up


@pytest.mark.parametrize("rule,name", RULES, ids=[r[1] for r in RULES])
def test_generated_dense(gpu, rule, name):
    from oracle import generate_dense, solve_dense as orc
    m, n = 300, 1500
    A, b, c = generate_dense(4, m, n)
    g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=100000, pricing=rule)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000, price_rule=rule)
    if rule == 1:
        assert o.stats["devex_resets"] > 0  # the framework restart is on the path
    _same(g, o)


@pytest.mark.parametrize("rule,name", RULES, ids=[r[1] for r in RULES])
def test_general_form_phase1(gpu, rule, name):
    """Both phases, bound flips (boxed columns), free columns, all row kinds."""
    from oracle import solve_dense as orc
    for trial in range(4):
        A, dirs, rhs, obj, lo, up = _general_lp(50 + trial, 40 + 9 * trial, 90 + 13 * trial,
                                                boxed=trial % 2 == 0)
        mx = bool(trial % 2)
        g = gpu.solve_dense(A, dirs, rhs, obj, lo, up, mx, trace=100000, pricing=rule)
        o = orc(A, dirs, rhs, obj, lo, up, mx, trace_cap=100000, price_rule=rule)
        _same(g, o)


@pytest.mark.parametrize("rule,name", RULES, ids=[r[1] for r in RULES])
def test_bland_fallback(gpu, rule, name):
    """degen_switch=1: every degenerate pivot switches to Bland's rule, during
    which Devex keeps updating weights over all priced columns."""
    from oracle import solve_dense as orc
    rng = np.random.default_rng(7)
    m, n = 60, 150
    # sparse integer data, 8 rows with rhs 0: degenerate vertices, bound flips
    A = np.round(rng.uniform(0, 3, (m, n))) * (rng.random((m, n)) < 0.15)
    rhs = np.full(m, 10.0)
    rhs[:8] = 0.0
    obj = rng.uniform(0, 1, n)
    dirs = np.ones(m, np.int32)
    up = np.full(n, 3.0)
    g = gpu.solve_dense(A, dirs, rhs, obj, np.zeros(n), up, True, trace=100000, pricing=rule,
                        degen_switch=1)
    o = orc(A, dirs, rhs, obj, np.zeros(n), up, True, trace_cap=100000, price_rule=rule,
            degen_switch=1)
    assert o.stats["degenerate"] > 0
    _same(g, o)


@pytest.mark.parametrize("rule,name", RULES, ids=[r[1] for r in RULES])
def test_csc_path(gpu, rule, name):
    from oracle import solve_dense as orc
    names = ("klee_minty_7", "general_s12_50x150", "packing_s3_120x400")
    recs = [r for r in load_sparse_lps() if r["name"] in names]
    assert len(recs) == len(names)
    for rec in recs:
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        g = gpu.solve_sparse(*args, trace=100000, pricing=rule, basis=1)
        o = orc(*args, trace_cap=100000, price_mode=1, price_rule=rule)
        _same(g, o)


def test_devex_fewer_iterations(gpu):
    """The point of the weights: fewer pivots than Dantzig to the same optimum."""
    from oracle import generate_dense
    m, n = 400, 2000
    A, b, c = generate_dense(2, m, n)
    d = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, pricing=0)
    v = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, pricing=1)
    assert d.status == v.status == 0
    assert abs(d.objval - v.objval) <= 1e-9 * abs(d.objval)
    assert v.stats["iterations"] < d.stats["iterations"]


def test_invalid_pricing_rejected(gpu):
    with pytest.raises(Exception):
        gpu.Problem(3, 3, pricing=7)
