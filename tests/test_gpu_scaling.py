"""GPU: scaling (elp_control.scaling, default geometric + equilibrate as
lp_solve's) and the numerically hard fixtures.  The factors are powers of two
computed from integer exponents on the device (k_scale_*), so the scaled LP the
kernels see is the oracle's bit for bit: same pivots, same x and y after the
(exact) unscaling, and HiGHS's optimum on every fixture."""
import numpy as np
import pytest

from conftest import load_robust_lps

pytestmark = pytest.mark.gpu

ROBUST = load_robust_lps()


def _args(r):
    return r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"]


def _same(g, o):
    assert g.status == o.status
    np.testing.assert_array_equal(g.trace, o.trace)
    np.testing.assert_array_equal(g.basis, o.basis)
    assert g.objval == o.objval
    np.testing.assert_array_equal(g.x, o.x)
    np.testing.assert_array_equal(g.y, o.y)


@pytest.mark.parametrize("rec", ROBUST, ids=[r["name"] for r in ROBUST])
def test_robust_dense_vs_oracle_and_highs(gpu, rec):
    from oracle import solve_dense as orc
    g = gpu.solve_dense(*_args(rec), trace=100000)
    o = orc(*_args(rec), trace_cap=100000)
    _same(g, o)
    assert abs(g.objval - rec["objective"]) <= 1e-9 * max(1.0, abs(rec["objective"]))


@pytest.mark.parametrize("rec", ROBUST[::2], ids=[r["name"] for r in ROBUST[::2]])
def test_robust_csc_vs_oracle(gpu, rec):
    from oracle import solve_dense as orc
    g = gpu.solve_sparse(*_args(rec), trace=100000, basis=1)
    o = orc(*_args(rec), trace_cap=100000, price_mode=1)
    _same(g, o)


@pytest.mark.parametrize("name", ["badly_scaled_1", "badly_scaled_4", "wide_range_1"])
def test_scaled_sensitivity_vs_oracle(gpu, name):
    """Ranging runs on the scaled problem and is reported in the user's units."""
    from oracle import solve_dense as orc
    rec = next(r for r in ROBUST if r["name"] == name)
    g = gpu.solve_dense(*_args(rec), sensitivity=True)
    o = orc(*_args(rec), sens=True)
    assert g.status == o.status == 0
    for k in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
        a, b = g.sens[k], o.sens[k]
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(b[np.abs(b) < 1e29]).max(initial=1.0)),
                                   err_msg=k)


def test_scaling_modes_and_device_input(gpu):
    """geometric only, equilibrate only, both, none: each matches the oracle;
    elp_load_dense_device scales a copy (the caller's A is left as it was)."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 200, 900, 3
    A, b, c = generate_dense(seed, m, n)
    dirs = np.ones(m, np.int32)
    for mode in (0, 4, 64, 68):
        g = gpu.solve_dense(A, dirs, b, c, maximize=True, trace=100000, scaling=mode)
        o = orc(A, dirs, b, c, maximize=True, trace_cap=100000, scaling=mode)
        _same(g, o)
    dA, b2, c2 = gpu.generate_dense_device(seed, m, n, 0)
    before = dA.clone()
    with gpu.Problem(m, n) as p:
        p.set_trace(100000)
        p.load_dense_device(dA.data_ptr(), dirs, b2, c2, maximize=True)
        g = p.solution(p.solve())
    assert bool((dA == before).all())
    o = orc(A, dirs, b, c, maximize=True, trace_cap=100000)
    _same(g, o)


@pytest.mark.parametrize("ngpu", [2, 3])
def test_scaled_ngpu_vs_oracle(gpu, ngpu):
    from oracle import solve_dense as orc
    rec = next(r for r in ROBUST if r["name"] == "badly_scaled_2")
    g = gpu.solve_dense(*_args(rec), trace=100000, ngpu=ngpu)
    o = orc(*_args(rec), trace_cap=100000)
    _same(g, o)


def test_scaled_mip_vs_oracle(gpu):
    from conftest import load_mip_known_answers
    from oracle import solve_mip
    for rec in load_mip_known_answers():
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        g = gpu.solve_dense(*args, is_int=rec["is_int"])
        o = solve_mip(*args, rec["is_int"])
        assert (g.status, g.objval, g.stats["mip_nodes"]) == (o.status, o.objval, o.stats["nodes"])


def test_large_finite_bound_and_rhs_survive_scaling(gpu):
    """A finite bound / rhs that crosses 1e30 only after scaling stays finite
    (clamped once, before scaling, as the oracle does): column 1's
    coefficients are ~1e3 (its bound is scaled up ~2^10), row 1's ~1e-3 (its rhs
    too).  The re-clamp this guards against turned both infinite: unbounded."""
    from oracle import solve_dense as orc
    A = np.array([[1e3, -1e3, 0.0], [0.0, 0.0, 1e-3]])
    args = (A, np.ones(2, np.int32), np.array([5.0, 1e27]), np.array([1.0, 0.0, 1.0]),
            np.zeros(3), np.array([np.inf, 1e27, np.inf]), True)
    g = gpu.solve_dense(*args, trace=1000)
    o = orc(*args, trace_cap=1000)
    _same(g, o)
    assert g.status == 0
    assert g.x[1] == 1e27
