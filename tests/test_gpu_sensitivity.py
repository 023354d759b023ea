"""GPU sensitivity report (elp_sensitivity; R/class.R:613-646): the fp64-MFMA
contractions with fused ratio tests against the oracle's sequential
restatement.  Both end on the same basis (bit-exact solve), so the reports
must agree to rounding: 1e-9 relative (north_star's 1e-8 bar), infinite
limits (+-1e30) exactly."""
import numpy as np
import pytest

from conftest import load_dense_lps, load_known_answers, load_sparse_lps

pytestmark = pytest.mark.gpu

KNOWN = [r for r in load_known_answers() if r["expected"]["status"] == 0]
SPARSE = load_sparse_lps()


def _close(g, o, key):
    a, b = np.asarray(g[key]), np.asarray(o[key])
    inf_a, inf_b = np.abs(a) >= 1e30, np.abs(b) >= 1e30
    np.testing.assert_array_equal(inf_a, inf_b, err_msg=key)
    np.testing.assert_array_equal(a[inf_a], b[inf_b], err_msg=key)
    scale = max(1.0, float(np.abs(b[~inf_b]).max(initial=0.0)))
    np.testing.assert_allclose(a[~inf_a], b[~inf_b], rtol=1e-9, atol=1e-9 * scale, err_msg=key)


def _check(g, o):
    assert g.status == o.status == 0
    np.testing.assert_array_equal(g.basis, o.basis)
    for key in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
        _close(g.sens, o.sens, key)


@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answers_sensitivity(gpu, rec):
    from oracle import solve_dense as orc
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    _check(gpu.solve_dense(*args, sensitivity=True), orc(*args, sens=True))


def test_wyndor_gpu():
    import easylp_amd
    A = np.array([[1, 0], [0, 2], [3, 2.0]])
    g = easylp_amd.solve_dense(A, [1, 1, 1], [4, 12, 18], [3, 5], maximize=True, sensitivity=True)
    np.testing.assert_allclose(g.sens["objfrom"], [0, 2], atol=1e-12)
    np.testing.assert_allclose(g.sens["objtill"], [7.5, 1e30])
    np.testing.assert_allclose(g.sens["dualsfrom"][:3], [2, 6, 12])
    np.testing.assert_allclose(g.sens["dualstill"][:3], [1e30, 18, 24])


@pytest.mark.parametrize("rec", [load_dense_lps()[i] for i in (0, 8, 11)], ids=lambda r: f"s{r['seed']}_{r['m']}x{r['n']}")
def test_dense_sensitivity(gpu, rec):
    from oracle import generate_dense, solve_dense as orc
    m, n = rec["m"], rec["n"]
    A, b, c = generate_dense(rec["seed"], m, n)
    d = np.ones(m, np.int32)
    _check(gpu.solve_dense(A, d, b, c, maximize=True, sensitivity=True),
           orc(A, d, b, c, maximize=True, sens=True))


@pytest.mark.parametrize("rec", SPARSE, ids=[r["name"] for r in SPARSE])
def test_csc_sensitivity(gpu, rec):
    from oracle import solve_dense as orc
    g = gpu.solve_sparse(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                         rec["maximize"], sensitivity=True, basis=1)
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            sens=True, price_mode=1)
    _check(g, o)


def test_bump_beyond_one_mfma_tile(gpu):
    """All-equality LP with a bump of > 64 positions: several MFMA row / column
    tiles and partial-tile edges in both contractions."""
    from oracle import solve_dense as orc
    rng = np.random.default_rng(3)
    m, n = 150, 260
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 1, n)
    rhs = A @ x0
    obj = rng.uniform(-1, 1, n)
    args = (A, np.full(m, 3, np.int32), rhs, obj, np.zeros(n), np.full(n, 5.0), False)
    o = orc(*args, sens=True)
    assert o.stats["bump_dim"] > 64
    _check(gpu.solve_dense(*args, sensitivity=True), o)


def test_not_optimal_raises(gpu):
    import easylp_amd
    from easylp_amd._lib import ElpError
    A = np.array([[1.0, -1.0]])
    with easylp_amd.Problem(1, 2) as p:
        p.load_dense(A, [1], [1.0], [1.0, 1.0], maximize=True)
        assert p.solve() == 3
        with pytest.raises(ElpError, match="not optimal"):
            p.sensitivity()
