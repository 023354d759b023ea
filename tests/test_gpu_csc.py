"""GPU parity of the CSC path (elp_load_csc, BASELINE config 5): the HIP
kernels against the oracle in its CSC pricing order (price_mode 1, DESIGN.md
"Reduction-order contract") -- status, pivot trace and basis identical,
objective and x bit-identical (asserted within 1e-12) -- and against the HiGHS
optima of tests/golden/sparse_lps.json (1e-9)."""
import os
import sys

import numpy as np
import pytest

from conftest import feasible, load_known_answers, load_sparse_lps

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

pytestmark = pytest.mark.gpu

SPARSE = load_sparse_lps()
KNOWN = load_known_answers()


def _same(g, o):
    assert g.status == o.status
    np.testing.assert_array_equal(g.trace, o.trace)
    if g.status in (0, 1):
        np.testing.assert_array_equal(g.basis, o.basis)
        assert abs(g.objval - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
        np.testing.assert_allclose(g.x, o.x, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(o.x).max()))
    if g.status == 3:
        assert g.objval == o.objval
        np.testing.assert_array_equal(g.x, o.x)


def _gpu_csc(gpu, rec, **ctl):
    ctl.setdefault("basis", 1)  # ELP_BASIS_INVERSE: the bump inverse, oracle price_mode 1
    return gpu.solve_sparse(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                            rec["maximize"], trace=200000, **ctl)


@pytest.mark.parametrize("rec", SPARSE, ids=[r["name"] for r in SPARSE])
def test_sparse_fixtures_gpu(gpu, rec):
    from oracle import solve_dense as orc
    g = _gpu_csc(gpu, rec)
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            trace_cap=200000, price_mode=1)
    _same(g, o)
    exp = rec["expected"]
    assert g.status == exp["status"]
    assert abs(g.objval - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"]))
    assert feasible(rec["A"], rec["dir"], rec["rhs"], g.x, rec["lo"], rec["up"])


@pytest.mark.parametrize("rec", KNOWN, ids=[r["name"] for r in KNOWN])
def test_known_answers_csc(gpu, rec):
    from oracle import solve_dense as orc
    g = _gpu_csc(gpu, rec)
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            trace_cap=200000, price_mode=1)
    assert g.status == rec["expected"]["status"]
    _same(g, o)


@pytest.mark.parametrize("rule", [0, 1], ids=["dantzig", "devex"])
def test_klee_minty_12(gpu, rule):
    """Degenerate-path case (unscaled: scaling breaks the construction):
    2^12 - 1 Dantzig pivots to the optimum 5^12; Devex weights take a short
    path to it."""
    from make_sparse import klee_minty
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up, mx = klee_minty(12)
    g = gpu.solve_sparse(A, dirs, rhs, obj, lo, up, mx, trace=10000, pricing=rule, scaling=0, basis=1)
    o = orc(A.toarray(), dirs, rhs, obj, lo, up, mx, trace_cap=10000, price_mode=1, price_rule=rule,
            scaling=0)
    _same(g, o)
    assert g.objval == 5.0 ** 12
    if rule == 0:
        assert g.stats["iterations"] == 2 ** 12 - 1
    else:
        assert g.stats["iterations"] < 2 ** 12 // 8


@pytest.mark.parametrize("kind", ["packing", "general"])
def test_larger_sparse_vs_oracle(gpu, kind):
    from make_sparse import sparse_general, sparse_packing
    from oracle import solve_dense as orc
    gen = sparse_packing if kind == "packing" else sparse_general
    A, dirs, rhs, obj, lo, up, mx = gen(31, 600, 3000, 5)
    g = gpu.solve_sparse(A, dirs, rhs, obj, lo, up, mx, trace=100000, basis=1)
    o = orc(A.toarray(), dirs, rhs, obj, lo, up, mx, trace_cap=100000, price_mode=1)
    assert g.status == 0
    _same(g, o)


def test_large_bump_launch_shape(gpu, monkeypatch):
    """ELP_FORCE_SELECT: the launch shapes used for bumps beyond the LDS budget
    (single-workgroup select + bump FTRAN, global z partials, global B^-1 row
    staging), on the dense and the CSC path."""
    from oracle import solve_dense as orc
    monkeypatch.setenv("ELP_FORCE_SELECT", "1")
    rec = next(r for r in SPARSE if r["name"] == "general_s13_90x300")
    g = _gpu_csc(gpu, rec)
    o = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
            trace_cap=200000, price_mode=1)
    _same(g, o)
    gd = gpu.solve_dense(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"],
                         rec["maximize"], trace=200000)
    od = orc(rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"],
             trace_cap=200000)
    _same(gd, od)


def test_csc_usage_errors(gpu):
    from easylp_amd import Problem
    from easylp_amd._lib import ElpError
    with Problem(2, 2) as p:
        with pytest.raises(ElpError, match="strictly increasing"):
            p.load_csc([0, 2, 3], [1, 0, 1], [1.0, 2.0, 3.0], [1, 1], [1.0, 1.0], [1.0, 1.0])
        with pytest.raises(ElpError, match="out of range"):
            p.load_csc([0, 1, 2], [0, 5], [1.0, 2.0], [1, 1], [1.0, 1.0], [1.0, 1.0])


def test_mps_file_through_csc(gpu, tmp_path):
    """An MPS file (ranges, bounds, sense, objective constant) read by
    easylp_amd.mps and solved on the GPU: same pivots as the oracle."""
    from easylp_amd.mps import read_mps, solve_mps
    from easylp_amd.solver import csc_arrays
    from oracle import solve_dense as orc
    from test_mps import TEXT
    f = tmp_path / "t.mps"
    f.write_text(TEXT)
    p, g = solve_mps(str(f))  # (CSC input)
    o = orc(p.dense(), p.dirs, p.rhs, p.obj, p.lo, p.up, p.maximize, price_mode=1)
    assert g.status == o.status == 0
    assert g.objval == o.objval
    np.testing.assert_array_equal(g.basis, o.basis)
    assert read_mps(str(f)).objective_constant == 3.5


def _empty_tail_lp(seed, rows_ge):
    """An LP whose last pricing tile (columns 256..299 of 300, TILE_COLS = 128)
    holds only empty columns: that tile's extent is [nnz, nnz), so the staged
    CSC pricing must not read rind / cval at nnz (the r05q fault: an
    out-of-bounds read at s0 == nnz, elp_kernels.hip price_csc_body)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    m, n, nfull = 40, 300, 256
    rows, cols, vals = [], [], []
    for j in range(nfull):
        for i in rng.choice(m, 3, replace=False):
            rows.append(int(i))
            cols.append(j)
            vals.append(float(rng.uniform(0.5, 2.0)))
    A = sp.csc_matrix((vals, (rows, cols)), shape=(m, n))
    assert A.indptr[nfull] == A.indptr[n] == A.nnz
    dirs = np.ones(m, np.int32)
    rhs = rng.uniform(5.0, 10.0, m)
    if rows_ge:  # rows the slack basis violates: the dual phase (k_dual_price_csc)
        dirs[:rows_ge] = 2
        rhs[:rows_ge] = rng.uniform(1.0, 2.0, rows_ge)
    obj = rng.uniform(0.1, 1.0, n)
    lo = np.zeros(n)
    up = np.full(n, 4.0)  # boxed: the empty columns go to their upper bound
    return A, dirs, rhs, obj, lo, up


@pytest.mark.parametrize("rows_ge", [0, 6], ids=["primal", "dual"])
def test_empty_last_tile(gpu, rows_ge):
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up = _empty_tail_lp(5, rows_ge)
    g = gpu.solve_sparse(A, dirs, rhs, obj, lo, up, True, trace=100000, basis=1, resident=2)
    o = orc(A.toarray(), dirs, rhs, obj, lo, up, True, trace_cap=100000, price_mode=1)
    assert g.status == o.status == 0
    _same(g, o)
    assert feasible(A.toarray(), dirs, rhs, g.x, lo, up)
    assert np.all(g.x[256:] == 4.0)
