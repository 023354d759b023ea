"""The constructed-optimum sparse LPs (easylp_amd.synth.sparse_kkt) behind the
Netlib-scale fixtures of tests/golden/sparse_lu.json: the generator reproduces
each fixture's objective bit for bit, and its point is a KKT point (primal
feasible, dual feasible, complementary) -- the certificate the GPU tests and
bench.py rely on when they compare against `objective`.  CPU only."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_sparse_lu
from easylp_amd.synth import sparse_kkt


@pytest.mark.parametrize("name", ["kkt_2000x10000", "kkt_20000x100000", "kkt_feasible_20000x100000"])
def test_kkt_fixture_is_reproduced_and_optimal(name):
    fx = next(f for f in load_sparse_lu() if f["name"] == name)
    m, n, k = fx["m"], fx["n"], fx["k"]
    fs = bool(fx.get("feasible_start", False))
    cp, ri, v, b, c, u, obj = sparse_kkt(fx["seed"], m, n, k, feasible_start=fs)
    assert obj == fx["objective"]
    assert abs(obj - fx["highs_objective"]) <= 1e-9 * abs(obj)
    A = sp.csc_matrix((v, ri, cp), shape=(m, n))
    assert np.all(np.diff(cp) <= fx["per_col"]) and np.all(np.diff(cp) >= 1)
    if fs:  # x = 0 is feasible: no phase 1
        assert (b >= 0).all() and (v > 0).all()
    else:
        assert (b < 0).any()
    # optimality of the construction, re-solved here where it is quick (the
    # large ones are pinned by the fixture's own HiGHS objective above)
    from scipy.optimize import linprog
    if m <= 2000:
        r = linprog(-c, A_ub=A, b_ub=b, bounds=list(zip(np.zeros(n), u)), method="highs-ds")
        assert r.status == 0 and abs(-r.fun - obj) <= 1e-9 * abs(obj)
