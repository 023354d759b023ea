"""The benchmark LP at full size (BASELINE configs[2]: 5000 x 50000) on the GPU.

Size-independent checks of the GPU optimum: primal feasibility, dual
feasibility (reduced costs) and strong duality c'x = b'y -- a certificate of
optimality that needs no reference solver; then the oracle's pivot trace
(bit-identical path, ~1 min of CPU) and, when present, the HiGHS fixture
tests/golden/dense_c3.json (objective to 1e-8, basis bit-exact)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

M, N, SEED = 5000, 50000, 1


@pytest.fixture(scope="module")
def c3(gpu):
    easylp_amd = gpu
    from oracle import generate_dense
    with easylp_amd.Problem(M, N) as p:
        p.set_trace(100000)
        p.load_generated(SEED)
        st = p.solve()
        sol = p.solution(st)
    A, b, c = generate_dense(SEED, M, N)
    return sol, A, b, c


def test_c3_optimality_certificate(c3):
    sol, A, b, c = c3
    assert sol.status == 0
    x, y = sol.x, sol.y
    scale = np.abs(b).max()
    assert (x >= -1e-12).all()
    assert (A @ x <= b + 1e-9 * scale).all()                    # primal feasible
    tol_dual = 1e-9                                             # elp_control.tol_dual
    assert (y >= -tol_dual).all()                               # slack reduced costs
    assert (c - A.T @ y <= 2 * tol_dual).all()                  # structural reduced costs
    assert abs(c @ x - b @ y) <= 1e-10 * abs(c @ x)             # strong duality
    assert abs(sol.objval - c @ x) <= 1e-10 * abs(sol.objval)
    k = int((sol.basis < N).sum())
    assert k == sol.stats["bump_dim"]


def test_c3_trace_matches_oracle(c3):
    from oracle import solve_dense
    sol, A, b, c = c3
    o = solve_dense(A, np.ones(M, np.int32), b, c, maximize=True, trace_cap=100000)
    assert o.status == 0
    np.testing.assert_array_equal(sol.trace, o.trace)
    np.testing.assert_array_equal(sol.basis, o.basis)
    assert sol.objval == o.objval
    # the maintained bump inverse drifts the same way on both sides (bit-identical E)
    assert sol.stats["max_inv_resid"] == o.stats["max_inv_resid"] <= 1e-6
    assert sol.stats["gj_refactors"] == o.stats["gj_refactors"] == 0


def test_c3_vs_highs_fixture(c3):
    path = os.path.join(GOLDEN, "dense_c3.json")
    if not os.path.exists(path):
        pytest.skip("tests/golden/dense_c3.json not generated")
    rec = json.load(open(path))
    sol = c3[0]
    assert abs(sol.objval - rec["objective"]) <= 1e-8 * abs(rec["objective"])
    assert rec["nondegenerate"]
    np.testing.assert_array_equal(sol.basis, rec["basis"])
