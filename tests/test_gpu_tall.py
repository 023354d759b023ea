"""Tall LPs (m > 8192: more FTRAN-z row tiles than CUs) against the oracle.

At m = 10 000 (SURVEY config 4's row count) k_ftran_zr switches to 4-wave row
tiles while the bump has at most 8 chunks of ZCHUNK positions, then back to
8-wave tiles as the bump grows; the select kernel's candidate loop runs its
batched path when the tiles exceed 1024.  The pivot trace of a capped run
(refactors included) must be the oracle's, bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n,iters", [(10000, 6000, 1300), (8300, 140000, 150)])
def test_tall_trace_matches_oracle(gpu, m, n, iters):
    easylp_amd = gpu
    from oracle import generate_dense, solve_dense
    A, b, c = generate_dense(3, m, n)
    dirs = np.ones(m, np.int32)
    g = easylp_amd.solve_dense(A, dirs, b, c, maximize=True, trace=100000, max_iter=iters)
    o = solve_dense(A, dirs, b, c, maximize=True, trace_cap=100000, max_iter=iters)
    assert g.status == o.status
    assert g.stats["iterations"] == o.stats["iterations"] == iters
    np.testing.assert_array_equal(g.trace, o.trace)
    np.testing.assert_array_equal(g.basis, o.basis)
    assert g.objval == o.objval
