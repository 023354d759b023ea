"""CPU: the oracle's generated-A entry point (orc_solve_generated, used for the
10 000 x 500 000 config whose A does not fit the host) walks the same pivots as
the materialised solve, and generate_rows regenerates rows of the same matrix."""
import numpy as np
import pytest


@pytest.mark.parametrize("m,n,seed", [(200, 800, 1), (300, 1200, 5), (150, 3000, 2)])
def test_generated_solve_equals_materialised(m, n, seed):
    from oracle import generate_dense, solve_dense, solve_generated
    A, b, c = generate_dense(seed, m, n)
    o = solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    g = solve_generated(seed, m, n, trace_cap=100000)
    assert o.status == g.status == 0
    np.testing.assert_array_equal(o.trace, g.trace)
    np.testing.assert_array_equal(o.basis, g.basis)
    np.testing.assert_array_equal(o.x, g.x)
    assert o.objval == g.objval


def test_generated_capped_prefix():
    from oracle import solve_generated
    full = solve_generated(3, 120, 900, trace_cap=100000)
    part = solve_generated(3, 120, 900, trace_cap=40, max_iter=40)
    assert part.status == 1 and part.stats["iterations"] == 40
    np.testing.assert_array_equal(part.trace, full.trace[:40])


def test_generate_rows():
    from oracle import generate_dense, generate_rows
    A, _, _ = generate_dense(7, 64, 300)
    rows = [0, 17, 63]
    np.testing.assert_array_equal(generate_rows(7, 64, 300, rows), A[rows])
