"""One handle, many loads (what bench.py's full-solve steps and a long R session
do): every reload starts from a clean state and solves to the same answer --
no device buffer or capacity carried over grows or leaks between loads."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_reload_same_handle_many_times(gpu):
    m, n, seed = 400, 3000, 2
    A, b, c = gpu.generate_dense_device(seed, m, n, 0)
    dirs = np.ones(m, np.int32)
    res = []
    with gpu.Problem(m, n, refactor_period=20) as p:
        for _ in range(12):
            p.load_dense_device(A.data_ptr(), dirs, b, c, maximize=True)
            st = p.solve()
            s = p.stats()
            res.append((st, p.solution(st).objval, s["iterations"], s["refactors"]))
    assert res[0][0] == 0 and res[0][3] > 2
    assert all(r == res[0] for r in res), res



@pytest.mark.parametrize("m", [30, 0])
def test_reload_reuses_buffers(gpu, m):
    """Reloads of one handle reuse A's device copy (elp_load_dense); m = 0 (no
    rows: a zero-size A) included -- each load solves to the right answer."""
    rng = np.random.default_rng(5)
    n = 40
    with gpu.Problem(m, n) as p:
        for _ in range(3):
            A = rng.uniform(0, 1, (m, n))
            c = rng.uniform(0, 1, n)
            up = np.full(n, 5.0)
            p.load_dense(A, np.ones(m, np.int32), np.full(m, 10.0), c, up=up, maximize=True)
            st = p.solve()
            sol = p.solution(st)
            assert st == 0
            if m == 0:  # every column at its upper bound
                assert abs(sol.objval - 5.0 * c.sum()) <= 1e-9 * 5.0 * c.sum()
            else:
                from oracle import solve_dense as orc
                o = orc(A, np.ones(m, np.int32), np.full(m, 10.0), c, up=up, maximize=True)
                assert sol.objval == o.objval
