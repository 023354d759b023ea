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
