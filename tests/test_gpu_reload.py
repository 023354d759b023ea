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


def test_reload_pool_alternating_inputs(gpu, monkeypatch):
    """The reload pool (free_dev keeps the last load's buffers by size for the
    next alloc_all): one handle loads dense LPs of one shape, a CSC LP and dense
    again, with the bump and AR capacities forced to grow inside each solve
    (grown buffers are never pooled) -- every pivot trace is the oracle's."""
    import scipy.sparse as sp
    from oracle import generate_dense, solve_dense as orc
    monkeypatch.setenv("ELP_KCAP_INIT", "3")
    monkeypatch.setenv("ELP_AR_INIT_ROWS", "4")
    m, n = 120, 700
    dirs = np.ones(m, np.int32)
    with gpu.Problem(m, n) as p:
        p.set_trace(100000)
        for step, seed in enumerate((3, 4, 5, 6, 7)):
            A, b, c = generate_dense(seed, m, n)
            if step == 2:  # a CSC load between the dense ones
                A = A * (np.random.default_rng(seed).random((m, n)) < 0.2)
                S = sp.csc_matrix(A)
                p.load_csc(S.indptr, S.indices, S.data, dirs, b, c, maximize=True)
                o = orc(A, dirs, b, c, maximize=True, trace_cap=100000, price_mode=1)
            else:
                p.load_dense(A, dirs, b, c, maximize=True)
                o = orc(A, dirs, b, c, maximize=True, trace_cap=100000)
            g = p.solution(p.solve())
            assert g.status == o.status == 0, step
            assert g.stats["bump_dim"] > 3
            np.testing.assert_array_equal(g.trace, o.trace)
            assert g.objval == o.objval


def test_handle_spares_across_shapes(gpu):
    """Destroyed one-GPU handles leave their stream, buffers and pinned blocks
    for the next elp_create (elp_api.hip Spare; R creates one handle per
    solve): handles of alternating shapes -- resident-sized, pipeline-sized,
    dense and CSC, LP and MIP -- created and destroyed in turn, each trace and
    objective the oracle's, whatever the previous handle left behind."""
    import scipy.sparse as sp
    from oracle import solve_dense as orc, solve_mip
    rng = np.random.default_rng(11)
    shapes = [(12, 30, "dense"), (150, 600, "dense"), (12, 30, "csc"), (40, 90, "mip"), (150, 600, "dense"),
              (12, 31, "dense"), (40, 90, "mip"), (12, 30, "dense")]
    for m, n, kind in shapes:
        A = rng.uniform(-1, 1, (m, n)) * (rng.uniform(0, 1, (m, n)) < 0.4)
        A[:, 0] = 1.0
        dirs = rng.integers(1, 4, m).astype(np.int32)
        rhs = rng.uniform(1, 5, m) * np.where(dirs == 2, -1, 1)
        c = rng.uniform(-1, 1, n)
        up = np.full(n, 4.0)
        with gpu.Problem(m, n) as p:
            p.set_trace(100000)
            if kind == "csc":
                S = sp.csc_matrix(A)
                p.load_csc(S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data, dirs, rhs, c,
                           np.zeros(n), up, maximize=True)
            else:
                p.load_dense(A, dirs, rhs, c, up=up, maximize=True)
            if kind == "mip":
                isint = np.zeros(n, np.int32)
                isint[::3] = 1
                p.set_int(isint)
            st = p.solve()
            sol = p.solution(st)
            tr = p.trace() if kind != "mip" else None
        if kind == "mip":
            o = solve_mip(A, dirs, rhs, c, np.zeros(n), up, True, isint)
            assert st == o.status and (st != 0 or sol.objval == o.objval), (m, n, kind)
        else:
            o = orc(A, dirs, rhs, c, up=up, maximize=True, trace_cap=100000,
                    **({"price_mode": 1} if kind == "csc" else {}))
            assert st == o.status, (m, n, kind)
            assert np.array_equal(tr, o.trace), (m, n, kind)
            if st == 0:
                assert sol.objval == o.objval, (m, n, kind)
