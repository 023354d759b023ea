"""Column-sharded solve on the GPU: 2 and 3 ranks (one process each, all on
the one GPU of the test box, host transport over gloo), with A replicated on
every rank or sharded, must reproduce the
single-rank pivot trace, objective, x and basis bit for bit (the reduction
order never spans shards; the min-loc order is total)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cases():
    rng = np.random.default_rng(5)
    m, n = 40, 90
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 2, n)
    dirs = rng.integers(1, 4, m).astype(np.int32)
    rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
    lo = np.where(rng.random(n) < 0.3, -3.0, 0.0)
    up = np.full(n, 5.0)
    obj = rng.uniform(-1, 1, n)
    return [
        {"kind": "generated", "m": 300, "n": 1201, "seed": 11},
        {"kind": "dense", "lp": (A, dirs, rhs, obj, lo, up, True)},
    ]


@pytest.mark.parametrize("world,replicate,p2p", [(2, 1, False), (3, 1, False), (2, 2, False),
                                                 (3, 2, False), (2, 1, True), (3, 1, True)])
def test_sharded_matches_oracle(world, replicate, p2p):
    """replicate 1: every rank holds all of A and only the min-loc record is
    exchanged; 2: column shards only, the entering column is all-reduced.
    p2p: the min-loc records travel through the IPC mailbox (the select kernel
    writes into every peer's memory and waits for theirs) -- here all ranks
    share one GPU, on the 8-GPU node the stores go over xGMI."""
    from dist_worker import sharded_solve_worker
    from oracle import generate_dense, solve_dense as orc
    cases = _cases()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=sharded_solve_worker, args=(r, world, port, q, cases, replicate, p2p))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, results, errors = q.get(timeout=240)
        assert errors == 0
        res[r] = results
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for ci, case in enumerate(cases):
        if case["kind"] == "generated":
            A, b, c = generate_dense(case["seed"], case["m"], case["n"])
            o = orc(A, np.ones(case["m"], np.int32), b, c, maximize=True, trace_cap=200000)
        else:
            A, dirs, rhs, obj, lo, up, mx = case["lp"]
            o = orc(A, dirs, rhs, obj, lo, up, mx, trace_cap=200000)
        for r in range(world):
            g = res[r][ci]
            assert g["status"] == o.status
            np.testing.assert_array_equal(g["trace"], o.trace)
            np.testing.assert_array_equal(g["basis"], o.basis)
            assert g["objval"] == o.objval
            np.testing.assert_array_equal(g["x"], o.x)
            assert g["stats"]["world_size"] == world


@pytest.mark.parametrize("world,replicate,p2p", [(2, 1, False), (3, 1, False), (2, 1, True), (2, 2, False),
                                                 (3, 2, False)])
def test_sharded_dual_matches_oracle(world, replicate, p2p):
    """SIMPLEX_DUAL_PRIMAL across processes (host transport, A replicated): the
    ranks all-gather their ratio-test candidates every dual iteration and walk
    the oracle's run_dual path bit for bit; with the mailbox on (p2p) the dual
    iterations skip it and the primal phase 2 uses it."""
    from dist_worker import sharded_solve_worker
    from fuzz_lps import fuzz_set
    from oracle import solve_dense as orc
    cases = [_cases()[1]] + [{"kind": "dense", "lp": (r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"],
                                                      r["maximize"])}
                             for r in fuzz_set(40) if len(r["obj"]) >= world][:12]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=sharded_solve_worker, args=(r, world, port, q, cases, replicate, p2p,
                                                            {"simplex": 6}))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, results, errors = q.get(timeout=240)
        assert errors == 0
        res[r] = results
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    duals = 0
    for ci, case in enumerate(cases):
        A, dirs, rhs, obj, lo, up, mx = case["lp"]
        o = orc(A, dirs, rhs, obj, lo, up, mx, trace_cap=200000, simplex=6)
        duals += o.stats["dual_iterations"] > 0
        for r in range(world):
            g = res[r][ci]
            assert g["status"] == o.status, ci
            np.testing.assert_array_equal(g["trace"], o.trace)
            assert g["stats"]["dual_iterations"] == o.stats["dual_iterations"]
            if o.status == 0:
                np.testing.assert_array_equal(g["basis"], o.basis)
                assert abs(g["objval"] - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
    assert duals >= 5, duals


@pytest.mark.parametrize("world,replicate", [(2, 1), (3, 2)])
def test_sharded_sensitivity(world, replicate):
    """elp_sensitivity after one process per rank (elp_comm_init*): a collective
    -- each rank ranges its own columns, the parts are all-gathered -- and every
    rank's report is the one-GPU report bit for bit (R/class.R:613-646 read
    after a sharded solve)."""
    import easylp_amd
    from dist_worker import sharded_solve_worker
    from oracle import generate_dense
    A, b, c = generate_dense(3, 120, 700)
    cases = [{"kind": "dense", "lp": (A, np.ones(120, np.int32), b, c, None, None, True), "sens": True},
             dict(_cases()[1], sens=True)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=sharded_solve_worker, args=(r, world, port, q, cases, replicate, False))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, results, errors = q.get(timeout=240)
        assert errors == 0
        res[r] = results
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for ci, case in enumerate(cases):
        one = easylp_amd.solve_dense(*case["lp"][:6], maximize=case["lp"][6], sensitivity=True)
        assert one.status == 0
        for r in range(world):
            g = res[r][ci]
            assert g["status"] == 0
            for key in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
                np.testing.assert_array_equal(g["sens"][key], one.sens[key], err_msg=(ci, r, key))


def test_rccl_single_rank_p2p_mailbox(monkeypatch):
    """The mailbox exchange on a 1-rank RCCL communicator: the select kernel
    writes its record into its own mailbox and waits for it."""
    monkeypatch.setenv("ELP_RCCL_SINGLE", "1")
    import easylp_amd
    from easylp_amd._lib import load
    from oracle import generate_dense, solve_dense as orc
    import ctypes
    lib = load()
    uid = ctypes.create_string_buffer(128)
    assert lib.elp_comm_unique_id(uid) == 0, lib.elp_last_error()
    m, n, seed = 250, 1000, 6
    with easylp_amd.Problem(m, n, replicate=1) as p:
        p.set_trace(100000)
        p.comm_init(uid.raw, 1, 0)
        p.comm_enable_p2p()
        p.load_generated(seed)
        st = p.solve()
        g = p.solution(st)
        # a second load on the same handle: new mailbox epoch, stale slots ignored
        p.load_generated(seed)
        g2 = p.solution(p.solve())
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    assert g.status == o.status == 0
    np.testing.assert_array_equal(g.trace, o.trace)
    assert g.objval == o.objval == g2.objval


def test_rccl_transport_single_rank(monkeypatch):
    """The RCCL transport (in-place all-gather, f64 all-reduce, broadcast) driving
    the sharded pipeline on a 1-rank communicator: bit-identical to the oracle."""
    monkeypatch.setenv("ELP_RCCL_SINGLE", "1")
    import easylp_amd
    from easylp_amd._lib import load
    from oracle import generate_dense, solve_dense as orc
    import ctypes
    lib = load()
    uid = ctypes.create_string_buffer(128)
    assert lib.elp_comm_unique_id(uid) == 0, lib.elp_last_error()
    m, n, seed = 250, 1000, 4
    with easylp_amd.Problem(m, n) as p:
        p.set_trace(100000)
        p.comm_init(uid.raw, 1, 0)
        p.load_generated(seed)
        st = p.solve()
        g = p.solution(st)
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    assert g.status == o.status == 0
    np.testing.assert_array_equal(g.trace, o.trace)
    assert g.objval == o.objval
