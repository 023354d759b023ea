"""Single-process multi-device (elp_control.ngpu > 1, SURVEY.md 8b "Threading":
the R caller stays one process): one handle drives P rank handles from P host
threads.  On the one-GPU test box the ranks share the device and talk over the
in-process ThreadGroup; on a node with P devices the same handle builds an
RCCL communicator with ncclCommInitAll.  The column-sharded solve must walk the
oracle's pivot path bit for bit, for A replicated or sharded, and for every
load entry point."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def run_child(tmp_path, *args, hw_queues=16, timeout=600):
    """tests/ngpu_child.py in a fresh process with one hardware queue per rank
    stream (GPU_MAX_HW_QUEUES, set before HIP starts); returns its npz."""
    out = str(tmp_path / "res.npz")
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(hw_queues))
    r = subprocess.run([sys.executable, os.path.join(HERE, "ngpu_child.py"), out, *map(str, args)],
                       capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return dict(np.load(out))


def _general_lp():
    rng = np.random.default_rng(5)
    m, n = 40, 90
    A = rng.uniform(-1, 1, (m, n))
    x0 = rng.uniform(0, 2, n)
    dirs = rng.integers(1, 4, m).astype(np.int32)
    rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
    lo = np.where(rng.random(n) < 0.3, -3.0, 0.0)
    up = np.full(n, 5.0)
    obj = rng.uniform(-1, 1, n)
    return A, dirs, rhs, obj, lo, up


def _same(g, o, ngpu):
    assert g.status == o.status
    np.testing.assert_array_equal(g.trace, o.trace)
    np.testing.assert_array_equal(g.basis, o.basis)
    assert g.objval == o.objval
    np.testing.assert_array_equal(g.x, o.x)
    assert g.stats["world_size"] == ngpu


@pytest.mark.parametrize("ngpu,replicate", [(2, 1), (3, 1), (2, 2), (3, 2), (4, 0)])
def test_ngpu_generated_matches_oracle(gpu, ngpu, replicate):
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 300, 1201, 11
    with gpu.Problem(m, n, ngpu=ngpu, replicate=replicate) as p:
        p.set_trace(200000)
        p.load_generated(seed)
        g = p.solution(p.solve())
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=200000)
    assert o.status == 0
    _same(g, o, ngpu)


@pytest.mark.parametrize("ngpu", [2, 3])
def test_ngpu_general_lp_matches_oracle(gpu, ngpu):
    """free / boxed columns, >= and == rows, phase 1 -- through elp_load_dense."""
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up = _general_lp()
    g = gpu.solve_dense(A, dirs, rhs, obj, lo, up, maximize=True, trace=200000, ngpu=ngpu)
    o = orc(A, dirs, rhs, obj, lo, up, True, trace_cap=200000)
    _same(g, o, ngpu)


@pytest.mark.parametrize("replicate", [1, 2])
def test_ngpu_device_resident_input(gpu, replicate):
    """elp_load_dense_device on an ngpu handle (A in HBM of the first device;
    ranks on other devices would get a copy), solved twice on one handle; the
    default scaling is applied on the fly (the caller's A is not copied), also
    to the entering column that travels between column-only shards."""
    from oracle import solve_dense as orc
    m, n, seed = 250, 1000, 4
    A, b, c = gpu.generate_dense_device(seed, m, n, 0)
    with gpu.Problem(m, n, ngpu=2, replicate=replicate) as p:
        p.set_trace(100000)
        for _ in range(2):
            p.load_dense_device(A.data_ptr(), np.ones(m, np.int32), b, c, maximize=True)
            g = p.solution(p.solve())
    Ah = A.cpu().numpy().reshape(n, m).T
    o = orc(Ah, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    _same(g, o, 2)


def test_ngpu_mip_and_refusals(gpu):
    from easylp_amd._lib import ElpError
    from conftest import load_mip_known_answers
    from oracle import solve_mip
    rec = next(r for r in load_mip_known_answers() if r["name"] == "investments")
    args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
    g = gpu.solve_dense(*args, is_int=rec["is_int"], ngpu=2)
    o = solve_mip(*args, rec["is_int"])
    assert g.status == o.status == 0 and g.objval == o.objval
    assert g.stats["mip_nodes"] == o.stats["nodes"]
    with gpu.Problem(2, 2, ngpu=2) as p:
        with pytest.raises(ElpError, match="owns its communicator"):
            p.comm_init(bytes(128), 2, 0)
        with pytest.raises(ElpError, match="no problem loaded"):
            p.solve()  # a uniform state error: no rank waits, the handle stays usable
        with pytest.raises(ElpError, match="no problem loaded"):
            p.set_int([1, 1])  # (every rank fails alike; nothing is aborted)
        p.load_dense(np.eye(2), [1, 1], [1.0, 1.0], [1.0, 1.0], maximize=True)
        assert p.solve() == 0
        p.set_int([1, 1])
        assert p.solve() == 0
        with pytest.raises(ElpError, match="integer"):
            p.sensitivity()  # R/class.R:617-618


def _sens_equal(g, o, exact=False):
    """ngpu reports against the single-GPU / oracle reports: +-1e30 exactly,
    finite entries to 1e-9 (or bit for bit against one GPU)."""
    for key in ("objfrom", "objtill", "duals", "dualsfrom", "dualstill"):
        a, b = np.asarray(g[key]), np.asarray(o[key])
        if exact:
            np.testing.assert_array_equal(a, b, err_msg=key)
            continue
        ia, ib = np.abs(a) >= 1e30, np.abs(b) >= 1e30
        np.testing.assert_array_equal(ia, ib, err_msg=key)
        np.testing.assert_array_equal(a[ia], b[ib], err_msg=key)
        scale = max(1.0, float(np.abs(b[~ib]).max(initial=0.0)))
        np.testing.assert_allclose(a[~ia], b[~ib], rtol=1e-9, atol=1e-9 * scale, err_msg=key)


@pytest.mark.parametrize("ngpu,replicate", [(2, 1), (3, 1), (2, 2), (3, 2)])
def test_ngpu_sensitivity(gpu, ngpu, replicate):
    """get.sensitivity.obj / .rhs (R/class.R:613-646) after a
    column-sharded solve -- each rank ranges its own columns, the host merges --
    equal to the oracle's report to 1e-9 (+-1e30 exactly) and to the
    single-GPU report bit for bit; a dense generated LP and a general LP (free
    / boxed columns, >= and == rows, phase 1)."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 120, 700, 3
    A, b, c = generate_dense(seed, m, n)
    d = np.ones(m, np.int32)
    cases = [(A, d, b, c, None, None, True), _general_lp() + (True,)]
    for (A_, d_, r_, c_, lo_, up_, mx) in cases:
        o = orc(A_, d_, r_, c_, lo_, up_, mx, sens=True)
        one = gpu.solve_dense(A_, d_, r_, c_, lo_, up_, maximize=mx, sensitivity=True)
        g = gpu.solve_dense(A_, d_, r_, c_, lo_, up_, maximize=mx, sensitivity=True, ngpu=ngpu,
                            replicate=replicate)
        assert g.status == one.status == o.status == 0
        assert g.stats["world_size"] == ngpu
        np.testing.assert_array_equal(g.basis, o.basis)
        _sens_equal(g.sens, o.sens)
        _sens_equal(g.sens, one.sens, exact=True)


@pytest.mark.parametrize("replicate", [1, 2])
def test_ngpu_larger_capped_window(gpu, replicate):
    """the column-only variant (replicate = 2: the entering
    column is exchanged every iteration) beyond toy sizes -- 2000 x 20000 on two
    ranks, the first 400 pivots against the oracle's generated-A solve (scaled,
    the default), plus the state both reach at the cap."""
    from oracle import solve_generated
    m, n, seed, cap = 2000, 20000, 9, 400
    with gpu.Problem(m, n, ngpu=2, replicate=replicate, max_iter=cap) as p:
        p.set_trace(cap)
        p.load_generated(seed)
        st = p.solve()
        g = p.solution(st)
        s = p.stats()
    o = solve_generated(seed, m, n, trace_cap=cap, max_iter=cap)
    assert st == o.status == 1  # the iteration cap: sub-optimal
    assert s["iterations"] == o.stats["iterations"] == cap
    np.testing.assert_array_equal(g.trace, o.trace)
    np.testing.assert_array_equal(g.basis, o.basis)
    assert g.objval == o.objval


@pytest.mark.parametrize("ngpu", [2, 3, 8])
def test_ngpu_peer_mailbox_matches_oracle(tmp_path, ngpu):
    """the ngpu handle's per-iteration min-loc through the direct
    peer mailbox (each rank's select kernel stores its record into every peer's
    device memory and polls its own; peer access, no IPC, no collective launch),
    here with all P ranks on the test GPU (same-device peer pointers; on an
    8-GPU node the stores cross xGMI).  Bit-identical to the oracle's pivot
    path; a second load on the same handle (new sequence epoch) too."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 300, 1201, 11
    g = run_child(tmp_path, "generated", m, n, seed, ngpu, 1, 200000)
    assert int(g["exchange"]) == 1  # the mailbox, not the collective fallback
    assert int(g["world"]) == ngpu
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=200000)
    assert int(g["status"]) == o.status == 0
    np.testing.assert_array_equal(g["trace"], o.trace)
    np.testing.assert_array_equal(g["basis"], o.basis)
    assert float(g["objval"]) == o.objval == float(g["objval2"])
    np.testing.assert_array_equal(g["x"], o.x)


def test_ngpu_mailbox_in_process(gpu):
    """The same in the test process (box default of 4 hardware queues): two ranks
    use the mailbox when their probe round trip succeeds, else the in-process
    collective -- either way bit-identical; column-only A (replicate = 2) always
    takes the collective (the entering column must travel)."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 300, 1201, 11
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=200000)
    for replicate in (1, 2):
        with gpu.Problem(m, n, ngpu=2, replicate=replicate) as p:
            p.set_trace(200000)
            p.load_generated(seed)
            g = p.solution(p.solve())
        assert g.stats["exchange"] in ((1, 2) if replicate == 1 else (2,))
        _same(g, o, 2)


def test_ngpu_exchange_collective_forced(gpu):
    """elp_control.exchange = 1 keeps the collective."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 200, 900, 3
    with gpu.Problem(m, n, ngpu=2, replicate=1, exchange=1) as p:
        p.set_trace(100000)
        p.load_generated(seed)
        g = p.solution(p.solve())
    assert g.stats["exchange"] == 2
    A, b, c = generate_dense(seed, m, n)
    _same(g, orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000), 2)


def test_ngpu_host_load_once(gpu):
    """elp_load_dense on an ngpu handle: A is read from host memory once (the
    pinned staging pipeline feeds every rank's device), replicated or column-
    only; larger than the staging threshold so the chunked path runs."""
    from oracle import generate_dense, solve_dense as orc
    m, n, seed = 400, 6000, 2  # 19.2 MB of A: two 16 MB chunks
    A, b, c = generate_dense(seed, m, n)
    o = orc(A, np.ones(m, np.int32), b, c, maximize=True, trace_cap=100000)
    for ngpu, replicate in ((1, 0), (2, 1), (3, 2)):
        g = gpu.solve_dense(A, np.ones(m, np.int32), b, c, maximize=True, trace=100000, ngpu=ngpu,
                            replicate=replicate)
        assert g.stats["h2d_bytes"] == 8.0 * m * n
        assert g.stats["seconds_h2d"] > 0
        if ngpu == 1:
            assert g.status == o.status and g.objval == o.objval
            np.testing.assert_array_equal(g.trace, o.trace)
        else:
            _same(g, o, ngpu)


def _same_dual(g, o, tag):
    assert g.status == o.status, (tag, g.status, o.status)
    np.testing.assert_array_equal(g.trace, o.trace, err_msg=tag)
    assert g.stats["dual_iterations"] == o.stats["dual_iterations"], tag
    assert g.stats["bound_flips"] == o.stats["bound_flips"], tag
    if g.status in (0, 1):
        np.testing.assert_array_equal(g.basis, o.basis, err_msg=tag)
        assert abs(g.objval - o.objval) <= 1e-12 * max(1.0, abs(o.objval)), tag
        if len(o.x):
            np.testing.assert_allclose(g.x, o.x, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(o.x).max()), err_msg=tag)


@pytest.mark.parametrize("ngpu,replicate", [(2, 0), (3, 0), (4, 0), (2, 2), (3, 2), (4, 2)])
def test_ngpu_dual_matches_oracle(gpu, ngpu, replicate):
    """SIMPLEX_DUAL_PRIMAL (lp_solve's default, R/class.R:262 / :276) on the
    column-sharded ranks of one handle, A replicated: each rank prices its
    shard and packs its ratio-test candidates (the last rank also the slacks),
    the all-gather hands every rank all of them in one-GPU order, and the
    bound-flipping ratio test runs identically on every rank -- the pivot
    trace, flips and optimum are the oracle's run_dual bit for bit.  With
    column-only shards (replicate 2) the entering column is all-reduced from
    its owner and the flipped columns' sum a_F is one per-row chain continued
    shard after shard."""
    from conftest import load_known_answers, load_robust_lps
    from fuzz_lps import fuzz_set
    from oracle import solve_dense as orc
    used = 0
    recs = load_known_answers() + load_robust_lps() + fuzz_set(60)
    for rec in recs:
        if len(rec["obj"]) < ngpu:
            continue  # (every rank prices at least one column)
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        tag = rec.get("name", "f%s" % rec.get("seed"))
        g = gpu.solve_dense(*args, trace=100000, simplex=6, ngpu=ngpu, replicate=replicate)
        o = orc(*args, trace_cap=100000, simplex=6)
        _same_dual(g, o, tag)
        used += o.stats["dual_iterations"] > 0
        if o.stats["dual_iterations"] > 0:
            assert g.stats["simplex"] == 6 and g.stats["world_size"] == ngpu, tag
    assert used >= 30, used


def test_ngpu_dual_kkt_flips(gpu):
    """The Netlib-shaped KKT LP (boxed columns, bound flips every few pivots)
    on 3 column shards: flips of columns on every shard, the trace and the
    optimum the oracle's."""
    from conftest import load_sparse_lu
    from easylp_amd.synth import dense_of, sparse_kkt
    from oracle import solve_dense as orc
    k = next(f for f in load_sparse_lu() if f["name"] == "kkt_2000x10000")
    cp, ri, v, b, c, u, obj = sparse_kkt(k["seed"], 600, 3000, 60)
    m, n = 600, 3000
    A = dense_of(cp, ri, v, m, n)
    dirs, lo = np.ones(m, np.int32), np.zeros(n)
    o = orc(A, dirs, b, c, lo, u, True, trace_cap=100000, simplex=6)
    assert o.stats["bound_flips"] > 0 and o.stats["dual_iterations"] > 0
    for replicate in (1, 2):
        g = gpu.solve_dense(A, dirs, b, c, lo, u, True, trace=100000, simplex=6, ngpu=3, replicate=replicate)
        _same_dual(g, o, "kkt600x3000 replicate %d" % replicate)


@pytest.mark.parametrize("replicate", [0, 2])
def test_ngpu_warm_mip_trees_match_oracle(gpu, replicate):
    """Branch and bound on two column shards under the default SIMPLEX_DUAL_PRIMAL:
    node LPs warm-start from the last node's basis on every rank (node bounds
    by global id, lower > upper checked over all N columns everywhere), the
    dual phase repairing them with the candidates all-gathered -- the trees are
    the oracle's warm trees node for node (status, nodes, LP iterations,
    incumbent) on the fuzz MIPs and the reference's three MIP tests."""
    from conftest import load_mip_known_answers
    from fuzz_lps import fuzz_mip
    from oracle import solve_mip
    recs = [fuzz_mip(s) for s in range(20)] + load_mip_known_answers()
    for i, rec in enumerate(recs):
        if len(rec["obj"]) < 2:
            continue
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        g = gpu.solve_dense(*args, is_int=rec["is_int"], ngpu=2, replicate=replicate)
        o = solve_mip(*args, rec["is_int"])
        tag = rec.get("name", f"mip{i}")
        assert (g.status, g.stats["mip_nodes"], g.stats["mip_lp_iterations"]) == (
            o.status, o.stats["nodes"], o.stats["lp_iterations"]), tag
        if o.status == 0:
            assert g.objval == o.objval, tag
            np.testing.assert_array_equal(g.x, o.x, err_msg=tag)
