"""N > 1 host path on CPU (gloo, world size 2 and 3): the transport behind
elp_comm_init_host -- record all-gather (candidate min-loc exchange), f64 sum
with a single contributor (entering-column packet), i32 max (cross-rank
flags) and the rank-ordered broadcast chain (row activities)."""
import multiprocessing as mp
import socket

import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_torch_dist_transport(world):
    from dist_worker import transport_worker
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=transport_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect_ag = b"".join(bytes([r + 1] * 24) for r in range(world))
    chain = [0.0] * 3
    for r in range(world):
        chain = [c * 2.0 + (r + 1) for c in chain]
    for r in range(world):
        out = res[r]
        assert out["ag_rc"] == 0 and out["ag"] == expect_ag
        assert out["ar_rc"] == 0 and out["ar"] == [0.1 * (i + 1) for i in range(7)]  # exact
        assert out["mx_rc"] == 0 and out["mx"] == [world - 1, 0]
        assert out["chain"] == chain
