"""Worker bodies for the multi-rank tests (spawned; module-level for pickling)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _init(rank, world, port):
    from datetime import timedelta
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # a failing rank must not leave its peers waiting for gloo's 30-minute default
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=120))
    return dist


def transport_worker(rank, world, port, q):
    """CPU: the host transport's three primitives through their C signatures."""
    import ctypes
    import numpy as np
    import torch
    dist = _init(rank, world, port)
    from easylp_amd.dist import TorchDistTransport
    t = TorchDistTransport()
    out = {}
    # all-gather of a 24-byte record (one Cand) per rank, via the C callback
    rec = (ctypes.c_uint8 * 24)(*([rank + 1] * 24))
    recv = (ctypes.c_uint8 * (24 * world))()
    out["ag_rc"] = t._allgather(ctypes.addressof(rec), ctypes.addressof(recv), 24, None)
    out["ag"] = bytes(recv)
    # f64 sum where only the "owner" rank contributes: exact copy
    owner = world - 1
    vals = np.array([0.1 * (i + 1) for i in range(7)]) if rank == owner else np.zeros(7)
    buf = (ctypes.c_double * 7)(*vals)
    out["ar_rc"] = t._allreduce(ctypes.addressof(buf), 7, 0, None)
    out["ar"] = list(buf)
    ib = (ctypes.c_int32 * 2)(rank, -rank)
    out["mx_rc"] = t._allreduce(ctypes.addressof(ib), 2, 1, None)
    out["mx"] = list(ib)
    # broadcast of doubles from each root in turn (the row-activity chain)
    chain = (ctypes.c_double * 3)(0.0, 0.0, 0.0)
    for r in range(world):
        if r == rank:
            for i in range(3):
                chain[i] = chain[i] * 2.0 + (r + 1)
        t._bcast(ctypes.addressof(chain), 3 * 8, r, None)
    out["chain"] = list(chain)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def sharded_solve_worker(rank, world, port, q, cases, replicate=0, p2p=False, ctl=None):
    """GPU: every rank solves the same LPs on one shared GPU with the host transport.
    replicate: elp_control.replicate (1 every rank holds all of A, 2 shards only);
    p2p: the per-iteration min-loc over the IPC mailbox instead of the transport;
    ctl: further elp_control fields (e.g. pricing)."""
    ctl = dict(ctl or {})
    import numpy as np
    dist = _init(rank, world, port)
    import easylp_amd
    from easylp_amd.dist import TorchDistTransport
    t = TorchDistTransport()
    results = []
    for case in cases:
        if case["kind"] == "generated":
            m, n = case["m"], case["n"]
            p = easylp_amd.Problem(m, n, replicate=replicate, **ctl)
            p.set_trace(200000)
            p.comm_init_host(t)
            if p2p:
                p.comm_enable_p2p()
            p.load_generated(case["seed"])
        else:
            A, dirs, rhs, obj, lo, up, mx = case["lp"]
            p = easylp_amd.Problem(A.shape[0], A.shape[1], replicate=replicate, **ctl)
            p.set_trace(200000)
            p.comm_init_host(t)
            if p2p:
                p.comm_enable_p2p()
            p.load_dense(A, dirs, rhs, obj, lo, up, mx)
        st = p.solve()
        sol = p.solution(st)
        res = {"status": sol.status, "objval": sol.objval, "x": sol.x,
               "basis": sol.basis, "trace": sol.trace, "stats": sol.stats}
        if case.get("sens") and st == 0:  # (a collective: every rank asks)
            res["sens"] = p.sensitivity()
        results.append(res)
        p.close()
    q.put((rank, results, t.errors))
    dist.barrier()
    dist.destroy_process_group()
