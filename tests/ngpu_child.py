"""Child process of the ngpu peer-mailbox tests (tests/test_gpu_ngpu.py,
tests/test_gpu_c4.py): P rank handles of one process sharing the test GPU need
a hardware queue per rank stream for the mailbox (spinning select kernels
queued behind each other never meet), so the parent starts this with
GPU_MAX_HW_QUEUES raised (<= 16) before HIP starts.  Writes the solution to
OUT (npz) for the parent to compare with the oracle.

    python tests/ngpu_child.py OUT generated M N SEED NGPU REPLICATE TRACE [SCALING]
    python tests/ngpu_child.py OUT resident  M N SEED NGPU REPLICATE TRACE [SCALING]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, kind = sys.argv[1], sys.argv[2]
    m, n, seed, ngpu, replicate, cap = (int(v) for v in sys.argv[3:9])
    scaling = int(sys.argv[9]) if len(sys.argv) > 9 else None
    import easylp_amd
    ctl = {"ngpu": ngpu, "replicate": replicate}
    if scaling is not None:
        ctl["scaling"] = scaling
    res = {}
    with easylp_amd.Problem(m, n, **ctl) as p:
        if cap:
            p.set_trace(cap)
        if kind == "generated":
            p.load_generated(seed)
            st = p.solve()
            g = p.solution(st)
            p.load_generated(seed)  # a second load: new mailbox epoch, stale slots ignored
            g2 = p.solution(p.solve())
            res["objval2"] = g2.objval
        else:  # A resident on the (shared) device: every rank reads the same copy
            A, b, c = easylp_amd.generate_dense_device(seed, m, n, 0)
            p.load_dense_device(A.data_ptr(), np.ones(m, np.int32), b, c, maximize=True)
            st = p.solve()
            g = p.solution(st)
        s = p.stats()
    np.savez(out, status=st, objval=g.objval, x=g.x, basis=g.basis,
             trace=g.trace if g.trace is not None else np.zeros((0, 2), np.int64),
             iterations=s["iterations"], exchange=s["exchange"], world=s["world_size"],
             objval2=res.get("objval2", np.nan))
    print("ok", st, s["iterations"], s["exchange"], flush=True)


if __name__ == "__main__":
    main()
