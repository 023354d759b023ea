"""Host-path timing of the reference-sized models (diagnostic): the DOP LP
(tests/testthat/test-DOP.R:27-54) and the investments MIP (test-investments.R)
solved `reps` times through the C ABI from host memory, load / solve split,
best and median.  Run under `rocprofv3 --runtime-trace --stats` for the HIP
API calls each solve makes; ELP_DEBUG_LOAD=1 prints the load's phases."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    from conftest import load_known_answers, load_mip_known_answers
    from easylp_amd import Problem
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dop = next(r for r in load_known_answers() if r["name"] == "dop")
    inv = next(r for r in load_mip_known_answers() if r["name"] == "investments")
    only = sys.argv[2] if len(sys.argv) > 2 else None  # (one model: dop / investments)
    for name, rec, is_int in (("dop", dop, None), ("investments", inv, inv["is_int"])):
        if only and name != only:
            continue
        m, n = rec["A"].shape
        args = (rec["A"], rec["dir"], rec["rhs"], rec["obj"], rec["lo"], rec["up"], rec["maximize"])
        tl, ts, tt, th = [], [], [], []
        for _ in range(reps):
            t_h = time.perf_counter()
            with Problem(m, n) as p:
                t0 = time.perf_counter()
                p.load_dense(*args)
                if is_int is not None:
                    p.set_int(is_int)
                t1 = time.perf_counter()
                st = p.solve()
                t2 = time.perf_counter()
                s = p.stats()
            th.append(time.perf_counter() - t_h)
            tl.append(t1 - t0)
            ts.append(t2 - t1)
            tt.append(t2 - t0)
        print("%-12s st %d it %d nodes %d resident %d | load %.1f us  solve %.1f us  total %.1f us (best; median %.1f)"
              "  with create/destroy %.1f us" % (name, st, s["iterations"], s["mip_nodes"], s["resident"], 1e6 * min(tl),
                                                 1e6 * min(ts), 1e6 * min(tt), 1e6 * float(np.median(tt)),
                                                 1e6 * min(th)), flush=True)


if __name__ == "__main__":
    main()
