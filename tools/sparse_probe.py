"""Netlib-scale sparse LPs on the GPU (diagnostic): the
20 000 x 100 000 sparse_kkt LPs of tests/golden/sparse_lu.json -- the
feasible-start one and the phase-1 one (dual simplex phase 1) -- solved to
optimality with the default basis (the bump inverse), timed, against the HiGHS
objective.  ELP_LIB_PATH picks a library variant (A/B); ELP_PROBE_VERBOSE sets
elp_control.verbose (diagnostic builds: 2 = the pricing stamps, for
ELP_PDBG_FILE / ELP_PDBG_ITER timelines)."""
import json
import os
import sys
import time

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)


def main():
    from easylp_amd import Problem
    from easylp_amd.synth import sparse_kkt
    fx = {f["name"]: f for f in json.load(open(os.path.join(ROOT, "tests", "golden", "sparse_lu.json")))}
    for name in sys.argv[1:] or ["kkt_feasible_20000x100000", "kkt_20000x100000"]:
        k = fx[name]
        cp, ri, v, b, c, u, obj = sparse_kkt(k["seed"], k["m"], k["n"], k["k"], feasible_start=k["feasible_start"])
        m, n = k["m"], k["n"]
        with Problem(m, n, verbose=int(os.environ.get("ELP_PROBE_VERBOSE", "0"))) as p:
            t0 = time.perf_counter()
            p.load_csc(cp, ri, v, np.ones(m, np.int32), b, c, np.zeros(n), u, maximize=True)
            st = p.solve()
            tt = time.perf_counter() - t0
            s = p.stats()
            z = p.solution(st).objval
        print("%-26s st %d it %6d (dual %5d) flips %5d k %5d  %.3f s  %.0f it/s  rel.err vs HiGHS %.1e" % (
            name, st, s["iterations"], s["dual_iterations"], s["bound_flips"], s["bump_dim"], tt,
            s["iterations"] / tt, abs(z - k["highs_objective"]) / abs(k["highs_objective"])), flush=True)


if __name__ == "__main__":
    main()
