"""Sparse-LU engine timing on the GPU (diagnostic): solve a few sparse LPs with
a time limit and print iterations, seconds and factor sizes per LP."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def run(name, m, n, cp, ri, v, b, c, lo=None, up=None, tl=60.0, **ctl):
    import easylp_amd
    with easylp_amd.Problem(m, n, time_limit=tl, **ctl) as p:
        t0 = time.perf_counter()
        p.load_csc(cp, ri, v, np.ones(m, np.int32), b, c, lo, up, maximize=True)
        t1 = time.perf_counter()
        st = p.solve()
        t2 = time.perf_counter()
        s = p.stats()
        z = p.solution(st).objval
    it = s["iterations"]
    print("%-22s st %d obj %.12g it %6d flips %6d load %.3fs solve %.2fs -> %.0f it/s (%.1f us/it) refac %d "
          "lu_nnz %d eta %d k %d" % (name, st, z, it, s["bound_flips"], t1 - t0, t2 - t1, it / (t2 - t1),
                                     1e6 * (t2 - t1) / max(it, 1), s["refactors"], s["lu_nnz"], s["eta_nnz"],
                                     s["bump_dim"]), flush=True)


def main():
    from easylp_amd.synth import sparse_kkt, sparse_packing
    which = sys.argv[1:] or ["kkt2k", "pack1k", "kkt20k"]
    for w in which:
        if w == "pack2k":  # VERDICT r03 #8's yardstick: LU within 2x of the bump inverse
            cp, ri, v, b, c = sparse_packing(1, 2000, 10000, 5)
            run(w + "-inv", 2000, 10000, cp, ri, v, b, c, basis=1)
            run(w, 2000, 10000, cp, ri, v, b, c, basis=2, tl=120.0)
        elif w == "pack1k":
            cp, ri, v, b, c = sparse_packing(1, 1000, 10000, 5)
            run(w, 1000, 10000, cp, ri, v, b, c)
            run(w + "-inv", 1000, 10000, cp, ri, v, b, c, basis=1)
        elif w == "kkt2k":
            cp, ri, v, b, c, u, obj = sparse_kkt(1, 2000, 10000, 200)
            run(w, 2000, 10000, cp, ri, v, b, c, np.zeros(10000), u)
            run(w + "-inv", 2000, 10000, cp, ri, v, b, c, np.zeros(10000), u, basis=1)
        elif w == "kkt20k":
            cp, ri, v, b, c, u, obj = sparse_kkt(1, 20000, 100000, 2000)
            run(w, 20000, 100000, cp, ri, v, b, c, np.zeros(100000), u, tl=120.0)


if __name__ == "__main__":
    main()
