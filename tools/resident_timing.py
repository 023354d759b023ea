"""Klee-Minty / DOP / reference MIPs: wall time of load + solve through the C ABI,
resident solver on (1) and off (2), beside the CPU oracle (one core)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch
    torch.cuda.init()
    from easylp_amd import Problem
    from make_sparse import klee_minty
    from oracle import solve_dense as orc
    out = {}
    for nk in (12, 14):
        A, dirs, rhs, obj, lo, up, mx = klee_minty(nk)
        Ad = A.toarray()
        for res in (1, 2):
            ts = []
            for rep in range(3):
                with Problem(nk, nk, pricing=0, scaling=0, resident=res) as p:
                    t0 = time.perf_counter()
                    p.load_dense(Ad, dirs, rhs, obj, lo, up, mx)
                    st = p.solve()
                    ts.append(time.perf_counter() - t0)
                    s = p.stats()
            out[f"km{nk}_res{res}"] = {"s": min(ts), "iters": s["iterations"], "load_s": s["seconds_load"],
                                       "resident": s["resident"], "ticks_us": s["resident_ticks"] / 100.0}
        t0 = time.perf_counter()
        r = orc(Ad, dirs, rhs, obj, lo, up, mx, price_rule=0, scaling=0)
        out[f"km{nk}_cpu"] = {"s": time.perf_counter() - t0, "iters": r.stats["iterations"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
