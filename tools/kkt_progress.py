"""Progress of the 20 000 x 100 000 sparse_kkt solve on the GPU in iteration
chunks (elp_iterate): iterations, phase-1 iterations, k, |Y|, refactors and
seconds per chunk, so a slow solve shows where its time goes.
usage: python tools/kkt_progress.py [basis] [chunk] [wall_s]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from easylp_amd import Problem  # noqa: E402
from easylp_amd.synth import sparse_kkt  # noqa: E402

basis = int(sys.argv[1]) if len(sys.argv) > 1 else 0
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
wall = float(sys.argv[3]) if len(sys.argv) > 3 else 200.0
fx = {f["name"]: f for f in json.load(open(os.path.join(ROOT, "tests", "golden", "sparse_lu.json")))}
k = fx["kkt_20000x100000"]
cp, ri, v, b, c, u, obj = sparse_kkt(k["seed"], k["m"], k["n"], k["k"])
m, n = k["m"], k["n"]
t0 = time.perf_counter()
with Problem(m, n, basis=basis) as p:
    p.load_csc(cp, ri, v, np.ones(m, np.int32), b, c, np.zeros(n), u, maximize=True)
    print("load %.3f s" % (time.perf_counter() - t0), flush=True)
    st, last = -1, time.perf_counter()
    while time.perf_counter() - t0 < wall:
        st = p.iterate(chunk)
        s = p.stats()
        now = time.perf_counter()
        print("it %6d p1 %6d k %5d ny %5d refac %4d gj %3d flips %5d  %.3f s/chunk  st %d" % (
            s["iterations"], s["phase1_iterations"], s["bump_dim"], s["y_rows"], s["refactors"],
            s["gj_refactors"], s["bound_flips"], now - last, st), flush=True)
        last = now
        if st != 1:
            break
    if st == 0:
        z = p.solution(st).objval
        print("optimal %.15g (constructed %.15g) total %.2f s" % (z, obj, time.perf_counter() - t0), flush=True)
