"""Probe: share of phase 1 in a general-form dense LP (>=, == rows) and its per-iteration cost."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
torch.cuda.init()
import easylp_amd as gpu

def lp(m, n, seed):
    rng = np.random.default_rng(seed)
    A = rng.uniform(0, 1, (m, n))
    x0 = rng.uniform(0, 1, n) * (rng.random(n) < 0.05)
    dirs = rng.choice([1, 2, 3], m, p=[0.5, 0.3, 0.2]).astype(np.int32)
    rhs = A @ x0 + np.where(dirs == 1, 1.0, np.where(dirs == 2, -1.0, 0.0))
    return A, dirs, rhs, rng.uniform(-1, 1, n)

for (m, n) in [(1000, 10000), (2000, 20000)]:
    A, dirs, rhs, obj = lp(m, n, 1)
    with gpu.Problem(m, n) as p:
        p.load_dense(A, dirs, rhs, obj, np.zeros(n), np.full(n, 10.0), False)
        t = time.perf_counter(); st = p.solve(); el = time.perf_counter() - t
        s = p.stats()
    p1 = s["phase1_iterations"]
    with gpu.Problem(m, n) as p:
        p.load_dense(A, dirs, rhs, obj, np.zeros(n), np.full(n, 10.0), False)
        t = time.perf_counter(); p.iterate(p1); e1 = time.perf_counter() - t
    print(m, n, "status", st, "iters", s["iterations"], "phase1", p1, "solve s", round(el, 3),
          "phase1 s", round(e1, 3), "us/it p1", round(1e6 * e1 / max(p1, 1), 1),
          "us/it p2", round(1e6 * (el - e1) / max(s["iterations"] - p1, 1), 1), flush=True)
