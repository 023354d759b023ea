"""Find the first iteration where the GPU pivot trace leaves the oracle's."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import easylp_amd
from oracle import solve_dense as orc
from test_gpu_parity import _equality_lp

A, dirs, rhs, obj, lo, up = _equality_lp(420, 700, 3)
o = orc(A, dirs, rhs, obj, lo, up, False, trace_cap=200000)
g = easylp_amd.solve_dense(A, dirs, rhs, obj, lo, up, False, trace=200000, max_iter=o.stats["iterations"] + 50)
n = min(len(o.trace), len(g.trace))
diff = np.nonzero(np.any(o.trace[:n] != g.trace[:n], axis=1))[0]
print("oracle iters", o.stats["iterations"], "gpu iters", g.stats["iterations"], "status", o.status, g.status)
if len(diff):
    i = int(diff[0])
    print("first divergence at iteration", i, "oracle", o.trace[i-2:i+3].tolist(), "gpu", g.trace[i-2:i+3].tolist())
    for cap in (i - 1, i, i + 1):
        oc = orc(A, dirs, rhs, obj, lo, up, False, max_iter=cap)
        gc = easylp_amd.solve_dense(A, dirs, rhs, obj, lo, up, False, max_iter=cap)
        dx = np.abs(oc.x - gc.x)
        print(f"cap={cap} k={oc.stats['bump_dim']}/{gc.stats['bump_dim']} ny={oc.stats['y_rows']}/{gc.stats['y_rows']} "
              f"phase1={oc.stats['phase1_iterations']} max|dx|={dx.max():.3e} at {int(dx.argmax())} "
              f"basis_eq={np.array_equal(oc.basis, gc.basis)} dy={np.abs(oc.y-gc.y).max():.3e}")
