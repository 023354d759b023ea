"""HiGHS fixture for the full benchmark LP (5000 x 50000, seed 1): objective,
nonzero x and the sorted optimal basis.  Slow (~15-20 min, one core); run in
the build container:  python tests/golden/make_golden_c3.py"""
import json
import os
import sys
import time

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import generate_dense  # noqa: E402


def main(seed=1, m=5000, n=50000):
    A, b, c = generate_dense(seed, m, n)
    t = time.time()
    r = linprog(-c, A_ub=A, b_ub=b, bounds=(0, None), method="highs-ds", options={"presolve": False})
    secs = time.time() - t
    assert r.status == 0, r.message
    xb = np.nonzero(r.x > 1e-9)[0]
    sb = np.nonzero(r.slack > 1e-9)[0]
    basis = np.sort(np.concatenate([xb, n + sb]))
    rec = {"seed": seed, "m": m, "n": n, "objective": -r.fun,
           "x_nonzero": {str(int(j)): float(r.x[j]) for j in xb},
           "basis": [int(v) for v in basis], "nondegenerate": bool(len(basis) == m),
           "highs_iterations": int(r.nit), "highs_seconds": secs}
    with open(os.path.join(HERE, "dense_c3.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("objective", "nondegenerate", "highs_iterations", "highs_seconds")}))


if __name__ == "__main__":
    main()
