"""Fixtures of the Netlib-scale CSC LPs (tests/test_gpu_basis.py, test_gpu_dual.py,
bench.py's sparse config): generator specs plus the optimum each is pinned to.

  packing_2000x10000   easylp_amd.synth.sparse_packing(1, 2000, 10000, 5):
                       HiGHS dual simplex optimum (scipy.optimize.linprog,
                       method="highs-ds");
  kkt_*                easylp_amd.synth.sparse_kkt: the optimum by
                       construction (a KKT point) and the HiGHS optimum;
  kkt_feasible_*       the same with feasible_start=True (x = 0 feasible,
                       no column at its upper bound in the optimum).

Run from the repo root:  python tests/golden/make_sparse_lu.py
(SciPy's HiGHS in this container; the script is committed with its output.)"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.optimize import linprog

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from easylp_amd.synth import sparse_kkt, sparse_packing  # noqa: E402


def main():
    out = []
    m, n = 2000, 10000
    cp, ri, v, b, c = sparse_packing(1, m, n, 5)
    A = sp.csc_matrix((v, ri, cp), shape=(m, n))
    t = time.time()
    r = linprog(-c, A_ub=A, b_ub=b, bounds=(0, None), method="highs-ds")
    assert r.status == 0
    out.append({"name": "packing_2000x10000", "generator": "sparse_packing", "seed": 1, "m": m, "n": n,
                "per_col": 5, "objective": -r.fun, "highs_iterations": int(r.nit),
                "highs_seconds": round(time.time() - t, 2)})
    for (m, n, k, fs) in ((2000, 10000, 200, False), (20000, 100000, 2000, False), (20000, 100000, 2000, True)):
        cp, ri, v, b, c, u, obj = sparse_kkt(1, m, n, k, feasible_start=fs)
        A = sp.csc_matrix((v, ri, cp), shape=(m, n))
        t = time.time()
        r = linprog(-c, A_ub=A, b_ub=b, bounds=list(zip(np.zeros(n), u)), method="highs-ds")
        assert r.status == 0 and abs(-r.fun - obj) <= 1e-9 * abs(obj)
        out.append({"name": f"kkt_{'feasible_' if fs else ''}{m}x{n}", "generator": "sparse_kkt", "seed": 1,
                    "m": m, "n": n, "k": k, "feasible_start": fs,
                    "per_col": 5, "objective": obj, "highs_objective": -r.fun, "highs_iterations": int(r.nit),
                    "highs_seconds": round(time.time() - t, 2)})
    with open(os.path.join(ROOT, "tests", "golden", "sparse_lu.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
