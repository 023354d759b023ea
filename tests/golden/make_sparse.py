"""Generate tests/golden/sparse_lps.json: sparse LPs for the CSC path
(elp_load_csc; BASELINE config 5) with their SciPy-HiGHS optimum.

Run in the build container (needs scipy; NOT run on the GPU box):

    python tests/golden/make_sparse.py

Each record holds the problem as plain data (CSC arrays colptr / rowind / val,
dir, rhs, obj, lo, up, sense) and HiGHS's status / objective / x.  Netlib MPS
files are not in this image (no network), so the "Netlib-scale" half of the
config is represented by seeded sparse LPs of Netlib-like shapes (a few
nonzeros per column, mixed row senses, boxed and free columns) and by
Klee-Minty cubes written in sparse form (optimum 5^n, the degenerate-path case).
"""
from __future__ import annotations

import json
import os

import numpy as np
import scipy.sparse as sp
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))


def sparse_packing(seed, m, n, per_col):
    """maximize c'x, A x <= b, x >= 0; A >= 0 with per_col random rows per column
    (so x is bounded), b_i = (row sum)/4 + U[0,1)."""
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for j in range(n):
        k = max(1, min(m, rng.poisson(per_col)))
        r = rng.choice(m, size=k, replace=False)
        rows += list(r)
        cols += [j] * k
        vals += list(rng.uniform(0.05, 1.0, k))
    A = sp.csc_matrix((vals, (rows, cols)), shape=(m, n))
    b = np.asarray(A.sum(axis=1)).ravel() / 4.0 + rng.uniform(0, 1, m)
    c = rng.uniform(0, 1, n)
    return A, np.ones(m, np.int32), b, c, np.zeros(n), np.full(n, np.inf), True


def sparse_general(seed, m, n, per_col):
    """Mixed <=, >=, == rows around a known interior point, boxed / free /
    negative-lower columns, min or max of a signed objective."""
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for j in range(n):
        k = max(1, min(m, rng.poisson(per_col)))
        r = rng.choice(m, size=k, replace=False)
        rows += list(r)
        cols += [j] * k
        vals += list(rng.uniform(-1.0, 1.0, k))
    A = sp.csc_matrix((vals, (rows, cols)), shape=(m, n))
    lo = np.where(rng.random(n) < 0.25, -2.0, 0.0)
    up = np.where(rng.random(n) < 0.8, 4.0, 6.0)
    free = rng.random(n) < 0.05  # free columns with zero cost: bounded LP
    lo[free] = -np.inf
    up[free] = np.inf
    x0 = np.clip(rng.uniform(-1, 3, n), np.where(np.isfinite(lo), lo, -1), np.where(np.isfinite(up), up, 3))
    dirs = rng.integers(1, 4, m).astype(np.int32)
    ax = A @ x0
    rhs = ax + np.where(dirs == 1, rng.uniform(0.1, 1, m), np.where(dirs == 2, -rng.uniform(0.1, 1, m), 0.0))
    obj = np.where(free, 0.0, rng.uniform(-1, 1, n))
    return A, dirs, rhs, obj, lo, up, bool(seed % 2)


def klee_minty(n):
    """max sum_j 2^(n-j) x_j  s.t.  2 sum_{j<i} 2^(i-j) x_j + x_i <= 5^i, x >= 0
    (i, j = 1..n); optimum 5^n at x = (0, .., 0, 5^n)."""
    rows, cols, vals = [], [], []
    for i in range(n):
        for j in range(i):
            rows.append(i); cols.append(j); vals.append(2.0 ** (i - j + 1))
        rows.append(i); cols.append(i); vals.append(1.0)
    A = sp.csc_matrix((vals, (rows, cols)), shape=(n, n))
    rhs = np.array([5.0 ** (i + 1) for i in range(n)])
    obj = np.array([2.0 ** (n - 1 - j) for j in range(n)])
    return A, np.ones(n, np.int32), rhs, obj, np.zeros(n), np.full(n, np.inf), True


def highs(A, dirs, rhs, obj, lo, up, maximize):
    A = sp.csr_matrix(A)
    c = -obj if maximize else obj
    ub_r, ub_b, eq_r, eq_b = [], [], [], []
    for i, d in enumerate(dirs):
        row = A.getrow(i)
        if d == 1:
            ub_r.append(row); ub_b.append(rhs[i])
        elif d == 2:
            ub_r.append(-row); ub_b.append(-rhs[i])
        else:
            eq_r.append(row); eq_b.append(rhs[i])
    kw = {}
    if ub_r:
        kw["A_ub"] = sp.vstack(ub_r); kw["b_ub"] = ub_b
    if eq_r:
        kw["A_eq"] = sp.vstack(eq_r); kw["b_eq"] = eq_b
    bounds = [(None if not np.isfinite(l) else l, None if not np.isfinite(u) else u) for l, u in zip(lo, up)]
    r = linprog(c, bounds=bounds, method="highs-ds", options={"presolve": False}, **kw)
    status = {0: 0, 2: 2, 3: 3}.get(r.status, 5)
    out = {"status": status}
    if status == 0:
        out["objective"] = float(-r.fun if maximize else r.fun)
        out["x"] = [float(v) for v in r.x]
    return out


def enc(v):
    return "inf" if v == np.inf else "-inf" if v == -np.inf else float(v)


def record(name, A, dirs, rhs, obj, lo, up, maximize):
    A = sp.csc_matrix(A)
    A.sum_duplicates()
    A.sort_indices()
    return {
        "name": name, "m": A.shape[0], "n": A.shape[1],
        "colptr": [int(v) for v in A.indptr], "rowind": [int(v) for v in A.indices],
        "val": [float(v) for v in A.data], "dir": [int(v) for v in dirs],
        "rhs": [enc(v) for v in rhs], "obj": [float(v) for v in obj],
        "lo": [enc(v) for v in lo], "up": [enc(v) for v in up], "maximize": bool(maximize),
        "expected": highs(A, dirs, rhs, obj, lo, up, maximize),
    }


def main():
    recs = []
    for seed, (m, n, pc) in enumerate([(30, 80, 3), (60, 200, 4), (120, 400, 5), (200, 700, 4)], 1):
        recs.append(record(f"packing_s{seed}_{m}x{n}", *sparse_packing(seed, m, n, pc)))
    for seed, (m, n, pc) in enumerate([(25, 60, 3), (50, 150, 4), (90, 300, 4)], 11):
        recs.append(record(f"general_s{seed}_{m}x{n}", *sparse_general(seed, m, n, pc)))
    for n in (4, 7, 10):
        rec = record(f"klee_minty_{n}", *klee_minty(n))
        assert abs(rec["expected"]["objective"] - 5.0 ** n) <= 1e-9 * 5.0 ** n
        recs.append(rec)
    for r in recs:
        print(r["name"], r["expected"]["status"], r["expected"].get("objective"))
    with open(os.path.join(HERE, "sparse_lps.json"), "w") as f:
        json.dump(recs, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
