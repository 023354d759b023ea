"""Generate tests/golden/robust_lps.json: numerically hard general LPs with the
SciPy-HiGHS optimum (run in the build container; NOT on the GPU box):

    python tests/golden/make_robust.py

Kinds (VERDICT r01 "numerical robustness"):
  badly_scaled   random rows / columns multiplied by factors spanning 1e-4 .. 1e4,
                 mixed <=, >=, == rows around a feasible point, boxed columns
  near_dependent pairs of rows that agree to 1e-7 relative (rhs consistent)
  transport      degenerate transportation LP (integral supplies and demands
                 that balance exactly: every basis is degenerate)
  assignment     n x n assignment LP (equality rows and columns)
  wide_range     costs and rhs spanning 1e-3 .. 1e5 on a well-conditioned A
Stored as plain arrays (A row-major); HiGHS dual simplex, presolve off,
gives the reference objective (lp_solve is absent: its paths are unpinned).
"""
from __future__ import annotations

import json
import os

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))


def _enc(v):
    return "inf" if v == np.inf else "-inf" if v == -np.inf else float(v)


def highs(A, dirs, rhs, obj, lo, up, maximize):
    c = -obj if maximize else obj
    ub = [(A[i], rhs[i]) if d == 1 else (-A[i], -rhs[i]) for i, d in enumerate(dirs) if d != 3]
    eq = [(A[i], rhs[i]) for i, d in enumerate(dirs) if d == 3]
    kw = {}
    if ub:
        kw.update(A_ub=np.array([u[0] for u in ub]), b_ub=np.array([u[1] for u in ub]))
    if eq:
        kw.update(A_eq=np.array([e[0] for e in eq]), b_eq=np.array([e[1] for e in eq]))
    bounds = [(None if not np.isfinite(l) else l, None if not np.isfinite(u) else u) for l, u in zip(lo, up)]
    r = linprog(c, bounds=bounds, method="highs-ds", options={"presolve": False}, **kw)
    return r.status, (-r.fun if maximize else r.fun) if r.status == 0 else None


def badly_scaled(seed, m=20, n=40, span=4.0):
    rng = np.random.default_rng(seed)
    A = rng.uniform(-1, 1, (m, n)) * (rng.random((m, n)) < 0.6)
    A *= 10.0 ** rng.uniform(-span, span, (m, 1))
    A *= 10.0 ** rng.uniform(-span, span, (1, n))
    x0 = rng.uniform(0, 1, n) * 10.0 ** rng.uniform(-2, 2, n)
    dirs = rng.integers(1, 4, m).astype(np.int32)
    act = A @ x0
    slack = np.abs(A).sum(axis=1) * 0.05 * x0.mean()
    rhs = np.where(dirs == 1, act + slack, np.where(dirs == 2, act - slack, act))
    lo = np.zeros(n)
    up = x0 * rng.uniform(1.5, 4.0, n)
    obj = rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-span, span, n)
    return A, dirs, rhs, obj, lo, up, bool(seed % 2)


def near_dependent(seed, m=16, n=30):
    rng = np.random.default_rng(seed)
    B = rng.uniform(0, 1, (m // 2, n))
    A = np.vstack([B, B * (1.0 + 1e-7 * rng.uniform(-1, 1, (m // 2, n)))])
    x0 = rng.uniform(0, 1, n)
    rhs = A @ x0 + 0.5
    dirs = np.ones(m, np.int32)
    obj = rng.uniform(0, 1, n)
    return A, dirs, rhs, obj, np.zeros(n), np.full(n, np.inf), True


def transport(seed, s=5, t=6):
    rng = np.random.default_rng(seed)
    supply = rng.integers(5, 20, s).astype(float)
    demand = np.zeros(t)
    left = supply.sum()
    for j in range(t - 1):
        demand[j] = float(rng.integers(1, max(2, int(left / (t - j)) + 1)))
        left -= demand[j]
    demand[t - 1] = left
    cost = rng.integers(1, 10, (s, t)).astype(float)
    n = s * t
    A = np.zeros((s + t, n))
    for i in range(s):
        A[i, i * t:(i + 1) * t] = 1.0
    for j in range(t):
        A[s + j, j::t] = 1.0
    dirs = np.array([1] * s + [3] * t, np.int32)
    rhs = np.concatenate([supply, demand])
    return A, dirs, rhs, cost.ravel(), np.zeros(n), np.full(n, np.inf), False


def assignment(seed, k=7):
    rng = np.random.default_rng(seed)
    cost = rng.integers(1, 20, (k, k)).astype(float)
    n = k * k
    A = np.zeros((2 * k, n))
    for i in range(k):
        A[i, i * k:(i + 1) * k] = 1.0
        A[k + i, i::k] = 1.0
    return A, np.full(2 * k, 3, np.int32), np.ones(2 * k), cost.ravel(), np.zeros(n), np.ones(n), False


def wide_range(seed, m=18, n=36):
    rng = np.random.default_rng(seed)
    A = rng.uniform(0.5, 2.0, (m, n)) * (rng.random((m, n)) < 0.5)
    A[np.arange(m), rng.integers(0, n, m)] += 1.0
    rhs = 10.0 ** rng.uniform(-3, 5, m)
    obj = 10.0 ** rng.uniform(-3, 5, n)
    return A, np.ones(m, np.int32), rhs, obj, np.zeros(n), np.full(n, np.inf), True


KINDS = [("badly_scaled", badly_scaled, [1, 2, 3, 4, 5, 6]), ("near_dependent", near_dependent, [1, 2]),
         ("transport", transport, [1, 2, 3]), ("assignment", assignment, [1, 2]),
         ("wide_range", wide_range, [1, 2])]


def main():
    out = []
    for kind, fn, seeds in KINDS:
        for seed in seeds:
            A, dirs, rhs, obj, lo, up, mx = fn(seed)
            st, val = highs(A, dirs, rhs, obj, lo, up, mx)
            assert st == 0, (kind, seed, st)
            m, n = A.shape
            out.append({"name": f"{kind}_{seed}", "kind": kind, "m": m, "n": n,
                        "A_rowmajor": [float(v) for v in A.ravel()], "dir": [int(d) for d in dirs],
                        "rhs": [_enc(v) for v in rhs], "obj": [float(v) for v in obj],
                        "lo": [_enc(v) for v in lo], "up": [_enc(v) for v in up], "maximize": mx,
                        "objective": val})
            print(kind, seed, m, n, val)
    with open(os.path.join(HERE, "robust_lps.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
