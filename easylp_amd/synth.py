"""Synthetic sparse LPs for the CSC path (bench.py `sparse_config`, tests).

Netlib files are not in this image, so BASELINE config 5 ("Netlib-scale sparse
A in CSC") is measured on a seeded LP of Netlib-like shape: maximize c'x s.t.
A x <= b, x >= 0, each column with `per_col` distinct rows (A_ij ~ U[0.05, 1)),
b_i = (row sum) / 4 + U[0, 1) -- every column has a positive entry, so the LP
is bounded, and x = 0 is feasible (no phase 1).  Vectorised numpy, so a
2000 x 20000 instance takes well under a second.
"""
from __future__ import annotations

import numpy as np


def sparse_packing(seed: int, m: int, n: int, per_col: int = 5):
    """-> colptr (int64), rowind (int32), val, b, c  (CSC, rows ascending)."""
    rng = np.random.default_rng(seed)
    k = min(per_col, m)
    # distinct rows per column: sample with replacement, sort, drop repeats
    rows = np.sort(rng.integers(0, m, size=(n, k + 2)), axis=1)
    keep = np.ones_like(rows, dtype=bool)
    keep[:, 1:] = rows[:, 1:] != rows[:, :-1]
    # at most k distinct rows per column (the first k distinct ones)
    keep &= np.cumsum(keep, axis=1) <= k
    counts = keep.sum(axis=1)
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=colptr[1:])
    rowind = rows[keep].astype(np.int32)
    val = rng.uniform(0.05, 1.0, size=rowind.size)
    rowsum = np.bincount(rowind, weights=val, minlength=m)
    b = rowsum / 4.0 + rng.uniform(0.0, 1.0, size=m)
    c = rng.uniform(0.0, 1.0, size=n)
    return colptr, rowind, val, b, c


def dense_of(colptr, rowind, val, m: int, n: int) -> np.ndarray:
    A = np.zeros((m, n), order="F")
    cols = np.repeat(np.arange(n), np.diff(colptr))
    A[rowind, cols] = val
    return A


def sparse_kkt(seed: int, m: int, n: int, k: int, per_col: int = 5, feasible_start: bool = False):
    """A sparse boxed LP of Netlib-like size whose optimum is known by
    construction (a KKT point), for the sparse-LU engine at scales no offline
    reference solver finishes here:

        maximize c'x  s.t.  A x <= b,  0 <= x <= u,

    every column with `per_col` distinct rows (A_ij ~ +-U[0.1, 1)); k binding
    rows R and k fractional columns S with A[R_p, S_p] = 2 + U (a strong
    diagonal, so A[R, S] is nonsingular); x*: the S columns strictly inside
    their bounds, the others at 0 or at u (one in ten); y* > 0 on R only;
    b = A x* on R and A x* + U[0.1, 1) elsewhere; c_j = a_j'y* on S and
    a_j'y* -+ U[0.05, 1) on the columns at 0 / at u, so (x*, y*) is primal and
    dual feasible and complementary: optimal.  Returns colptr, rowind, val, b,
    c, u, objective (c'x*, computed here in float64).

    feasible_start: every entry positive and no column at its upper bound in
    x*, so b >= 0 and the slack basis is feasible (no phase 1) and no column
    has to cross the basis on its way to u.  The default LP needs a phase 1
    over the rows with b_i < 0 and moves one column in ten to its upper bound
    through the basis: a primal simplex walks ~70 000 pivots on it at
    20 000 x 100 000 with up to ~8 800 basic structurals."""
    rng = np.random.default_rng(seed)
    R = np.sort(rng.choice(m, k, replace=False))
    S = np.sort(rng.choice(n, k, replace=False))
    rows = np.sort(rng.integers(0, m, size=(n, per_col + 2)), axis=1)
    keep = np.ones_like(rows, dtype=bool)
    keep[:, 1:] = rows[:, 1:] != rows[:, :-1]
    keep &= np.cumsum(keep, axis=1) <= per_col
    cols = [list(rows[j][keep[j]]) for j in range(n)]
    for p in range(k):  # the diagonal of A[R, S]
        col = cols[S[p]]
        if R[p] not in col:
            col[-1] = R[p]
            col.sort()
            while len(set(col)) < len(col):  # (a duplicate: take the next free row)
                col = sorted(set(col))
            cols[S[p]] = col
    counts = np.array([len(cc) for cc in cols], dtype=np.int64)
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=colptr[1:])
    rowind = np.concatenate([np.asarray(cc, dtype=np.int32) for cc in cols])
    val = rng.uniform(0.1, 1.0, size=rowind.size) * rng.choice([-1.0, 1.0], size=rowind.size, p=[0.3, 0.7])
    if feasible_start:
        val = np.abs(val)
    colid = np.repeat(np.arange(n), counts)
    rpos = np.full(m, -1)
    rpos[R] = np.arange(k)
    spos = np.full(n, -1)
    spos[S] = np.arange(k)
    diag = (spos[colid] >= 0) & (rpos[rowind] == spos[colid])
    val[diag] = 2.0 + rng.uniform(0.0, 1.0, size=int(diag.sum()))
    u = rng.uniform(1.0, 10.0, size=n)
    x = np.zeros(n)
    at_up = rng.random(n) < 0.1
    if feasible_start:
        at_up[:] = False
    x[at_up] = u[at_up]
    x[S] = u[S] * rng.uniform(0.2, 0.8, size=k)
    at_up[S] = False
    y = np.zeros(m)
    y[R] = rng.uniform(0.5, 2.0, size=k)
    ax = np.bincount(rowind, weights=val * x[colid], minlength=m)
    b = ax.copy()
    nb = np.ones(m, dtype=bool)
    nb[R] = False
    b[nb] += rng.uniform(0.1, 1.0, size=int(nb.sum()))
    aty = np.bincount(colid, weights=val * y[rowind], minlength=n)
    delta = rng.uniform(0.05, 1.0, size=n)
    c = aty - delta
    c[at_up] = aty[at_up] + delta[at_up]
    c[S] = aty[S]
    objective = float(c @ x)
    return colptr, rowind, val, b, c, u, objective
