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
