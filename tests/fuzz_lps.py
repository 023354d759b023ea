"""Seeded general-form LPs of every shape the R front-end can hand to
easylp$solve() (R/class.R:251-302): constraint rows of all three directions,
bounds of every kind (lower only, boxed, fixed, upper only, free), empty and
one-row / one-column models, integer-valued degenerate matrices, badly scaled
rows and columns, zero objectives, and LPs that are infeasible or unbounded by
construction.  Shared by tests/test_fuzz_oracle.py (oracle vs HiGHS, CPU) and
tests/test_gpu_fuzz.py (HIP path vs oracle)."""
import numpy as np

INF = np.inf

# kind of the LP's outcome by construction: "feasible" (x0 satisfies every
# row and bound), "infeasible" (a row no x >= 0 can meet), "open" (rhs drawn
# at random: any status)
KINDS = ("feasible", "feasible", "feasible", "infeasible", "open")


def _shape(rng):
    r = rng.random()
    if r < 0.08:
        return 0, int(rng.integers(1, 12))  # no constraint rows
    if r < 0.16:
        return 1, int(rng.integers(1, 40))
    if r < 0.24:
        return int(rng.integers(1, 30)), 1
    if r < 0.40:
        m = int(rng.integers(20, 90))
        return m, int(rng.integers(5, m))  # tall
    return int(rng.integers(2, 70)), int(rng.integers(2, 160))


def _matrix(rng, m, n):
    style = rng.integers(0, 4)
    if style == 0:
        A = rng.uniform(-1, 1, (m, n))
    elif style == 1:  # small integers, many zeros and ties: degenerate pivots
        A = rng.integers(-3, 4, (m, n)).astype(np.float64)
        A[rng.random((m, n)) < 0.5] = 0.0
    elif style == 2:  # nonnegative sparse (packing / covering shapes)
        A = rng.uniform(0, 1, (m, n))
        A[rng.random((m, n)) < 0.6] = 0.0
    else:  # badly scaled rows and columns
        A = rng.uniform(-1, 1, (m, n))
        A *= 10.0 ** rng.uniform(-3, 3, (m, 1))
        A *= 10.0 ** rng.uniform(-3, 3, (1, n))
    return A, int(style)


def _bounds(rng, n):
    lo = np.zeros(n)
    up = np.full(n, INF)
    # half of the LPs keep every column bounded below (lp_solve's default
    # [0, inf), boxed, fixed); the rest mix in free and upper-only columns
    mixed = rng.random() < 0.5
    kind = rng.integers(0, 6, n)
    if not mixed:
        kind[(kind == 2) | (kind == 4)] = 0
    for j in range(n):
        if kind[j] == 1:  # boxed
            lo[j] = float(rng.integers(-3, 1))
            up[j] = lo[j] + float(rng.integers(1, 6))
        elif kind[j] == 2:  # free
            lo[j], up[j] = -INF, INF
        elif kind[j] == 3:  # fixed
            lo[j] = up[j] = float(rng.integers(0, 3))
        elif kind[j] == 4:  # upper only
            lo[j], up[j] = -INF, float(rng.integers(0, 4))
        # 0, 5: [0, inf), the R default
    return lo, up


def fuzz_lp(seed):
    """One LP: dict with A (m x n), dir (1 <=, 2 >=, 3 ==), rhs, obj, lo, up,
    maximize, and the generator's labels (kind, style)."""
    rng = np.random.default_rng(1000 + seed)
    m, n = _shape(rng)
    kind = KINDS[seed % len(KINDS)] if m > 0 else "feasible"
    A, style = _matrix(rng, m, n)
    lo, up = _bounds(rng, n)
    # a point inside the bounds
    x0 = np.where(np.isfinite(lo), lo, np.where(np.isfinite(up), up - 2.0, 0.0))
    span = np.where(np.isfinite(up) & np.isfinite(lo), up - lo, 2.0)
    x0 = x0 + rng.uniform(0, 1, n) * span
    dirs = rng.integers(1, 4, m).astype(np.int32)
    act = A @ x0 if m else np.zeros(0)
    slack = rng.uniform(0, 1, m) * (rng.random(m) < 0.7)  # tight rows stay degenerate
    rhs = np.where(dirs == 1, act + slack, np.where(dirs == 2, act - slack, act))
    if kind == "open":
        rhs = rng.uniform(-2, 2, m)
    if kind == "infeasible":
        # row 0 becomes  sum_j |a_0j| (x_j - lo_j) <= -1  over columns with finite
        # lo (the others get coefficient 0): impossible for x >= lo
        fin = np.isfinite(lo)
        A[0, :] = np.where(fin, np.abs(A[0, :]) + 0.5, 0.0)
        if not fin.any():  # every column free: make column 0 [0, inf)
            lo[0], up[0] = 0.0, INF
            A[0, 0] = 1.0
            fin = np.isfinite(lo)
        dirs[0] = 1
        rhs[0] = float(A[0, fin] @ lo[fin]) - 1.0
    obj = rng.uniform(-1, 1, n) if rng.random() > 0.1 else np.zeros(n)
    if style == 1:
        obj = rng.integers(-3, 4, n).astype(np.float64)
    return {"A": A, "dir": dirs, "rhs": rhs, "obj": obj, "lo": lo, "up": up,
            "maximize": bool(rng.random() < 0.5), "kind": kind, "style": style,
            "m": m, "n": n, "seed": seed}


def fuzz_set(count, start=0):
    return [fuzz_lp(s) for s in range(start, start + count)]


def fuzz_mip(seed):
    """A small MIP (branch and bound stays at a few hundred nodes): integer
    coefficients, every column boxed or bounded by a packing row, a random
    subset of the columns integer; one in five is integer-infeasible by
    construction (an equality row 2 x_0 + 2 x_1 = odd over integer columns)."""
    rng = np.random.default_rng(5000 + seed)
    m, n = int(rng.integers(1, 9)), int(rng.integers(2, 11))
    A = rng.integers(-2, 6, (m, n)).astype(np.float64)
    dirs = rng.integers(1, 4, m).astype(np.int32)
    dirs[0] = 1
    A[0, :] = rng.integers(1, 6, n)  # a packing row bounds every column
    lo = np.zeros(n)
    up = np.where(rng.random(n) < 0.5, rng.integers(1, 8, n).astype(np.float64), INF)
    x0 = np.floor(rng.uniform(0, 1, n) * np.where(np.isfinite(up), up + 1, 4.0))
    act = A @ x0
    rhs = np.where(dirs == 1, act + rng.integers(0, 4, m), np.where(dirs == 2, act - rng.integers(0, 4, m), act))
    is_int = (rng.random(n) < 0.7).astype(np.int32)
    infeasible = seed % 5 == 4
    if infeasible:
        is_int[:2] = 1
        A = np.vstack([A, np.zeros(n)])
        A[-1, :2] = 2.0
        dirs = np.append(dirs, np.int32(3))
        rhs = np.append(rhs, 2.0 * (x0[0] + x0[1]) + 1.0)
        m += 1
    obj = rng.integers(-4, 9, n).astype(np.float64)
    return {"A": A, "dir": dirs, "rhs": rhs.astype(np.float64), "obj": obj, "lo": lo, "up": up,
            "maximize": bool(rng.random() < 0.7), "is_int": is_int, "m": m, "n": n, "seed": seed,
            "kind": "infeasible" if infeasible else "feasible"}
