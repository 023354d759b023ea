"""Generate the committed golden fixtures for the parity tests.

Run in the build container (needs scipy; NOT run on the GPU box):

    python tests/golden/make_golden.py

Outputs (all plain JSON data, no code):
  known_answers.json   LPs transcribed from the reference's tests / README /
                       vignettes, as the exact arrays easylp$solve() hands to
                       lp_solve (R/class.R:260-274), with the answers the
                       reference pins, cross-checked with SciPy-HiGHS.
  dense_lps.json       seeded dense LPs (SURVEY.md 8d generator) with the
                       HiGHS optimum: objective, nonzero x, sorted basis.
  generator_vectors.json  known-answer vectors of the counter-based generator
                       (hex bit patterns), computed here in numpy independently
                       of the C / HIP implementations.

lp_solve itself (the reference's backend) is absent from /root/reference and
from this image; the reference pins only objective values (test-DOP.R:53,
test-unbounded.R:8-9) and the README/vignette outputs.  Basis indices are
pinned to HiGHS ("parity unpinned" against lp_solve).
"""
from __future__ import annotations

import json
import os

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
INF = float("inf")

# ----------------------------------------------------------------------------
# generator (independent numpy restatement of oracle/elp_oracle.c gen_u01)
# ----------------------------------------------------------------------------
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def gen_u01(seed, stream, idx):
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = _mix64(np.array([np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
                               + np.uint64(stream) * np.uint64(0xD1B54A32D192ED03)
                               + np.uint64(0x632BE59BD9B4E019)], dtype=np.uint64))[0]
        z = _mix64(key + (idx + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15))
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def generate_dense(seed, m, n):
    i = np.arange(m, dtype=np.uint64)
    j = np.arange(n, dtype=np.uint64)
    idx = i[:, None] + j[None, :] * np.uint64(m)
    A = gen_u01(seed, 0, idx)
    c = gen_u01(seed, 1, j)
    b = (n / 8.0) + gen_u01(seed, 2, i) * (n / 4.0)
    return A, b, c


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------
def highs(A, dirs, rhs, obj, lo, up, maximize):
    A = np.asarray(A, dtype=float).reshape(len(rhs), len(obj))
    c = -np.asarray(obj, float) if maximize else np.asarray(obj, float)
    ub_rows, ub_rhs, eq_rows, eq_rhs = [], [], [], []
    for i, d in enumerate(dirs):
        if d == 1:
            ub_rows.append(A[i]); ub_rhs.append(rhs[i])
        elif d == 2:
            ub_rows.append(-A[i]); ub_rhs.append(-rhs[i])
        else:
            eq_rows.append(A[i]); eq_rhs.append(rhs[i])
    kw = {}
    if ub_rows:
        kw["A_ub"], kw["b_ub"] = np.array(ub_rows), np.array(ub_rhs)
    if eq_rows:
        kw["A_eq"], kw["b_eq"] = np.array(eq_rows), np.array(eq_rhs)
    bounds = [(None if l == -INF else l, None if u == INF else u) for l, u in zip(lo, up)]
    r = linprog(c, bounds=bounds, method="highs-ds", options={"presolve": False}, **kw)
    return r


def enc(v):
    """JSON-safe float (inf as string)."""
    if v == INF:
        return "inf"
    if v == -INF:
        return "-inf"
    return float(v)


def lp_record(name, source, A, dirs, rhs, obj, lo, up, maximize, expected, pinned_by,
              objective_add=0.0, feasibility_only=False):
    A = np.asarray(A, dtype=float).reshape(len(rhs), len(obj))
    return {
        "name": name,
        "source": source,
        "m": len(rhs),
        "n": len(obj),
        "A_rowmajor": A.tolist(),
        "dir": [int(d) for d in dirs],
        "rhs": [enc(v) for v in rhs],
        "obj": [float(v) for v in obj],
        "lo": [enc(v) for v in lo],
        "up": [enc(v) for v in up],
        "maximize": bool(maximize),
        "objective_add": objective_add,
        "expected": expected,
        "pinned_by": pinned_by,
        "feasibility_only": feasibility_only,
    }


# ----------------------------------------------------------------------------
# known answers from the reference
# ----------------------------------------------------------------------------
def known_answers():
    out = []
    LE, GE, EQ = 1, 2, 3

    # README.md:14-38 -- max x + y; x + 2y <= 3; y >= 3x - 2 (-> -3x + y >= -2,
    # R/methods.R:200-224 moves every variable to the lhs); x, y free
    # (default bounds -Inf/+Inf, R/class.R:86).
    A = [[1, 2], [-3, 1]]
    out.append(lp_record("readme", "README.md:14-38", A, [LE, GE], [3, -2], [1, 1],
                         [-INF, -INF], [INF, INF], True,
                         {"status": 0, "objective": 2.0, "x": [1.0, 1.0]}, "reference README output"))

    # tests/testthat/test-unbounded.R:2-10 -- max x, x free, no constraints.
    out.append(lp_record("unbounded", "tests/testthat/test-unbounded.R:2-10",
                         np.zeros((0, 1)), [], [], [1.0], [-INF], [INF], True,
                         {"status": 3, "objective": 1e30, "x": [1e30]},
                         "reference test (objective +Inf, x +Inf via large_to_infinity)"))

    # tests/testthat/test-DOP.R:1-54
    cap_rec = [6000, 7000, 8000, 7000]
    coef_ext = [.25, .3, .25, .2]
    cost_tdm = np.array([[54, 56], [60, 49], [41, 53], [54, 52]], float)  # DOP x Moli (byrow)
    cap_ext = [12000, 20000]
    cost_ext = [78, 82]
    cost_tms = np.array([[47, 56], [58, 51], [52, 59]], float)  # Super x Moli (byrow)
    demand = [1500, 3000, 2500]
    nd, nm, ns = 4, 2, 3
    tdm = lambda d, mo: d + nd * mo           # column-major DOP x Moli, vars 0..7
    tms = lambda mo, s: 8 + mo + nm * s       # column-major Moli x Super, vars 8..13
    n = 14
    obj = np.zeros(n)
    for d in range(nd):
        for mo in range(nm):
            obj[tdm(d, mo)] += cost_tdm[d, mo] + cost_ext[mo]
    # sum(cost_tms * tms): horizontal_multiply (R/methods.R:82-97) pairs the
    # coefficient rows of tms (storage order) with as.vector(cost_tms).
    cv = cost_tms.flatten(order="F")
    for k in range(6):
        obj[8 + k] += cv[k]
    rows, dirs, rhs = [], [], []
    for mo in range(nm):  # tdm_ext
        r = np.zeros(n)
        for d in range(nd):
            r[tdm(d, mo)] = coef_ext[d]
        for s in range(ns):
            r[tms(mo, s)] -= 1
        rows.append(r); dirs.append(EQ); rhs.append(0.0)
    for d in range(nd):  # recolleccio
        r = np.zeros(n)
        for mo in range(nm):
            r[tdm(d, mo)] = 1
        rows.append(r); dirs.append(LE); rhs.append(cap_rec[d])
    for mo in range(nm):  # extraccio
        r = np.zeros(n)
        for d in range(nd):
            r[tdm(d, mo)] = 1
        rows.append(r); dirs.append(LE); rhs.append(cap_ext[mo])
    for s in range(ns):  # satisfaccio
        r = np.zeros(n)
        for mo in range(nm):
            r[tms(mo, s)] = 1
        rows.append(r); dirs.append(GE); rhs.append(demand[s])
    out.append(lp_record("dop", "tests/testthat/test-DOP.R:27-54", np.array(rows), dirs, rhs, obj,
                         [0.0] * n, [INF] * n, False,
                         {"status": 0, "objective": 3985000.0, "objective_value": 3940000.0},
                         "reference test (objective_value == 3985000 - 45000)",
                         objective_add=-45000.0))

    # vignettes/objective.Rmd:30-52 -- max earnings - costs; earnings <= 3 costs;
    # costs <= 50; both free.
    out.append(lp_record("objective_basics", "vignettes/objective.Rmd:30-52", [[1, -3], [0, 1]],
                         [LE, LE], [0, 50], [1, -1], [-INF, -INF], [INF, INF], True,
                         {"status": 0, "objective": 100.0, "x": [150.0, 50.0]}, "vignette text + HiGHS"))

    # vignettes/objective.Rmd:155-171 -- min 4x + 3y + 50, x >= 10, y >= 10, no rows.
    out.append(lp_record("addend", "vignettes/objective.Rmd:155-171", np.zeros((0, 2)), [], [],
                         [4, 3], [10, 10], [INF, INF], False,
                         {"status": 0, "objective": 70.0, "objective_value": 120.0, "x": [10.0, 10.0]},
                         "vignette text (70 raw, 120 with addend)", objective_add=50.0))

    # vignettes/easylp.Rmd:211-218 -- min x + y, x >= 0, y >= 2, 2x + y >= 10.
    out.append(lp_record("import", "vignettes/easylp.Rmd:211-218", [[2, 1]], [GE], [10], [1, 1],
                         [0, 2], [INF, INF], False,
                         {"status": 0, "objective": 6.0, "x": [4.0, 2.0]}, "HiGHS"))

    # vignettes/constraints.Rmd:209-220 -- brass / bronze.
    out.append(lp_record("brass", "vignettes/constraints.Rmd:209-220",
                         [[0.90, 0.64], [0.10, 0.14], [0, 0.04]], [LE, LE, LE], [120, 15, 2],
                         [8, 6], [0, 0], [INF, INF], True,
                         {"status": 0, "objective": 33300.0 / 31.0, "x": [3600.0 / 31, 750.0 / 31]},
                         "HiGHS (exact rational 33300/31)"))

    # tests/testthat/test-modified.R:2-22 -- x[3x3], y[2x2x2] in [1,10], random
    # objective (unseeded runif in the test: fixed here), rowSums(x)==colSums(x),
    # diag(x)[2:3]==1:2, apply(y,1:2,mean)==2:5.  Pinned by feasibility only.
    rng = np.random.default_rng(2024)
    n = 9 + 8
    obj = np.concatenate([rng.uniform(-1, 1, 9), rng.uniform(-1, 1, 8)])
    X = lambda i, j: i + 3 * j
    Y = lambda i, j, k: 9 + i + 2 * j + 4 * k
    rows, dirs, rhs = [], [], []
    for i in range(3):
        r = np.zeros(n)
        for j in range(3):
            r[X(i, j)] += 1
            r[X(j, i)] -= 1
        rows.append(r); dirs.append(EQ); rhs.append(0.0)
    for d, v in ((1, 1.0), (2, 2.0)):
        r = np.zeros(n); r[X(d, d)] = 1
        rows.append(r); dirs.append(EQ); rhs.append(v)
    vals = {(0, 0): 2.0, (1, 0): 3.0, (0, 1): 4.0, (1, 1): 5.0}
    for (i, j), v in vals.items():
        r = np.zeros(n)
        r[Y(i, j, 0)] = 0.5; r[Y(i, j, 1)] = 0.5
        rows.append(r); dirs.append(EQ); rhs.append(v)
    out.append(lp_record("modified_simple", "tests/testthat/test-modified.R:2-22", np.array(rows),
                         dirs, rhs, obj, [1.0] * n, [10.0] * n, False,
                         {"status": 0}, "reference test (constraints hold)", feasibility_only=True))

    # tests/testthat/test-modified.R:25-41 -- x[4x3x2] in [-10,10], min sum(x).
    n = 24
    Xv = lambda a, b, c: a + 4 * b + 12 * c
    rows, dirs, rhs = [], [], []
    for a, v in ((0, 3.0), (1, 4.0)):
        r = np.zeros(n)
        for b in range(3):
            for c in range(2):
                r[Xv(a, b, c)] = 1
        rows.append(r); dirs.append(EQ); rhs.append(v)
    for a in (0, 1):
        r = np.zeros(n); r[Xv(a, 1, 0)] = 0.5; r[Xv(a, 1, 1)] = 0.5
        rows.append(r); dirs.append(EQ); rhs.append(2.0)
    out.append(lp_record("modified_indexed", "tests/testthat/test-modified.R:25-41", np.array(rows),
                         dirs, rhs, np.ones(n), [-10.0] * n, [10.0] * n, False,
                         {"status": 0}, "reference test (constraints hold)", feasibility_only=True))

    # Beale's cycling example (degeneracy).
    out.append(lp_record("beale", "SURVEY.md 8c (Beale 1955)",
                         [[0.25, -8, -1, 9], [0.5, -12, -0.5, 3], [0, 0, 1, 0]], [LE, LE, LE],
                         [0, 0, 1], [-0.75, 20, -0.5, 6], [0] * 4, [INF] * 4, False,
                         {"status": 0, "objective": -1.25, "x": [1.0, 0.0, 1.0, 0.0]}, "closed form"))

    # Klee-Minty cubes: optimum 5^n.
    for kn in (3, 6, 9):
        A = np.zeros((kn, kn))
        for i in range(kn):
            for j in range(i):
                A[i, j] = 2.0 ** (i - j + 1)
            A[i, i] = 1.0
        obj = [2.0 ** (kn - 1 - j) for j in range(kn)]
        rhs = [5.0 ** (i + 1) for i in range(kn)]
        x = [0.0] * (kn - 1) + [5.0 ** kn]
        out.append(lp_record(f"klee_minty_{kn}", "SURVEY.md 8c (Klee-Minty)", A, [LE] * kn, rhs, obj,
                             [0] * kn, [INF] * kn, True,
                             {"status": 0, "objective": 5.0 ** kn, "x": x}, "closed form"))

    # infeasible rows; and lower > upper (R/class.R:297-298 -> "unfeasible").
    out.append(lp_record("infeasible", "status 2 (R/class.R:281)", [[1, 1], [1, 0]], [LE, GE],
                         [1, 2], [1, 1], [0, 0], [INF, INF], True, {"status": 2}, "closed form"))
    out.append(lp_record("lower_gt_upper", "R/class.R:297-298", [[1]], [LE], [5], [1], [3], [2],
                         True, {"status": 2}, "reference status override"))
    # unbounded with rows (ray through a basic variable)
    out.append(lp_record("unbounded_rows", "status 3 (R/class.R:282)", [[1, -1]], [LE], [1], [1, 0],
                         [0, 0], [INF, INF], True, {"status": 3, "objective": 1e30}, "closed form"))
    # boxed variables (bound flips), mixed rows.
    out.append(lp_record("boxed", "bounded-variable path", [[1, 1, 1], [1, -1, 0], [0, 1, 1]],
                         [LE, GE, EQ], [10, -2, 6], [3, 2, 4], [0, 0, 1], [4, 5, 3], True,
                         {"status": 0}, "HiGHS"))

    # transportation LP relaxation, vignettes/easylp.Rmd:42-63 (integer flag dropped).
    supply = [50, 30, 45]
    dem = [30, 25, 40, 15]
    cost = np.array([[51, 89, 64, 32], [28, 87, 66, 48], [82, 78, 66, 29]], float)
    n = 12
    Xt = lambda f, mk: f + 3 * mk
    rows, dirs, rhs = [], [], []
    for f in range(3):
        r = np.zeros(n)
        for mk in range(4):
            r[Xt(f, mk)] = 1
        rows.append(r); dirs.append(LE); rhs.append(supply[f])
    for mk in range(4):
        r = np.zeros(n)
        for f in range(3):
            r[Xt(f, mk)] = 1
        rows.append(r); dirs.append(GE); rhs.append(dem[mk])
    out.append(lp_record("transport", "vignettes/easylp.Rmd:42-63 (LP relaxation)", np.array(rows),
                         dirs, rhs, cost.flatten(order="F"), [0] * n, [INF] * n, False,
                         {"status": 0}, "HiGHS"))

    # cross-check every record against HiGHS and fill HiGHS answers
    for rec in out:
        A = np.array(rec["A_rowmajor"], float).reshape(rec["m"], rec["n"])
        dec = lambda v: INF if v == "inf" else (-INF if v == "-inf" else v)
        lo = [dec(v) for v in rec["lo"]]
        up = [dec(v) for v in rec["up"]]
        if any(l > u for l, u in zip(lo, up)):
            continue
        r = highs(A, rec["dir"], [dec(v) for v in rec["rhs"]], rec["obj"], lo, up, rec["maximize"])
        exp = rec["expected"]
        hs = {0: 0, 2: 2, 3: 3}[r.status]
        assert hs == exp["status"], (rec["name"], r.status, exp)
        if hs == 0:
            hobj = -r.fun if rec["maximize"] else r.fun
            if "objective" in exp:
                assert abs(hobj - exp["objective"]) <= 1e-9 * max(1, abs(hobj)), (rec["name"], hobj)
            else:
                exp["objective"] = hobj
            exp.setdefault("highs_x", r.x.tolist())
    return out


def dense_lps():
    out = []
    for (m, n, seeds) in ((20, 60, (1, 2, 3)), (50, 200, (1, 2, 3, 4, 5)), (200, 800, (1, 2, 3)),
                          (500, 2000, (1, 2, 3, 4, 5)), (1000, 5000, (1,))):
        for seed in seeds:
            A, b, c = generate_dense(seed, m, n)
            r = linprog(-c, A_ub=A, b_ub=b, bounds=(0, None), method="highs-ds",
                        options={"presolve": False})
            assert r.status == 0
            xb = np.nonzero(r.x > 1e-9)[0]
            sb = np.nonzero(r.slack > 1e-9)[0]
            basis = np.sort(np.concatenate([xb, n + sb]))
            nondegenerate = len(basis) == m
            out.append({
                "seed": seed, "m": m, "n": n,
                "objective": -r.fun,
                "x_nonzero": {str(int(j)): float(r.x[j]) for j in xb},
                "basis": [int(v) for v in basis],
                "nondegenerate": bool(nondegenerate),
                "highs_iterations": int(r.nit),
            })
            print(f"dense seed={seed} m={m} n={n} obj={-r.fun:.9f} k={len(xb)} nondeg={nondegenerate}")
    return out


def generator_vectors():
    recs = []
    for seed, m, n in ((1, 500, 2000), (7, 5000, 50000), (3, 10000, 500000)):
        idx_i = [0, 1, m - 1, 17 % m]
        idx_j = [0, 1, n - 1, 12345 % n]
        A = [[i, j, gen_u01(seed, 0, [i + j * m])[0].hex()] for i in idx_i for j in idx_j]
        c = [[j, gen_u01(seed, 1, [j])[0].hex()] for j in idx_j]
        b = [[i, ((n / 8.0) + gen_u01(seed, 2, [i]) * (n / 4.0))[0].hex()] for i in idx_i]
        recs.append({"seed": seed, "m": m, "n": n, "A": A, "c": c, "b": b})
    return recs


def main():
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(known_answers(), f, indent=1)
    with open(os.path.join(HERE, "generator_vectors.json"), "w") as f:
        json.dump(generator_vectors(), f, indent=1)
    with open(os.path.join(HERE, "dense_lps.json"), "w") as f:
        json.dump(dense_lps(), f, indent=1)


if __name__ == "__main__":
    main()
