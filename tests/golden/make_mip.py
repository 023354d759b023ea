"""Generate tests/golden/mip_known_answers.json: the reference's MIP tests
transcribed into the arrays easylp$solve() hands to lp_solve (R/class.R:260-274,
set.type at :265), with the answers the reference pins, cross-checked here with
SciPy-HiGHS `milp`.

    python tests/golden/make_mip.py      (build container only; needs scipy)

  investments  tests/testthat/test-investments.R:1-45  objective 469, x = (0,0,1,1,1,0)
  students     tests/testthat/test-students.R:1-40     objective_value 131 (raw 130, addend 1)
  cyingair     tests/testthat/test-cyingair.R:1-28     x = (0,2,3,49), quin = (0,1,1,1)
"""
from __future__ import annotations

import json
import os

import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp

HERE = os.path.dirname(os.path.abspath(__file__))


def investments():
    npv = [141, 187, 121, 83, 265, 127]
    budget = [250, 75, 50, 50, 50]
    inv = np.array([[75, 25, 20, 15, 10], [90, 35, 0, 0, 30], [60, 15, 15, 15, 15],
                    [30, 20, 10, 5, 5], [100, 25, 20, 20, 20], [50, 20, 10, 30, 40]], float)
    NA = None
    inc = [[NA, 1, 0, 1, 0, 0], [NA, NA, 1, 0, 0, 0], [NA, NA, NA, 0, 0, 0],
           [NA, NA, NA, NA, 0, 0], [NA, NA, NA, NA, NA, 1], [NA] * 6]
    rows, dirs, rhs = [], [], []
    for a in range(5):  # budget[a]: sum_p x_p inv[p, a] <= budget[a]
        rows.append(inv[:, a]); dirs.append(1); rhs.append(budget[a])
    for p in range(5):  # x_p + x_q + incompatible[p, q] <= 2
        for q in range(p + 1, 6):
            r = np.zeros(6); r[p] = r[q] = 1
            rows.append(r); dirs.append(1); rhs.append(2 - inc[p][q])
    return dict(name="investments", source="tests/testthat/test-investments.R:1-45",
                A=np.array(rows), dir=dirs, rhs=rhs, obj=npv, lo=[0] * 6, up=[1] * 6,
                is_int=[1] * 6, maximize=True, objective_add=0,
                expected={"status": 0, "objective": 469, "x": [0, 0, 1, 1, 1, 0]})


AFFINITY = """-0 8 -2 5 -1 -0 7 -5 -1 5 3 4 -3 7 -2 5 -2 7 1 -0 3 -1
 -1 0 -7 -5 3 8 0 3 2 0 1 5 7 1 -1 6 5 -2 -4 5 -5 -2
 6 -2 0 -3 5 8 8 -4 4 4 6 4 8 -3 2 4 8 1 8 2 2 6
 -1 2 -1 0 -3 6 4 -0 5 6 3 -1 -2 4 7 6 -1 4 5 1 3 -1
 4 4 -0 -1 0 5 -5 2 2 6 4 -4 -6 -1 6 -4 4 1 7 -3 -7 0
 5 -5 2 5 -4 -0 1 -1 -5 -0 6 4 3 -2 3 8 3 8 8 8 5 4
 2 7 -3 3 -3 7 0 7 7 -4 5 3 5 -0 5 1 3 -8 2 3 4 0
 6 7 1 5 -8 7 3 0 7 -3 -4 4 -3 5 5 -6 -5 -5 -2 1 6 2
 -1 4 4 -2 2 5 4 4 0 -1 7 -0 1 -5 9 -4 5 7 6 5 3 8
 -1 1 7 -3 2 0 5 -5 8 0 -0 0 7 3 6 4 5 3 0 1 9 5
 -1 -1 2 6 3 7 -3 3 2 3 0 0 3 6 1 2 -1 1 4 -1 1 2
 -4 -0 2 8 6 -5 2 5 8 6 3 0 7 -1 -6 -2 0 7 0 3 4 9
 -6 -0 7 0 -0 6 5 1 -0 -2 7 8 0 5 -1 1 4 0 -3 5 6 1
 6 2 5 1 3 4 1 6 0 5 2 7 -5 -0 2 5 -5 3 3 8 5 5
 4 -4 1 7 3 -6 3 6 1 7 -2 8 -3 4 0 6 -5 7 5 -7 -5 -4
 8 5 -6 -6 6 3 9 7 -5 -6 7 1 -6 5 5 0 4 6 -0 1 8 4
 1 4 -3 -0 4 3 -1 5 -2 3 -7 5 8 1 1 -5 -0 3 5 2 8 1
 -6 5 -5 5 1 3 1 2 -5 -0 -4 2 -6 4 4 0 -4 0 7 -3 4 -5
 8 -2 2 -6 3 2 1 5 2 4 5 -1 7 6 8 -3 -1 -3 -0 2 6 5
 -1 4 4 6 -1 -6 -1 8 3 6 1 7 3 5 1 3 -2 2 4 0 -2 4
 5 -4 -5 3 1 5 3 4 4 3 5 2 -6 5 6 6 5 5 4 4 0 5
 7 -2 4 2 5 -2 8 -1 -1 4 7 -2 -2 7 1 7 -3 6 2 4 9 -0"""


def students():
    aff = np.array([int(v) for v in AFFINITY.split()], float)
    ns = int(round(np.sqrt(aff.size)))
    aff = aff.reshape(ns, ns)  # byrow = TRUE
    # pair[s1, s2]: R array, s1 fastest -> column index s1 + ns * s2
    col = lambda i, j: i + ns * j  # noqa: E731
    n = ns * ns
    obj = np.zeros(n)
    for i in range(ns):
        for j in range(ns):
            obj[col(i, j)] = aff[i, j]
    rows, dirs, rhs = [], [], []
    for i in range(ns):  # paired: pair[i, j] == pair[j, i], j in i:ns
        for j in range(i, ns):
            r = np.zeros(n); r[col(i, j)] += 1; r[col(j, i)] -= 1
            rows.append(r); dirs.append(3); rhs.append(0.0)
    for i in range(ns):  # everyone_has_one_pair: sum(pair[i, ]) == 1
        r = np.zeros(n)
        for j in range(ns):
            r[col(i, j)] = 1
        rows.append(r); dirs.append(3); rhs.append(1.0)
    return dict(name="students", source="tests/testthat/test-students.R:1-40",
                A=np.array(rows), dir=dirs, rhs=rhs, obj=obj, lo=[0] * n, up=[1] * n,
                is_int=[1] * n, maximize=True, objective_add=1,
                expected={"status": 0, "objective": 130, "objective_value": 131})


def cyingair():
    preu = [79, 67, 50, 35]
    ben = [5.8, 4.2, 3, 2.3]
    # columns: quin[0..3] (binary), x[0..3] (integer, [0, 100])
    n = 8
    Q = lambda a: a  # noqa: E731
    X = lambda a: 4 + a  # noqa: E731
    rows, dirs, rhs = [], [], []

    def row(coefs, d, b):
        r = np.zeros(n)
        for c, v in coefs:
            r[c] += v
        rows.append(r); dirs.append(d); rhs.append(b)
    for a in range(4):  # associate(x, quin, min1 = 1): R/class.R:349-355
        row([(X(a), 1), (Q(a), -100)], 1, 0)      # x <= 0 + (100 - 0) quin
    for a in range(4):
        row([(X(a), 1), (Q(a), -1)], 2, 0)        # x >= 0 + (1 - 0) quin
    row([(Q(a), 1) for a in range(4)], 3, 3)      # tipus
    row([(X(a), preu[a]) for a in range(4)], 1, 2000)  # r_pressupost
    row([(X(a), 1) for a in range(4)], 2, 35)     # min_avions
    row([(X(1), 1), (X(2), -1)], 1, 0)            # Petit <= Mitja
    row([(Q(0), 1), (Q(3), 1)], 1, 1)             # no_jumbo_i_grans
    row([(X(0), 1)] + [(X(a), -0.15) for a in range(4)], 1, 0)  # quinze_percent
    obj = [0, 0, 0, 0] + ben
    return dict(name="cyingair", source="tests/testthat/test-cyingair.R:1-28",
                A=np.array(rows), dir=dirs, rhs=rhs, obj=obj, lo=[0] * 8,
                up=[1, 1, 1, 1, 100, 100, 100, 100], is_int=[1] * 8, maximize=True,
                objective_add=0,
                expected={"status": 0, "objective": float(np.dot(ben, [0, 2, 3, 49])),
                          "x": [0, 1, 1, 1, 0, 2, 3, 49]})


def check(rec):
    A = np.asarray(rec["A"], float)
    d = np.asarray(rec["dir"])
    b = np.asarray(rec["rhs"], float)
    lb = np.where(d == 2, b, np.where(d == 3, b, -np.inf))
    ub = np.where(d == 1, b, np.where(d == 3, b, np.inf))
    c = -np.asarray(rec["obj"], float) if rec["maximize"] else np.asarray(rec["obj"], float)
    r = milp(c, constraints=LinearConstraint(A, lb, ub), integrality=np.asarray(rec["is_int"]),
             bounds=Bounds(rec["lo"], rec["up"]))
    assert r.status == 0
    obj = -r.fun if rec["maximize"] else r.fun
    assert abs(obj - rec["expected"]["objective"]) <= 1e-6, (rec["name"], obj)
    if "x" in rec["expected"]:
        assert np.allclose(r.x, rec["expected"]["x"], atol=1e-6), (rec["name"], r.x)
    return obj


def main():
    recs = [investments(), students(), cyingair()]
    out = []
    for r in recs:
        print(r["name"], check(r))
        r = dict(r)
        r["m"], r["n"] = np.asarray(r["A"]).shape
        A = np.asarray(r.pop("A"), float)
        ii, jj = np.nonzero(A)
        r["A_triplets"] = [ii.tolist(), jj.tolist(), A[ii, jj].tolist()]
        for k in ("rhs", "obj", "lo", "up"):
            r[k] = [float(v) for v in r[k]]
        r["dir"] = [int(v) for v in r["dir"]]
        r["is_int"] = [int(v) for v in r["is_int"]]
        out.append(r)
    with open(os.path.join(HERE, "mip_known_answers.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
