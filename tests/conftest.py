import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _dec(v):
    if v == "inf":
        return np.inf
    if v == "-inf":
        return -np.inf
    return float(v)


def load_known_answers():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        recs = json.load(f)
    for r in recs:
        r["A"] = np.array(r["A_rowmajor"], dtype=np.float64).reshape(r["m"], r["n"])
        r["rhs"] = np.array([_dec(v) for v in r["rhs"]], dtype=np.float64)
        r["lo"] = np.array([_dec(v) for v in r["lo"]], dtype=np.float64)
        r["up"] = np.array([_dec(v) for v in r["up"]], dtype=np.float64)
        r["obj"] = np.array(r["obj"], dtype=np.float64)
        r["dir"] = np.array(r["dir"], dtype=np.int32)
    return recs


def load_dense_lps():
    with open(os.path.join(GOLDEN, "dense_lps.json")) as f:
        return json.load(f)


def load_generator_vectors():
    with open(os.path.join(GOLDEN, "generator_vectors.json")) as f:
        return json.load(f)


def feasible(A, dirs, rhs, x, lo, up, tol=2e-8):
    """R/class.R:533-540 + R/utils.R:167-171 (compare_tol), plus bounds."""
    lhs = A @ x if A.shape[0] else np.zeros(0)
    ok = True
    for i, d in enumerate(dirs):
        t = tol * max(1.0, abs(rhs[i]))
        if d == 1:
            ok &= lhs[i] <= rhs[i] + t
        elif d == 2:
            ok &= lhs[i] >= rhs[i] - t
        else:
            ok &= abs(lhs[i] - rhs[i]) <= t
    ok &= bool(np.all(x >= lo - tol * np.maximum(1, np.abs(lo[np.isfinite(lo)]).max(initial=1))))
    ok &= bool(np.all(x <= up + tol * np.maximum(1, np.abs(up[np.isfinite(up)]).max(initial=1))))
    return bool(ok)


@pytest.fixture(scope="session")
def gpu():
    """The HIP library on a GPU.  torch initialises the device first (its
    availability probe must not follow the library's own HIP start-up)."""
    import torch
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    torch.cuda.init()
    from easylp_amd import build
    build.build()
    import easylp_amd
    return easylp_amd


def load_sparse_lps():
    """tests/golden/sparse_lps.json (make_sparse.py): CSC arrays + HiGHS optimum;
    A_dense is the same matrix densified (for the oracle)."""
    with open(os.path.join(GOLDEN, "sparse_lps.json")) as f:
        recs = json.load(f)
    for r in recs:
        r["colptr"] = np.array(r["colptr"], dtype=np.int64)
        r["rowind"] = np.array(r["rowind"], dtype=np.int32)
        r["val"] = np.array(r["val"], dtype=np.float64)
        A = np.zeros((r["m"], r["n"]))
        for j in range(r["n"]):
            s, e = r["colptr"][j], r["colptr"][j + 1]
            A[r["rowind"][s:e], j] = r["val"][s:e]
        r["A"] = A
        r["rhs"] = np.array([_dec(v) for v in r["rhs"]], dtype=np.float64)
        r["lo"] = np.array([_dec(v) for v in r["lo"]], dtype=np.float64)
        r["up"] = np.array([_dec(v) for v in r["up"]], dtype=np.float64)
        r["obj"] = np.array(r["obj"], dtype=np.float64)
        r["dir"] = np.array(r["dir"], dtype=np.int32)
    return recs


def load_mip_known_answers():
    """tests/golden/mip_known_answers.json (make_mip.py): the reference's MIP tests."""
    with open(os.path.join(GOLDEN, "mip_known_answers.json")) as f:
        recs = json.load(f)
    for r in recs:
        A = np.zeros((r["m"], r["n"]))
        ii, jj, vv = r["A_triplets"]
        A[np.array(ii, dtype=int), np.array(jj, dtype=int)] = vv
        r["A"] = A
        for k in ("rhs", "obj", "lo", "up"):
            r[k] = np.array(r[k], dtype=np.float64)
        r["dir"] = np.array(r["dir"], dtype=np.int32)
        r["is_int"] = np.array(r["is_int"], dtype=np.int32)
    return recs


def load_robust_lps():
    """tests/golden/robust_lps.json (make_robust.py): badly scaled, nearly
    dependent, degenerate transport / assignment and wide-range LPs with the
    HiGHS optimum."""
    with open(os.path.join(GOLDEN, "robust_lps.json")) as f:
        recs = json.load(f)
    for r in recs:
        r["A"] = np.array(r["A_rowmajor"], dtype=np.float64).reshape(r["m"], r["n"])
        for k in ("rhs", "lo", "up"):
            r[k] = np.array([_dec(v) for v in r[k]], dtype=np.float64)
        r["obj"] = np.array(r["obj"], dtype=np.float64)
        r["dir"] = np.array(r["dir"], dtype=np.int32)
    return recs


def load_sparse_lu():
    """tests/golden/sparse_lu.json (make_sparse_lu.py): the larger sparse LPs of
    the sparse-LU engine -- generator spec + HiGHS optimum (or the optimum by
    construction)."""
    with open(os.path.join(GOLDEN, "sparse_lu.json")) as f:
        return json.load(f)
