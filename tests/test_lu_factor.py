"""The sparse-LU basis of the CSC path, CPU side: the product's
host factorization (easylp_amd/csrc/elp_lu_factor.cpp, compiled here alone
with g++ -- no HIP) must produce exactly the oracle's factors
(oracle/elp_oracle_lu.c lu_factor): same pivot sequence, U diagonal, fill and
factor values (order-sensitive checksums).  Also the oracle engine against
HiGHS objectives (tests/golden/sparse_lps.json) and the dense oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_known_answers, load_robust_lps, load_sparse_lps

SRC = os.path.join(ROOT, "easylp_amd", "csrc", "elp_lu_factor.cpp")


@pytest.fixture(scope="module")
def host_lu(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("lu") / "liblu_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", so, SRC],
                   check=True)
    lib = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    lib.elp_lu_factor_host.restype = ctypes.c_int
    lib.elp_lu_factor_host.argtypes = [ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, ctypes.c_double,
                                       vp, vp, vp, vp, vp, vp, vp]
    return lib


def _host(lib, cp, ri, v, m, head):
    n = len(cp) - 1
    cp = np.ascontiguousarray(cp, np.int64)
    ri = np.ascontiguousarray(ri, np.int32)
    v = np.ascontiguousarray(v, np.float64)
    head = np.ascontiguousarray(head, np.int64)
    prow, pcol = np.zeros(max(m, 1), np.int64), np.zeros(max(m, 1), np.int64)
    ud, nz, nlev = np.zeros(max(m, 1)), np.zeros(2, np.int64), np.zeros(4, np.int32)
    ls, us = ctypes.c_double(0), ctypes.c_double(0)
    rc = lib.elp_lu_factor_host(m, n, cp.ctypes.data, ri.ctypes.data, v.ctypes.data, head.ctypes.data, 1e-13,
                                prow.ctypes.data, pcol.ctypes.data, ud.ctypes.data, nz.ctypes.data,
                                ctypes.addressof(ls), ctypes.addressof(us), nlev.ctypes.data)
    if rc:
        return None
    return prow[:m], pcol[:m], ud[:m], tuple(int(x) for x in nz), (ls.value, us.value), nlev


def _bases():
    from easylp_amd.solver import csc_arrays
    from easylp_amd.synth import sparse_packing
    from oracle import solve_lu
    out = []
    for r in load_sparse_lps() + load_robust_lps():
        cp, ri, v, (m, n) = csc_arrays(r["A"])
        o = solve_lu(cp, ri, v, r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"])
        if o.status == 0 and m:
            out.append((r.get("name", "lp"), cp, ri, v, m, o.basis))
    cp, ri, v, b, c = sparse_packing(3, 300, 2000, 5)
    o = solve_lu(cp, ri, v, np.ones(300, np.int32), b, c, maximize=True)
    out.append(("packing_300x2000", cp, ri, v, 300, o.basis))
    rng = np.random.default_rng(0)  # random mixed bases (some singular: both sides must agree)
    for t in range(6):
        head = np.sort(rng.choice(2000 + 300, 300, replace=False))
        out.append((f"random_{t}", cp, ri, v, 300, head))
    return out


@pytest.mark.parametrize("case", _bases(), ids=lambda c: c[0])
def test_host_factor_equals_oracle(host_lu, case):
    from oracle import lu_factor
    name, cp, ri, v, m, head = case
    o = lu_factor(cp, ri, v, m, head)
    h = _host(host_lu, cp, ri, v, m, head)
    assert (o is None) == (h is None)
    if o is None:
        return
    np.testing.assert_array_equal(h[0], o[0])
    np.testing.assert_array_equal(h[1], o[1])
    np.testing.assert_array_equal(h[2], o[2])
    assert h[3] == o[3]
    assert h[4] == o[4]
    assert (h[5] >= 1).all() and (h[5] <= m).all()


def test_oracle_lu_engine_vs_highs_and_dense():
    """orc_solve_lu on the sparse fixtures (HiGHS optimum), the reference's
    known answers and the robustness LPs: same status and optimum as the
    dense-engine oracle (CSC pricing order) and HiGHS."""
    from easylp_amd.solver import csc_arrays
    from oracle import solve_dense, solve_lu
    for r in load_sparse_lps() + load_known_answers() + load_robust_lps():
        cp, ri, v, (m, n) = csc_arrays(r["A"])
        o = solve_lu(cp, ri, v, r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"])
        d = solve_dense(r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"], price_mode=1)
        assert o.status == d.status, r.get("name")
        if o.status == 0:
            assert abs(o.objval - d.objval) <= 1e-9 * max(1.0, abs(d.objval)), r.get("name")
            exp = r.get("objective", (r.get("expected") or {}).get("objective"))
            if exp is not None:
                assert abs(o.objval - exp) <= 1e-8 * max(1.0, abs(exp)), r.get("name")
