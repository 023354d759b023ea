"""ctypes binding for oracle/_build/libelp_oracle.so -- TEST INFRASTRUCTURE ONLY.

Mirrors the argument meaning of the product C ABI (include/easylp_hip.h) so the
parity tests can feed both the same arrays.  The C code it wraps restates the
solve that /root/reference/R/class.R:260-278 hands to lp_solve.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libelp_oracle.so")
# ELP_ORACLE_SO: another build of the same source (the ASan/UBSan one of
# `make sanitize`, run_sanitized_tests.sh)
_SO = os.environ.get("ELP_ORACLE_SO") or _SO
_lib = None


class OrcControl(ctypes.Structure):
    _fields_ = [
        ("tol_primal", ctypes.c_double),
        ("tol_dual", ctypes.c_double),
        ("tol_pivot", ctypes.c_double),
        ("infinity", ctypes.c_double),
        ("max_iter", ctypes.c_int64),
        ("refactor_period", ctypes.c_int32),
        ("degen_switch", ctypes.c_int32),
        ("t_mark_iter", ctypes.c_int64),
        ("refactor_mode", ctypes.c_int32),
        ("price_mode", ctypes.c_int32),
        ("price_rule", ctypes.c_int32),
        ("scaling", ctypes.c_int32),
        ("tol_singular", ctypes.c_double),
        ("simplex", ctypes.c_int32),
        ("pad0", ctypes.c_int32),
    ]


class OrcStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int64),
        ("phase1_iterations", ctypes.c_int64),
        ("bound_flips", ctypes.c_int64),
        ("degenerate", ctypes.c_int64),
        ("refactors", ctypes.c_int64),
        ("bump_dim", ctypes.c_int64),
        ("y_rows", ctypes.c_int64),
        ("seconds", ctypes.c_double),
        ("price_bytes", ctypes.c_double),
        ("seconds_at_mark", ctypes.c_double),
        ("gj_refactors", ctypes.c_int64),
        ("devex_resets", ctypes.c_int64),
        ("max_inv_resid", ctypes.c_double),
        ("lu_nnz", ctypes.c_int64),
        ("eta_nnz", ctypes.c_int64),
        ("dual_iterations", ctypes.c_int64),
        ("flattened", ctypes.c_int64),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_SO):
        build()
    lib = ctypes.CDLL(_SO)
    P = ctypes.POINTER
    lib.orc_default_control.argtypes = [P(OrcControl)]
    lib.orc_solve_dense.restype = ctypes.c_int
    lib.orc_solve_dense.argtypes = [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, P(OrcControl),
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_int64, P(OrcStats),
    ]
    lib.orc_solve_dense_sens.restype = ctypes.c_int
    lib.orc_solve_dense_sens.argtypes = lib.orc_solve_dense.argtypes + [ctypes.c_void_p]
    lib.orc_solve_mip.restype = ctypes.c_int
    lib.orc_solve_mip.argtypes = [
        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
        P(OrcControl), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, P(ctypes.c_int64),
        P(ctypes.c_int64),
    ]
    lib.orc_generate_dense.restype = None
    lib.orc_generate_dense.argtypes = [
        ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
    ]
    lib.orc_solve_generated.restype = ctypes.c_int
    lib.orc_solve_generated.argtypes = [
        ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, P(OrcControl), ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, P(OrcStats),
    ]
    lib.orc_scale_factors.restype = None
    lib.orc_scale_factors.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p]
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.orc_generate_rows.restype = None
    lib.orc_generate_rows.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_void_p]
    _lib = lib
    return lib


@dataclass
class OracleResult:
    status: int
    objval: float
    x: np.ndarray
    y: np.ndarray
    basis: np.ndarray
    trace: np.ndarray
    stats: dict
    sens: dict | None = None


def _ptr(a):
    return None if a is None else a.ctypes.data


def solve_dense(A, dir, rhs, obj, lo=None, up=None, maximize=False, trace_cap=0, sens=False, **ctl):
    """sens=True: also the sensitivity report of the final basis (objfrom, objtill,
    duals, dualsfrom, dualstill; R/class.R:613-646) when the LP is optimal."""
    lib = load()
    obj = np.ascontiguousarray(obj, dtype=np.float64)
    n = obj.shape[0]
    rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(-1)
    m = rhs.shape[0]
    A = np.asfortranarray(np.asarray(A, dtype=np.float64).reshape(m, n))
    dir = np.ascontiguousarray(dir, dtype=np.int32).reshape(-1)
    lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
    up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
    c = OrcControl()
    lib.orc_default_control(ctypes.byref(c))
    for key, val in ctl.items():
        setattr(c, key, val)
    x = np.zeros(n)
    y = np.zeros(max(m, 1))
    basis = np.zeros(max(m, 1), dtype=np.int64)
    trace = np.full(2 * max(trace_cap, 1), -2, dtype=np.int64)
    objval = ctypes.c_double(0.0)
    st = OrcStats()
    sbuf = np.full(5 * n + 3 * m, np.nan) if sens else None
    status = lib.orc_solve_dense_sens(
        m, n, A.ctypes.data if m else None, _ptr(dir) if m else None, _ptr(rhs) if m else None,
        obj.ctypes.data, lo.ctypes.data, up.ctypes.data, int(bool(maximize)), ctypes.byref(c),
        ctypes.addressof(objval), x.ctypes.data, y.ctypes.data, basis.ctypes.data,
        trace.ctypes.data if trace_cap else None, trace_cap, ctypes.byref(st), _ptr(sbuf))
    if status < 0:
        raise ValueError(f"orc_solve_dense usage error {status}")
    stats = {f: getattr(st, f) for f, _ in OrcStats._fields_}
    it = min(stats["iterations"], trace_cap)
    sd = None
    if sens and status == 0:
        sd = {"objfrom": sbuf[:n], "objtill": sbuf[n:2 * n], "duals": sbuf[2 * n:2 * n + m + n],
              "dualsfrom": sbuf[3 * n + m:4 * n + 2 * m], "dualstill": sbuf[4 * n + 2 * m:]}
    return OracleResult(status, objval.value, x, y[:m], basis[:m],
                        trace[: 2 * it].reshape(-1, 2), stats, sd)


def generate_dense(seed, m, n, col0=0, ncols=None, want_A=True):
    lib = load()
    ncols = n - col0 if ncols is None else ncols
    A = np.zeros((m, ncols), dtype=np.float64, order="F") if want_A else None
    b = np.zeros(m)
    c = np.zeros(ncols)
    lib.orc_generate_dense(seed, m, n, col0, ncols, _ptr(A), b.ctypes.data, c.ctypes.data)
    return A, b, c


def solve_mip(A, dir, rhs, obj, lo, up, maximize, is_int, max_nodes=0, **ctl):
    """Branch and bound over the oracle's LP (rules: oracle/elp_oracle.c orc_solve_mip)."""
    lib = load()
    obj = np.ascontiguousarray(obj, dtype=np.float64)
    n = obj.shape[0]
    rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(-1)
    m = rhs.shape[0]
    A = np.asfortranarray(np.asarray(A, dtype=np.float64).reshape(m, n))
    dir = np.ascontiguousarray(dir, dtype=np.int32).reshape(-1)
    lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
    up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
    ii = np.ascontiguousarray(is_int, dtype=np.int32)
    c = OrcControl()
    lib.orc_default_control(ctypes.byref(c))
    for key, val in ctl.items():
        setattr(c, key, val)
    x = np.zeros(n)
    objval = ctypes.c_double(0.0)
    nodes, iters = ctypes.c_int64(0), ctypes.c_int64(0)
    status = lib.orc_solve_mip(m, n, A.ctypes.data if m else None, _ptr(dir) if m else None,
                               _ptr(rhs) if m else None, obj.ctypes.data, lo.ctypes.data,
                               up.ctypes.data, int(bool(maximize)), ii.ctypes.data, ctypes.byref(c),
                               int(max_nodes), ctypes.addressof(objval), x.ctypes.data,
                               ctypes.byref(nodes), ctypes.byref(iters))
    return OracleResult(status, objval.value, x, np.zeros(m), np.zeros(0, np.int64),
                        np.zeros((0, 2), np.int64), {"nodes": nodes.value, "lp_iterations": iters.value})


def solve_generated(seed, m, n, trace_cap=0, **ctl):
    """orc_solve_generated: the synthetic LP of generate_dense(seed, m, n) solved
    without materialising A (entries regenerated on read)."""
    lib = load()
    c = OrcControl()
    lib.orc_default_control(ctypes.byref(c))
    for key, val in ctl.items():
        setattr(c, key, val)
    x = np.zeros(n)
    y = np.zeros(max(m, 1))
    basis = np.zeros(max(m, 1), dtype=np.int64)
    trace = np.full(2 * max(trace_cap, 1), -2, dtype=np.int64)
    objval = ctypes.c_double(0.0)
    st = OrcStats()
    status = lib.orc_solve_generated(seed, m, n, ctypes.byref(c), ctypes.addressof(objval), x.ctypes.data,
                                     y.ctypes.data, basis.ctypes.data,
                                     trace.ctypes.data if trace_cap else None, trace_cap, ctypes.byref(st))
    if status < 0:
        raise ValueError(f"orc_solve_generated usage error {status}")
    stats = {f: getattr(st, f) for f, _ in OrcStats._fields_}
    it = min(stats["iterations"], trace_cap)
    return OracleResult(status, objval.value, x, y[:m], basis[:m], trace[: 2 * it].reshape(-1, 2), stats)


def generate_rows(seed, m, n, rows):
    """Rows `rows` of the generate_dense(seed, m, n) matrix, row-major."""
    lib = load()
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.zeros((len(rows), n))
    lib.orc_generate_rows(seed, m, n, rows.ctypes.data, len(rows), out.ctypes.data)
    return out


def scale_factors(A, mode=4 | 64):
    """(rho, gamma): the integer scaling exponents the solver applies to A."""
    lib = load()
    A = np.asfortranarray(np.asarray(A, dtype=np.float64))
    m, n = A.shape
    rho = np.zeros(max(m, 1), np.int32)
    gam = np.zeros(n, np.int32)
    lib.orc_scale_factors(m, n, A.ctypes.data, mode, rho.ctypes.data, gam.ctypes.data)
    return rho[:m], gam
