"""Host-side mirror of EasyLP's solver hand-off, over the HIP C ABI.

`solve_dense()` takes exactly the arrays easylp$solve() hands to lp_solve at
/root/reference/R/class.R:260-274 (constraint$mat column-major, dir, rhs,
objective_fun, per-column bounds, sense) and returns what R reads back at
:276-298 (status code and string, objective, variables with 1e30 -> Inf).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import ElpStats, check, default_control, load

# R/class.R:279-295
STATUS_TEXT = {
    0: "optimal",
    1: "sub-optimal",
    2: "unfeasible",
    3: "unbounded",
    4: "degenerate model",
    5: "numerical failure encountered",
    6: "process aborted",
    7: "timeout",
    9: "the model was solved by presolve",
    10: "the branch and bound routine failed",
    11: "the branch and bound was stopped because of a break-at-first or break-at-value",
    12: "a feasible branch and bound solution was found",
    13: "no feasible branch and bound solution was found",
}

DIR_CODES = {"<=": 1, "<": 1, ">=": 2, ">": 2, "==": 3, "=": 3}


def status_text(code: int) -> str:
    return STATUS_TEXT.get(int(code), "undocumented status")


def large_to_infinity(x, threshold: float = 1e30):
    """R/utils.R:172-176."""
    x = np.array(x, dtype=np.float64, copy=True)
    x[x >= threshold] = np.inf
    x[x <= -threshold] = -np.inf
    return x


def dir_codes(dirs) -> np.ndarray:
    if len(dirs) and isinstance(dirs[0], str):
        bad = [d for d in dirs if d not in DIR_CODES]
        if bad:
            raise ValueError(f"unknown constraint direction {bad[0]!r}")
        return np.array([DIR_CODES[d] for d in dirs], dtype=np.int32)
    return np.ascontiguousarray(dirs, dtype=np.int32)


@dataclass
class Solution:
    status: int
    objval: float                 # raw objective (get.objective)
    x: np.ndarray                 # get.variables
    y: np.ndarray                 # duals, user sense
    basis: np.ndarray             # sorted basic variable ids
    stats: dict = field(default_factory=dict)
    trace: np.ndarray | None = None
    sens: dict | None = None      # sensitivity report (Problem.sensitivity)

    @property
    def status_text(self) -> str:
        return status_text(self.status)


class Problem:
    """One LP on the GPU (the object R keeps in self$pointer, R/class.R:300)."""

    def __init__(self, m: int, n: int, **control):
        self._lib = load()
        self.m, self.n = int(m), int(n)
        self._ctl = default_control(**control)
        h = ctypes.c_void_p()
        check(self._lib.elp_create(ctypes.byref(h), self.m, self.n, ctypes.byref(self._ctl)),
              "elp_create")
        self._h = h
        self._trace_cap = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.elp_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_trace(self, capacity: int) -> None:
        check(self._lib.elp_set_trace(self._h, int(capacity)), "elp_set_trace")
        self._trace_cap = int(capacity)

    def comm_init(self, unique_id: bytes, world_size: int, rank: int) -> None:
        """RCCL transport: one process per GPU (see easylp_amd.dist.share_unique_id)."""
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        check(self._lib.elp_comm_init(self._h, buf, int(world_size), int(rank)), "elp_comm_init")

    def comm_init_host(self, transport) -> None:
        """Host-callback transport (easylp_amd.dist.TorchDistTransport)."""
        self._transport = transport  # keeps the ctypes thunks alive
        check(self._lib.elp_comm_init_host(self._h, transport.world, transport.rank,
                                           transport.c_allgather, transport.c_allreduce,
                                           transport.c_bcast, None), "elp_comm_init_host")

    def comm_enable_p2p(self) -> None:
        """xGMI mailbox min-loc (no collective launch per iteration); after comm_init*."""
        check(self._lib.elp_comm_enable_p2p(self._h), "elp_comm_enable_p2p")

    def load_dense(self, A, dirs, rhs, obj, lo=None, up=None, maximize=False) -> None:
        m, n = self.m, self.n
        A = np.asfortranarray(np.asarray(A, dtype=np.float64).reshape(m, n))
        d = dir_codes(dirs)
        rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(m)
        obj = np.ascontiguousarray(obj, dtype=np.float64).reshape(n)
        lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
        up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
        self._keep = (A, d, rhs, obj, lo, up)
        check(self._lib.elp_load_dense(
            self._h, A.ctypes.data if m else None, d.ctypes.data if m else None,
            rhs.ctypes.data if m else None, obj.ctypes.data, lo.ctypes.data, up.ctypes.data,
            int(bool(maximize))), "elp_load_dense")

    def load_dense_device(self, dA_ptr: int, dirs, rhs, obj, lo=None, up=None, maximize=False):
        m, n = self.m, self.n
        d = dir_codes(dirs)
        rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(m)
        obj = np.ascontiguousarray(obj, dtype=np.float64).reshape(n)
        lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
        up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
        self._keep = (d, rhs, obj, lo, up)
        check(self._lib.elp_load_dense_device(
            self._h, ctypes.c_void_p(int(dA_ptr)), d.ctypes.data, rhs.ctypes.data, obj.ctypes.data,
            lo.ctypes.data, up.ctypes.data, int(bool(maximize))), "elp_load_dense_device")

    def load_dense_device_multi(self, dA_ptrs, dirs, rhs, obj, lo=None, up=None, maximize=False):
        """ngpu handle, A resident on every device: dA_ptrs[r] is A (m*n float64,
        column-major) on rank r's device (device + r); each rank reads its own copy
        (elp_load_dense_device_multi)."""
        m, n = self.m, self.n
        d = dir_codes(dirs)
        rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(m)
        obj = np.ascontiguousarray(obj, dtype=np.float64).reshape(n)
        lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
        up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
        ptrs = (ctypes.c_void_p * len(dA_ptrs))(*[int(p) for p in dA_ptrs])
        self._keep = (d, rhs, obj, lo, up, ptrs)
        check(self._lib.elp_load_dense_device_multi(
            self._h, ptrs, len(dA_ptrs), d.ctypes.data, rhs.ctypes.data, obj.ctypes.data,
            lo.ctypes.data, up.ctypes.data, int(bool(maximize))), "elp_load_dense_device_multi")

    def load_csc(self, colptr, rowind, val, dirs, rhs, obj, lo=None, up=None, maximize=False) -> None:
        """Sparse A in compressed sparse columns (rows strictly increasing per column)."""
        m, n = self.m, self.n
        colptr = np.ascontiguousarray(colptr, dtype=np.int64).reshape(n + 1)
        rowind = np.ascontiguousarray(rowind, dtype=np.int32).reshape(-1)
        val = np.ascontiguousarray(val, dtype=np.float64).reshape(-1)
        d = dir_codes(dirs)
        rhs = np.ascontiguousarray(rhs, dtype=np.float64).reshape(m)
        obj = np.ascontiguousarray(obj, dtype=np.float64).reshape(n)
        lo = np.zeros(n) if lo is None else np.ascontiguousarray(lo, dtype=np.float64)
        up = np.full(n, np.inf) if up is None else np.ascontiguousarray(up, dtype=np.float64)
        self._keep = (colptr, rowind, val, d, rhs, obj, lo, up)
        check(self._lib.elp_load_csc(
            self._h, colptr.ctypes.data, rowind.ctypes.data if rowind.size else None,
            val.ctypes.data if val.size else None, d.ctypes.data if m else None,
            rhs.ctypes.data if m else None, obj.ctypes.data, lo.ctypes.data, up.ctypes.data,
            int(bool(maximize))), "elp_load_csc")

    def set_int(self, is_int) -> None:
        """set.type(..., "integer" | "binary") (R/class.R:265): integer columns;
        elp_solve then runs branch and bound over GPU LP relaxations."""
        if is_int is None:
            check(self._lib.elp_set_int(self._h, None), "elp_set_int")
            return
        ii = np.ascontiguousarray(is_int, dtype=np.int32).reshape(self.n)
        self._keep_int = ii
        check(self._lib.elp_set_int(self._h, ii.ctypes.data), "elp_set_int")

    def load_generated(self, seed: int) -> None:
        check(self._lib.elp_load_generated(self._h, int(seed)), "elp_load_generated")

    def solve(self) -> int:
        st = ctypes.c_int32(-1)
        check(self._lib.elp_solve(self._h, ctypes.byref(st)), "elp_solve")
        return st.value

    def iterate(self, iters: int) -> int:
        st = ctypes.c_int32(-1)
        check(self._lib.elp_iterate(self._h, int(iters), ctypes.byref(st)), "elp_iterate")
        return st.value

    def stats(self) -> dict:
        s = ElpStats()
        check(self._lib.elp_get_stats(self._h, ctypes.byref(s)), "elp_get_stats")
        return {f: getattr(s, f) for f, _ in ElpStats._fields_}

    def trace(self) -> np.ndarray:
        cap = self._trace_cap
        buf = np.zeros(2 * max(cap, 1), dtype=np.int64)
        cnt = ctypes.c_int64(0)
        check(self._lib.elp_get_trace(self._h, buf.ctypes.data, cap, ctypes.byref(cnt)),
              "elp_get_trace")
        return buf[: 2 * cnt.value].reshape(-1, 2)

    def sensitivity(self) -> dict:
        """get.sensitivity.obj + get.sensitivity.rhs of the final basis
        (R/class.R:613-646): objfrom/objtill (n), duals/dualsfrom/dualstill (m+n),
        infinite limits as +-1e30 (apply large_to_infinity as R/class.R does)."""
        m, n = self.m, self.n
        out = {k: np.zeros(n) for k in ("objfrom", "objtill")}
        out.update({k: np.zeros(m + n) for k in ("duals", "dualsfrom", "dualstill")})
        check(self._lib.elp_sensitivity(self._h, *(out[k].ctypes.data for k in (
            "objfrom", "objtill", "duals", "dualsfrom", "dualstill"))), "elp_sensitivity")
        return out

    def solution(self, status: int) -> Solution:
        m, n = self.m, self.n
        x = np.zeros(n)
        y = np.zeros(max(m, 1))
        basis = np.zeros(max(m, 1), dtype=np.int64)
        obj = ctypes.c_double(0.0)
        check(self._lib.elp_get_solution(self._h, ctypes.byref(obj), x.ctypes.data,
                                         y.ctypes.data, basis.ctypes.data), "elp_get_solution")
        tr = self.trace() if self._trace_cap else None
        return Solution(status, obj.value, x, y[:m], basis[:m], self.stats(), tr)


def generate_dense_device(seed: int, m: int, n: int, device: int = 0):
    """The synthetic LP of SURVEY.md 8d (maximize c'x, A x <= b, x >= 0) with A
    generated straight into HBM (elp_generate_dense): returns (A, b, c), A a
    torch float64 tensor of m*n elements on cuda:device (column-major, lda = m),
    b and c numpy arrays.  Pass A.data_ptr() to Problem.load_dense_device."""
    import torch
    lib = load()
    A = torch.empty(max(m * n, 1), dtype=torch.float64, device=f"cuda:{device}")
    b = np.zeros(max(m, 1))
    c = np.zeros(n)
    torch.cuda.synchronize(device)
    check(lib.elp_generate_dense(int(device), int(seed), int(m), int(n), ctypes.c_void_p(A.data_ptr()),
                                 b.ctypes.data, c.ctypes.data), "elp_generate_dense")
    return A, b[:m], c


def csc_arrays(A):
    """(colptr, rowind, val) of a scipy.sparse matrix or dense array: canonical
    CSC (duplicates summed, rows sorted), explicit zeros kept."""
    import scipy.sparse as sp
    M = sp.csc_matrix(A, dtype=np.float64)
    M.sum_duplicates()
    M.sort_indices()
    return (M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data.astype(np.float64),
            M.shape)


def solve_sparse(A, dirs, rhs, obj, lo=None, up=None, maximize=False, trace=0, sensitivity=False,
                 is_int=None, **control) -> Solution:
    """One-shot solve with A sparse (scipy.sparse or dense array) through the CSC path."""
    colptr, rowind, val, (m, n) = csc_arrays(A)
    with Problem(m, n, **control) as p:
        if trace:
            p.set_trace(trace)
        p.load_csc(colptr, rowind, val, dirs, rhs, obj, lo, up, maximize)
        if is_int is not None:
            p.set_int(is_int)
        st = p.solve()
        sol = p.solution(st)
        if sensitivity and st == 0:
            sol.sens = p.sensitivity()
        return sol


def solve_dense(A, dirs, rhs, obj, lo=None, up=None, maximize=False, trace=0, sensitivity=False,
                is_int=None, **control) -> Solution:
    """One-shot solve of a dense LP on the GPU (the R/class.R:260-278 hand-off).
    sensitivity=True adds Solution.sens (Problem.sensitivity()) when optimal;
    is_int (n flags) makes it a MIP solved by branch and bound."""
    m = len(rhs)
    n = len(obj)
    with Problem(m, n, **control) as p:
        if trace:
            p.set_trace(trace)
        p.load_dense(A, dirs, rhs, obj, lo, up, maximize)
        if is_int is not None:
            p.set_int(is_int)
        st = p.solve()
        sol = p.solution(st)
        if sensitivity and st == 0:
            sol.sens = p.sensitivity()
        return sol
