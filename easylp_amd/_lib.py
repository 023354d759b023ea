"""ctypes binding of include/easylp_hip.h (the C ABI of libeasylp_hip.so).

The product path has no fallback: if the HIP library is missing or no GPU is
visible, calls raise.  Nothing here imports or calls oracle/.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ELP_LIB_PATH") or os.path.join(HERE, "lib", "libeasylp_hip.so")

ELP_LE, ELP_GE, ELP_EQ = 1, 2, 3
ELP_OPTIMAL, ELP_SUBOPTIMAL, ELP_INFEASIBLE, ELP_UNBOUNDED = 0, 1, 2, 3
ELP_NUMFAILURE, ELP_TIMEOUT = 5, 7
ELP_PROFILE_PRICE = 2   # device-clock pricing timer
ELP_PROFILE_EVENTS = 4  # HIP events on every pricing dispatch
ELP_PROFILE_SAMPLE = 8  # ... on those of every 8th chunk between host polls
ELP_SCALE_GEOMETRIC, ELP_SCALE_EQUILIBRATE = 4, 64
ELP_BASIS_AUTO, ELP_BASIS_INVERSE, ELP_BASIS_LU = 0, 1, 2
ABI_VERSION = 7
ELP_SIMPLEX_PRIMAL_PRIMAL, ELP_SIMPLEX_DUAL_PRIMAL = 5, 6

# every entry point the header declares (checked by tests/test_abi.py)
EXPORTS = (
    "elp_default_control", "elp_create", "elp_load_dense", "elp_load_dense_device", "elp_load_dense_device_multi",
    "elp_load_generated", "elp_generate_dense", "elp_load_csc", "elp_set_int", "elp_solve", "elp_iterate", "elp_get_solution",
    "elp_get_stats", "elp_sensitivity",
    "elp_set_trace", "elp_get_trace", "elp_comm_unique_id", "elp_comm_init", "elp_comm_init_host", "elp_comm_enable_p2p",
    "elp_destroy", "elp_last_error", "elp_abi_version",
)

# host transports for elp_comm_init_host (include/easylp_hip.h)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
                                ctypes.c_void_p)
BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
                            ctypes.c_void_p)


class ElpControl(ctypes.Structure):
    _fields_ = [
        ("tol_primal", ctypes.c_double),
        ("tol_dual", ctypes.c_double),
        ("tol_pivot", ctypes.c_double),
        ("infinity", ctypes.c_double),
        ("time_limit", ctypes.c_double),
        ("max_iter", ctypes.c_int64),
        ("refactor_period", ctypes.c_int32),
        ("degen_switch", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("sync_every", ctypes.c_int32),
        ("verbose", ctypes.c_int32),
        ("refactor_mode", ctypes.c_int32),
        ("replicate", ctypes.c_int32),
        ("max_nodes", ctypes.c_int32),
        ("pricing", ctypes.c_int32),
        ("ngpu", ctypes.c_int32),
        ("scaling", ctypes.c_int32),
        ("exchange", ctypes.c_int32),
        ("tol_singular", ctypes.c_double),
        ("mailbox_timeout", ctypes.c_double),
        ("basis", ctypes.c_int32),
        ("simplex", ctypes.c_int32),
        ("resident", ctypes.c_int32),
        ("pad_resident", ctypes.c_int32),
    ]


class ElpStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int64),
        ("phase1_iterations", ctypes.c_int64),
        ("bound_flips", ctypes.c_int64),
        ("degenerate", ctypes.c_int64),
        ("refactors", ctypes.c_int64),
        ("bump_dim", ctypes.c_int64),
        ("y_rows", ctypes.c_int64),
        ("host_polls", ctypes.c_int64),
        ("seconds_total", ctypes.c_double),
        ("seconds_loop", ctypes.c_double),
        ("seconds_load", ctypes.c_double),
        ("price_bytes", ctypes.c_double),
        ("world_size", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("col0", ctypes.c_int64),
        ("ncols", ctypes.c_int64),
        ("price_seconds", ctypes.c_double),
        ("price_timed_bytes", ctypes.c_double),
        ("price_timed_launches", ctypes.c_int64),
        ("gj_refactors", ctypes.c_int64),
        ("mip_nodes", ctypes.c_int64),
        ("mip_lp_iterations", ctypes.c_int64),
        ("price_launches", ctypes.c_int64),
        ("max_inv_resid", ctypes.c_double),
        ("iter_bytes", ctypes.c_double),
        ("exchange", ctypes.c_int32),
        ("resident", ctypes.c_int32),
        ("seconds_h2d", ctypes.c_double),
        ("h2d_bytes", ctypes.c_double),
        ("resident_launches", ctypes.c_int64),
        ("resident_ticks", ctypes.c_int64),
        ("basis", ctypes.c_int32),
        ("simplex", ctypes.c_int32),
        ("exchange_rtt_us", ctypes.c_double),
        ("dual_iterations", ctypes.c_int64),
        ("price_seconds_stamps", ctypes.c_double),
        ("price_stamped_launches", ctypes.c_int64),
    ]


class ElpError(RuntimeError):
    pass


_lib = None


def hip_runtime_files() -> list[str]:
    """The HIP / HSA runtime files mapped into this process (/proc/self/maps)."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if "libamdhip64" in p or "libhsa-runtime64" in p:
                    out.add(p)
    except OSError:
        pass
    return sorted(out)


def _one_runtime() -> None:
    """One HIP runtime per process.  torch bundles its own ROCm (7.0) under the
    same SONAMEs the library needs (libamdhip64.so.7, libhsa-runtime64.so.1); if
    the library loaded first it would start /opt/rocm's runtime and a later
    torch would start a second HSA runtime beside it -- the r02 `elp_create:
    hipSetDevice failed` (tools/runtime_probe.py: lib_first).  Sharing
    /opt/rocm's runtime with torch works but aborts at exit (preload_all).  So a
    Python process that has torch binds the library to torch's runtime: torch
    is imported first (no device call), and the library's NEEDED entries then
    resolve to the runtime already loaded.  Processes without torch (R, the C
    driver, ELP_NO_TORCH=1) use /opt/rocm's runtime through the RUNPATH."""
    if os.environ.get("ELP_NO_TORCH"):
        return
    if any("libamdhip64" in p for p in hip_runtime_files()):
        return  # a runtime is already there: bind to it
    try:
        import torch  # noqa: F401
    except Exception:  # (absent, or its bundled ROCm libraries failed: /opt/rocm's runtime then)
        pass


def load(path: str | None = None):
    """Load the HIP library; raises (loudly) if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise ElpError(f"{path} not built: run `python -m easylp_amd.build` (no CPU fallback)")
    _one_runtime()
    lib = ctypes.CDLL(path)
    P, vp = ctypes.POINTER, ctypes.c_void_p
    i64, i32, dbl = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
    lib.elp_default_control.argtypes = [P(ElpControl)]
    lib.elp_default_control.restype = None
    lib.elp_create.argtypes = [P(vp), i64, i64, P(ElpControl)]
    lib.elp_load_dense.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32]
    lib.elp_load_dense_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32]
    lib.elp_load_dense_device_multi.argtypes = [vp, P(vp), i32, vp, vp, vp, vp, vp, i32]
    lib.elp_load_generated.argtypes = [vp, ctypes.c_uint64]
    lib.elp_generate_dense.argtypes = [i32, ctypes.c_uint64, i64, i64, vp, vp, vp]
    lib.elp_load_csc.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
    lib.elp_set_int.argtypes = [vp, vp]
    lib.elp_solve.argtypes = [vp, P(i32)]
    lib.elp_iterate.argtypes = [vp, i64, P(i32)]
    lib.elp_get_solution.argtypes = [vp, P(dbl), vp, vp, vp]
    lib.elp_get_stats.argtypes = [vp, P(ElpStats)]
    lib.elp_sensitivity.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.elp_set_trace.argtypes = [vp, i64]
    lib.elp_get_trace.argtypes = [vp, vp, i64, P(i64)]
    lib.elp_comm_unique_id.argtypes = [vp]
    lib.elp_comm_init.argtypes = [vp, vp, i32, i32]
    lib.elp_comm_init_host.argtypes = [vp, i32, i32, ALLGATHER_FN, ALLREDUCE_FN, BCAST_FN, vp]
    lib.elp_comm_enable_p2p.argtypes = [vp]
    lib.elp_destroy.argtypes = [vp]
    lib.elp_destroy.restype = None
    lib.elp_last_error.restype = ctypes.c_char_p
    lib.elp_abi_version.restype = i32
    for name in ("elp_create", "elp_load_dense", "elp_load_dense_device", "elp_load_dense_device_multi",
                 "elp_load_generated",
                 "elp_generate_dense",
                 "elp_load_csc", "elp_sensitivity", "elp_set_int",
                 "elp_solve", "elp_iterate", "elp_get_solution", "elp_get_stats",
                 "elp_set_trace", "elp_get_trace", "elp_comm_unique_id", "elp_comm_init",
                 "elp_comm_init_host", "elp_comm_enable_p2p"):
        getattr(lib, name).restype = ctypes.c_int
    if lib.elp_abi_version() != ABI_VERSION:  # (struct layouts would disagree)
        raise ElpError(f"{path} has ABI {lib.elp_abi_version()}, this binding expects {ABI_VERSION}: "
                       "rebuild it with `python -m easylp_amd.build`")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc < 0:
        msg = _lib.elp_last_error().decode(errors="replace") if _lib else ""
        raise ElpError(f"{what} failed ({rc}): {msg}")


def default_control(**overrides) -> ElpControl:
    lib = load()
    c = ElpControl()
    lib.elp_default_control(ctypes.byref(c))
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise KeyError(f"unknown control field {k!r}")
        setattr(c, k, v)
    return c
