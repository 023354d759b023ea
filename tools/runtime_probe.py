"""Which HIP runtime does libeasylp_hip.so bind to, and does loading it before
torch break either side?  Modes (one per child process):
  lib_first      ctypes.CDLL(lib) (RTLD_LOCAL), then torch     -- the r02 failure
  preload_first  system ROCm preloaded under the bare names (RTLD_GLOBAL), lib,
                 then torch (torch then shares /opt/rocm's runtime)
  torch_first    torch initialised, then the lib (torch's bundled runtime)
  no_torch       the lib alone (what an R process does)
Each prints the libamdhip64 / libhsa-runtime64 files mapped and the result of
elp_create + a 2x2 solve (and a torch op where torch is loaded)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "easylp_amd", "lib", "libeasylp_hip.so")


def mapped():
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if any(k in p for k in ("libamdhip64", "libhsa-runtime64", "librccl", "libamd_comgr")):
                out.add(p)
    return sorted(out)


def solve(lib):
    h = ctypes.c_void_p()
    rc = lib.elp_create(ctypes.byref(h), ctypes.c_int64(2), ctypes.c_int64(2), None)
    if rc:
        lib.elp_last_error.restype = ctypes.c_char_p
        return "elp_create rc=%d %s" % (rc, lib.elp_last_error())
    A = (ctypes.c_double * 4)(1.0, -3.0, 2.0, 1.0)  # column-major [[1,2],[-3,1]]
    d = (ctypes.c_int32 * 2)(1, 2)
    rhs = (ctypes.c_double * 2)(3.0, -2.0)
    obj = (ctypes.c_double * 2)(1.0, 1.0)
    lo = (ctypes.c_double * 2)(-1e30, -1e30)
    up = (ctypes.c_double * 2)(1e30, 1e30)
    rc = lib.elp_load_dense(h, A, d, rhs, obj, lo, up, 1)
    st = ctypes.c_int32(-9)
    rc2 = lib.elp_solve(h, ctypes.byref(st)) if rc == 0 else None
    z = ctypes.c_double(0)
    lib.elp_get_solution(h, ctypes.byref(z), None, None, None)
    lib.elp_destroy(h)
    return "load rc=%s solve rc=%s status=%d objective=%r" % (rc, rc2, st.value, z.value)


def main(mode):
    res = {}
    if mode == "preload_first":
        for nm in ("libhsa-runtime64.so", "libamdhip64.so", "librccl.so"):
            ctypes.CDLL(nm, mode=ctypes.RTLD_GLOBAL)
    if mode == "preload_all":
        for nm in ("librocprofiler-register.so", "libhsa-runtime64.so", "libamd_comgr.so", "libamdhip64.so",
                   "libhiprtc.so", "librocm_smi64.so", "libroctx64.so", "librccl.so"):
            ctypes.CDLL(nm, mode=ctypes.RTLD_GLOBAL)
    if mode == "import_torch_first":
        import torch  # noqa: F401  (no device call yet)
    lib = None
    if mode in ("lib_first", "preload_first", "preload_all", "no_torch", "import_torch_first"):
        lib = ctypes.CDLL(LIB)
    if mode != "no_torch":
        import torch
        ok = torch.cuda.is_available()
        t = torch.arange(10, device="cuda", dtype=torch.float64) if ok else None
        res["torch"] = "available=%s sum=%s hip=%s" % (ok, None if t is None else float((t @ t).item()), torch.version.hip)
    if lib is None:
        lib = ctypes.CDLL(LIB)
    res["elp"] = solve(lib)
    if mode != "no_torch":
        import torch
        res["torch_after"] = float(torch.ones(4, device="cuda").sum().item())
    res["mapped"] = mapped()
    print(mode, res, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main(sys.argv[1])
    else:
        import subprocess
        for m in ("no_torch", "torch_first", "lib_first", "preload_first", "preload_all", "import_torch_first"):
            r = subprocess.run([sys.executable, __file__, m], capture_output=True, text=True, timeout=300)
            print("==", m, "rc", r.returncode)
            print(r.stdout.strip())
            if r.returncode:
                print(r.stderr.strip()[-2000:])
