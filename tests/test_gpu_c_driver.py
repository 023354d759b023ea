"""The library as the R `.Call` shim loads it: a plain C
caller (tests/c_driver/elp_driver.c, built here with gcc against
include/easylp_hip.h) in a fresh child process -- no Python, no torch, so the
library binds /opt/rocm's HIP runtime through its RUNPATH -- solving from A in
host memory (elp_load_dense), on one device and with ngpu = 2 (one process, two
rank handles).  Results must equal the CPU oracle's (status, basis and pivot
trace bit for bit, objective to 1e-9 relative) and the committed fixtures.

Also the Python binding's runtime rule (easylp_amd._lib._one_runtime): loading
the library before torch must not break torch or a later elp_create, and a
torch-free Python process (ELP_NO_TORCH=1) runs on /opt/rocm's runtime.
Reference seam: R/class.R:260-278."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_dense_lps, load_known_answers

pytestmark = pytest.mark.gpu

LIBDIR = os.path.join(ROOT, "easylp_amd", "lib")
SRC = os.path.join(ROOT, "tests", "c_driver", "elp_driver.c")
CAP = 200000


def _driver(tmp_path):
    from easylp_amd import build
    build.build()
    exe = tmp_path / "elp_driver"
    subprocess.run(["gcc", "-O2", "-o", str(exe), SRC, f"-L{LIBDIR}", "-leasylp_hip",
                    f"-Wl,-rpath,{LIBDIR}", "-lm"], check=True)
    return str(exe)


def _fmt(v):
    return "inf" if v == np.inf else "-inf" if v == -np.inf else repr(float(v))


def _write(path, lps):
    with open(path, "w") as f:
        f.write(f"{len(lps)}\n")
        for A, dirs, rhs, obj, lo, up, mx in lps:
            m, n = A.shape
            f.write(f"{m} {n} {int(bool(mx))}\n")
            f.write(" ".join(_fmt(v) for v in np.asarray(A, dtype=np.float64).ravel(order="F")) + "\n")
            for vec in (dirs, rhs, obj, lo, up):
                f.write(" ".join(_fmt(v) for v in np.asarray(vec, dtype=np.float64)) + "\n")


def _run(exe, inp, *args, env=None):
    r = subprocess.run([exe, inp, *map(str, args)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out, cur = [], None
    runtime = None
    for line in r.stdout.splitlines():
        t = line.split()
        if t[0] == "lp":
            cur = {"rc": int(t[3]), "status": int(t[5]), "objval": float(t[7]), "iterations": int(t[9]),
                   "exchange": int(t[11])}
            out.append(cur)
        elif t[0] == "x":
            cur["x"] = np.array([float(v) for v in t[1:]])
        elif t[0] == "basis":
            cur["basis"] = np.array([int(v) for v in t[1:]], dtype=np.int64)
        elif t[0] == "trace":
            cur["trace"] = np.array([int(v) for v in t[2:]], dtype=np.int64).reshape(-1, 2)
        elif t[0] == "runtime":
            runtime = t[1]
    return out, runtime


def _cases():
    known = {r["name"]: r for r in load_known_answers()}
    lps = []
    for name in ("readme", "dop", "unbounded"):
        r = known[name]
        lps.append(((r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"]), r["expected"], name))
    from oracle import generate_dense
    rec = next(d for d in load_dense_lps() if d["m"] == 500 and d["n"] == 2000)
    A, b, c = generate_dense(rec["seed"], rec["m"], rec["n"])
    m, n = A.shape
    lps.append(((A, np.ones(m, np.int32), b, c, np.zeros(n), np.full(n, np.inf), True), rec, "dense_500x2000"))
    return lps


def _check(g, lp, exp, name):
    from oracle import solve_dense as orc
    A, dirs, rhs, obj, lo, up, mx = lp
    o = orc(A, dirs, rhs, obj, lo, up, mx, trace_cap=CAP)
    assert g["rc"] == 0 and g["status"] == o.status, (name, g["status"], o.status)
    np.testing.assert_array_equal(g["trace"], o.trace)
    if o.status == 0:
        np.testing.assert_array_equal(g["basis"], o.basis)
        assert abs(g["objval"] - o.objval) <= 1e-9 * max(1.0, abs(o.objval))
        np.testing.assert_allclose(g["x"], o.x, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(o.x).max()))
    if "objective" in exp:  # the reference's own answers / the HiGHS fixture
        assert abs(g["objval"] - exp["objective"]) <= 1e-9 * max(1.0, abs(exp["objective"])), name
    if "basis" in exp:
        np.testing.assert_array_equal(g["basis"], np.array(exp["basis"], dtype=np.int64))
    if g["status"] == 3:  # test-unbounded.R:8-9: objective +-Inf through large_to_infinity
        assert abs(g["objval"]) == 1e30


@pytest.mark.parametrize("ngpu", [1, 2])
def test_c_driver_host_input_matches_oracle(tmp_path, ngpu):
    exe = _driver(tmp_path)
    cases = _cases()
    inp = str(tmp_path / "lps.txt")
    _write(inp, [c[0] for c in cases])
    out, runtime = _run(exe, inp, "ngpu", ngpu, "trace", CAP)
    # the R path's runtime: /opt/rocm's, not torch's bundled copy
    assert runtime and "torch" not in runtime and "libamdhip64.so.7" in runtime, runtime
    assert len(out) == len(cases)
    for g, (lp, exp, name) in zip(out, cases):
        _check(g, lp, exp, name)
        if ngpu > 1 and lp[0].shape[1] >= 2:  # (n = 1: the driver runs one rank)
            assert g["exchange"] in (1, 2)


_CHILD_LIB_FIRST = r"""
import numpy as np
import easylp_amd
from easylp_amd._lib import load, hip_runtime_files
load()                      # the library before torch
import torch
torch.cuda.init()
t = float(torch.ones(8, device="cuda", dtype=torch.float64).sum().item())
g = easylp_amd.solve_dense(np.array([[1.0, 2.0], [-3.0, 1.0]]), [1, 2], [3.0, -2.0], [1.0, 1.0],
                           [-np.inf, -np.inf], [np.inf, np.inf], True)
print("RESULT", g.status, repr(g.objval), t, ";".join(hip_runtime_files()))
"""

_CHILD_NO_TORCH = r"""
import json, sys
import numpy as np
sys.path.insert(0, %(root)r)
sys.path.insert(0, %(tests)r)
import easylp_amd
from easylp_amd._lib import load, hip_runtime_files
from conftest import load_known_answers
load()
out = []
for r in load_known_answers():
    g = easylp_amd.solve_dense(r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"], trace=100000)
    out.append({"name": r["name"], "status": g.status, "objval": g.objval, "basis": g.basis.tolist(),
                "trace": g.trace.tolist(), "x": g.x.tolist()})
print("RESULT", json.dumps({"runs": out, "runtime": hip_runtime_files(), "torch": "torch" in sys.modules}))
"""


def _child(code, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = next(l for l in r.stdout.splitlines() if l.startswith("RESULT"))
    return line[len("RESULT "):]


def test_library_loaded_before_torch():
    """r02's gpurun_out/abi_fail.log: elp_create failed when the library was
    loaded before torch (two HIP runtimes in one process).  The binding now
    binds to torch's runtime when torch is installed; both work afterwards."""
    st, obj, t, rt = _child(_CHILD_LIB_FIRST).split(" ", 3)
    assert int(st) == 0 and float(obj) == 2.0 and float(t) == 8.0
    libs = rt.split(";")
    assert sum("libamdhip64" in p for p in libs) == 1, libs  # one runtime


def test_torch_free_python_runs_on_system_runtime():
    """The known-answer LPs from a Python process without torch (ELP_NO_TORCH=1):
    /opt/rocm's runtime, results bit-identical to the oracle's."""
    from conftest import load_known_answers
    from oracle import solve_dense as orc
    res = json.loads(_child(_CHILD_NO_TORCH % {"root": ROOT, "tests": os.path.join(ROOT, "tests")},
                            {"ELP_NO_TORCH": "1"}))
    assert not res["torch"]
    assert res["runtime"] and all("torch" not in p for p in res["runtime"]), res["runtime"]
    known = {r["name"]: r for r in load_known_answers()}
    for g in res["runs"]:
        r = known[g["name"]]
        o = orc(r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"], trace_cap=100000)
        assert g["status"] == o.status, g["name"]
        np.testing.assert_array_equal(np.array(g["trace"], dtype=np.int64).reshape(-1, 2), o.trace)
        if o.status == 0:
            np.testing.assert_array_equal(g["basis"], o.basis)
            assert abs(g["objval"] - o.objval) <= 1e-12 * max(1.0, abs(o.objval))
