"""Pricing-launch timeline (diagnostic): solve the C3 LP with a library built with
-DELP_PDBG (tools/build_variant.sh pdbg -DELP_PDBG) and the device pricing timer,
dumping the per-workgroup stamps of one launch every ELP_PDBG_ITER iterations,
then summarise each dump.  Run on the GPU box:
    ELP_LIB_PATH=$PWD/easylp_amd/lib/libeasylp_hip_pdbg.so python tools/pdbg_run.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from easylp_amd import Problem, generate_dense_device  # noqa: E402

out = os.environ.setdefault("ELP_PDBG_FILE", "gpurun_out/pdbg.txt")
os.environ.setdefault("ELP_PDBG_ITER", "500")
if os.path.exists(out):
    os.remove(out)
m, n = 5000, 50000
A, b, c = generate_dense_device(1, m, n, 0)
with Problem(m, n, verbose=2) as p:  # ELP_PROFILE_PRICE
    p.load_dense_device(A.data_ptr(), np.ones(m, np.int32), b, c, maximize=True)
    st = p.solve()
    print("status", st, p.stats()["iterations"])


def pct(v, q):
    return float(np.percentile(v, q)) / 1e3 if len(v) else float("nan")


for block in open(out).read().split("# ")[1:]:
    lines = block.strip().split("\n")
    head = lines[0]
    rows = [l.split() for l in lines[1:]]
    tile = [r for r in rows if r[1] == "tile"]
    t0 = np.array([int(r[2]) for r in tile])
    t1 = np.array([int(r[3]) for r in tile])
    t2 = np.array([int(r[4]) for r in tile])
    t2a = np.array([int(r[5]) for r in tile])
    t2b = np.array([int(r[6]) for r in tile])
    t3 = np.array([int(r[7]) for r in tile])
    ap = np.array([int(r[7]) for r in rows if r[1] == "apply"])
    ap0 = np.array([int(r[2]) for r in rows if r[1] == "apply"])
    sl = np.array([int(r[7]) for r in rows if r[1] == "slack"])
    print(head)
    print("  tile start  p50 %.2f max %.2f | ctl in p50 %.2f max %.2f | sweep done p50 %.2f p90 %.2f max %.2f |"
          " end p50 %.2f max %.2f (us)" % (pct(t0, 50), pct(t0, 100), pct(t1, 50), pct(t1, 100), pct(t2, 50),
                                            pct(t2, 90), pct(t2, 100), pct(t3, 50), pct(t3, 100)))
    print("  all waves done - wave 0 p50 %.2f max %.2f | devex epilogue p50 %.2f max %.2f | argmin+store p50 %.2f max %.2f"
          % (pct(t2a - t2, 50), pct(t2a - t2, 100), pct(t2b - t2a, 50), pct(t2b - t2a, 100), pct(t3 - t2b, 50),
             pct(t3 - t2b, 100)))
    print("  sweep per tile (ctl in -> done) p50 %.2f max %.2f | apply n %d start max %.2f end p50 %.2f max %.2f |"
          " slack end max %.2f" % (pct(t2 - t1, 50), pct(t2 - t1, 100), len(ap), pct(ap0, 100), pct(ap, 50),
                                   pct(ap, 100), pct(sl, 100)))
