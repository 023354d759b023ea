"""cyingair MIP (test_gpu_dual.py's dense warm tree) through the pipeline with
ELP_DEBUG_REFACTOR: every refactor's residual on stderr (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("ELP_RESIDENT", "0")
from conftest import load_mip_known_answers
import easylp_amd as gpu
r = next(x for x in load_mip_known_answers() if x["name"] == "cyingair")
g = gpu.solve_dense(r["A"], r["dir"], r["rhs"], r["obj"], r["lo"], r["up"], r["maximize"], is_int=r["is_int"], simplex=6)
print(g.status, g.stats["mip_nodes"], g.stats["mip_lp_iterations"], g.objval, flush=True)
