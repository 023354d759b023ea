import json, os, sys, time
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
from easylp_amd import Problem
from easylp_amd.synth import sparse_kkt
fx = {f["name"]: f for f in json.load(open(os.path.join(ROOT, "tests", "golden", "sparse_lu.json")))}
for name in ("kkt_feasible_20000x100000", "kkt_20000x100000"):
    k = fx[name]
    cp, ri, v, b, c, u, obj = sparse_kkt(k["seed"], k["m"], k["n"], k["k"], feasible_start=k["feasible_start"])
    with Problem(k["m"], k["n"]) as p:
        p.load_csc(cp, ri, v, np.ones(k["m"], np.int32), b, c, np.zeros(k["n"]), u, maximize=True)
        st = p.solve()
        s = p.stats()
    print(name, st, {x: s[x] for x in ("iterations", "refactors", "gj_refactors", "max_inv_resid", "bump_dim")}, flush=True)
