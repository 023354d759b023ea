"""C4 load-phase probe (diagnostic): load the 10000 x 500000 LP from HBM three
times (ELP_DEBUG_LOAD phase timers on stderr), fresh handle and reload.
    ELP_DEBUG_LOAD=1 python tools/c4_load_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from easylp_amd import Problem, generate_dense_device  # noqa: E402

m, n = 10000, 500000
A, b, c = generate_dense_device(1, m, n, 0)
torch.cuda.synchronize()
for trial in range(2):
    with Problem(m, n) as p:
        for rep in range(2):
            t = time.perf_counter()
            p.load_dense_device(A.data_ptr(), np.ones(m, np.int32), b, c, maximize=True)
            torch.cuda.synchronize()
            print("trial", trial, "load", rep, round(time.perf_counter() - t, 3), flush=True)
