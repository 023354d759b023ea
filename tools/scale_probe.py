import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, numpy as np, torch
torch.cuda.init()
from easylp_amd import Problem, generate_dense_device
for (m, n) in [(5000, 50000), (10000, 500000)]:
    A, b, c = generate_dense_device(1, m, n, 0)
    for sc in (0, 68, 4, 64):
        with Problem(m, n, scaling=sc) as p:
            t = time.perf_counter()
            p.load_dense_device(A.data_ptr(), np.ones(m, np.int32), b, c, maximize=True)
            torch.cuda.synchronize()
            print(m, n, sc, "load", round(time.perf_counter() - t, 4), p.stats()["seconds_load"], flush=True)
    del A
    torch.cuda.empty_cache()
