"""One resident Klee-Minty n=12 solve (Dantzig, unscaled) -- for counter passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch
    torch.cuda.init()
    from easylp_amd import Problem
    from make_sparse import klee_minty
    A, dirs, rhs, obj, lo, up, mx = klee_minty(12)
    for _ in range(2):
        with Problem(12, 12, pricing=0, scaling=0, resident=1) as p:
            p.load_dense(A.toarray(), dirs, rhs, obj, lo, up, mx)
            st = p.solve()
            s = p.stats()
    print(st, s["iterations"], s["resident_ticks"] / 100.0, "us")


if __name__ == "__main__":
    main()
