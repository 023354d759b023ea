"""The CSC path's row-wise FTRAN-z (k_ftran_zr_sp, with the dual flip update:
A[i, S] v from the rows' nonzeros in bump-position order, the oracle's zchunk
grouping).  The library switches to it once the dense walk over AS would stream
more than ELP_SPZ_MIN_MB; the fixtures here are far below that, so the CSC
parity tests run again in a child process with the threshold at 0 (every CSC
iteration takes the row-wise kernels) -- every trace must still be the
oracle's bit for bit: the sparse fixtures, the known answers, Klee-Minty, the
larger sparse LPs, the fuzz LPs, the dual phase with bound flips and the MIP
trees."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_csc_parity_with_rowwise_ftran():
    env = dict(os.environ, ELP_RESIDENT="0", ELP_SPZ_MIN_MB="0")
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
           os.path.join(HERE, "test_gpu_csc.py"),
           os.path.join(HERE, "test_gpu_dual.py") + "::test_dual_known_and_robust",
           os.path.join(HERE, "test_gpu_dual.py") + "::test_dual_fuzz",
           os.path.join(HERE, "test_gpu_dual.py") + "::test_dual_sparse_fixtures",
           os.path.join(HERE, "test_gpu_dual.py") + "::test_dual_kkt_2000x10000_matches_oracle",
           os.path.join(HERE, "test_gpu_fuzz.py") + "::test_fuzz_csc",
           os.path.join(HERE, "test_gpu_fuzz.py") + "::test_fuzz_mip",
           os.path.join(HERE, "test_gpu_mip.py") + "::test_reference_mips_gpu",
           "-k", "not dense"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=os.path.dirname(HERE))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert " passed" in r.stdout
