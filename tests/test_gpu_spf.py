"""The CSC path's hypersparse products against the bump inverse (DESIGN.md 9,
"sparse FTRAN"): alpha_S = Minv a_R and fS = Minv a_F[R] in the select kernel,
rho_r = A[i, S] Minv in k_dual_row, from lane-bucketed lists of the operand's
nonzeros (sparse_lane_chain: each lane's chain of the dense wave_dot over the
nonzero terms only).  The library takes them once the bump exceeds
ELP_SPF_MIN (512) positions; the fixtures here are far smaller, so the CSC
parity tests run again in a child process with the threshold at 1 (every CSC
iteration with k > 1 takes the sparse kernels) and the row-wise FTRAN-z forced
(so the dual pivots fold fS into the select kernel from k_dual_bfrt's a_F[R]
list) -- every trace must still be the oracle's bit for bit."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("spz,defer,minvt,sru", [("0", "1", "0", "1"), ("16", "1", "0", "1"), ("0", "0", "0", "1"),
                                                ("0", "1", "1", "1"), ("0", "1", "0", "0")],
                         ids=["rowwise", "default-zr", "rowwise-no-defer", "rowwise-minvt", "rowwise-dense-update"])
def test_csc_parity_with_sparse_ftran(spz, defer, minvt, sru):
    """(defer 0: the dual phase's update in its own k_update launch, ELP_DUAL_DEFER=0;
    minvt 1: the CSC load keeps the transposed inverse, ELP_CSC_MINVT=1; sru 0: the
    dense inverse update instead of the sparse one, ELP_SRU=0 -- the default CSC runs
    of every suite take the sparse one, and both keep the oracle's zero rule)"""
    env = dict(os.environ, ELP_RESIDENT="0", ELP_SPF_MIN="1", ELP_SPZ_MIN_MB=spz, ELP_DUAL_DEFER=defer, ELP_CSC_MINVT=minvt, ELP_SRU=sru)
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
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=os.path.dirname(HERE))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert " passed" in r.stdout
