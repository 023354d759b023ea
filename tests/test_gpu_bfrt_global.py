"""k_dual_bfrt's three paths for the bunch rounds: one wave with the candidates
in registers (up to 256 candidates: what the fixtures mostly have), the whole
workgroup from registers (up to 4 096), and the workgroup from dcomp / dalive
in global memory.  The dual parity tests run again in a child process with
ELP_BFRT_REG=1 (no one-wave path) and =0 (every BFRT from global memory) --
the traces, flips and pivots must still be the oracle's bit for bit, one GPU
and column-sharded ngpu ranks (the gathered records)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("mode", ["1", "0"])
def test_dual_parity_with_global_bfrt(mode):
    env = dict(os.environ, ELP_RESIDENT="0", ELP_BFRT_REG=mode)
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
           os.path.join(HERE, "test_gpu_dual.py"),
           os.path.join(HERE, "test_gpu_ngpu.py") + "::test_ngpu_dual_matches_oracle",
           os.path.join(HERE, "test_gpu_ngpu.py") + "::test_ngpu_dual_kkt_flips"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=os.path.dirname(HERE))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert " passed" in r.stdout
