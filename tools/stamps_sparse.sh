#!/bin/bash
# Phase stamps (ELP_STAMPS=1, the diagnostic build tools/build_variant.sh diag
# "-DELP_DIAG=1") of the dual iteration's ratio-test, select, FTRAN-z and
# k_ratio kernels on the 20 000 x 100 000 phase-1 LP; printed at elp_destroy.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
ELP_STAMPS=1 ELP_LIB_PATH="$ROOT/easylp_amd/lib/libeasylp_hip_diag.so" timeout -k 10 120 python3 tools/sparse_probe.py ${LP:-kkt_20000x100000} > gpurun_out/stamps_${1:-r05}.txt 2>&1
rc=$?
cat gpurun_out/stamps_${1:-r05}.txt
exit $rc
