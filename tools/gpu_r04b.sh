#!/bin/bash
# r04 session B: the dual simplex GPU tests, then the ngpu / sensitivity / ABI /
# parity subsets touched this round.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
(while sleep 30; do date +%T >> "$O/hb_r04b.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py -v -x --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_dual_r04b.log" 2>&1
rc=$?; tail -15 "$O/pytest_dual_r04b.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ngpu.py tests/test_gpu_sensitivity.py tests/test_gpu_parity.py tests/test_abi.py -v -x --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_sub_r04b.log" 2>&1
rc=$?; tail -5 "$O/pytest_sub_r04b.log"; exit $rc
