#!/bin/bash
# Round-5 GPU session for the sparse (CSC) path: selected parity tests, the
# 20 000 x 100 000 probe times, and a rocprofv3 kernel-stats pass of the
# phase-1 (dual) LP.  Usage: tools/gpu_r05.sh TAG "tests/a.py tests/b.py ..."
# Every GPU step has its own time limit; a failure ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r05}
TESTS=${2:-}
TMP=/tmp/elp_prof_$TAG
mkdir -p "$TMP"
(while sleep 30; do date +%T >> "$OUT/hb_$TAG.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -v -x --durations=15 --timeout 900 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?
  tail -25 "$OUT/pytest_$TAG.log"
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "${PROBE:-1}" = "1" ]; then
  timeout -k 10 300 python3 "$ROOT/tools/sparse_probe.py" > "$OUT/sparse_probe_$TAG.txt" 2>&1 && cat "$OUT/sparse_probe_$TAG.txt" || { echo "sparse probe failed"; cat "$OUT/sparse_probe_$TAG.txt"; exit 8; }
fi
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$TMP/sp" -o run -- python3 "$ROOT/tools/sparse_probe.py" ${PROF_LP:-kkt_20000x100000} > "$OUT/sparse_prof_$TAG.txt" 2>&1 || { echo "sparse rocprof failed"; tail -20 "$OUT/sparse_prof_$TAG.txt"; exit 9; }
  cp "$(find "$TMP/sp" -name '*kernel_stats.csv' | head -1)" "$OUT/sparse_kernel_stats_$TAG.csv"
  python3 "$ROOT/tools/kstats.py" "$OUT/sparse_kernel_stats_$TAG.csv"
fi
rm -rf "$TMP"
echo done
