#!/bin/bash
# Quick GPU iteration loop: parity tests (dense + CSC), bench (C3, no CPU leg),
# and a kernel-trace timeline over iterations [100, 1100).  Stops at the first
# failing GPU step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-q}
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_csc.py"}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS -p no:cacheprovider > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 200 python bench.py --no-cpu --c4 ${C4:-0} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed"; tail -5 "$OUT/bench_$TAG.err"; exit 4; }
python -c "import json; d=json.loads(open('$OUT/bench_$TAG.json').read().splitlines()[-1]); print('it/s', round(d['value']), 'ms/step', round(d['ms_per_step']*1e3,2), 'us; tto', d['time_to_optimal_s'], 'price frac', round(d['roofline']['frac'],3), 'c4', (d.get('scaling_config') or {}).get('value'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 1000 --no-cpu --no-optimal --c4 0 > "$OUT/tl_bench_$TAG.json" 2>&1 || { echo "rocprof failed"; exit 5; }
python3 "$ROOT/tools/timeline.py" $(find "$OUT/tl_$TAG" -name "*kernel_trace.csv") 100 1000 | tee "$OUT/tl_$TAG.txt"
