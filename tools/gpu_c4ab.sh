#!/bin/bash
# C4 (10 000 x 500 000) per-kernel A/B of library variants over the last 2000
# iterations (rocprofv3 kernel trace), after the parity tests of the default
# build.  VARIANTS="base pre" (base = libeasylp_hip.so); TESTS overrides the
# parity tests run first.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd "$R"
(while sleep 30; do date +%T >> gpurun_out/hb_c4ab.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/c4ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/c4ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
Q="--steps 0 --warmup 0 --c4 1 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0 --host-c4 0"
for v in ${VARIANTS:-base pre}; do
  if [ $v = base ]; then L="$R/easylp_amd/lib/libeasylp_hip.so"; else L="$R/easylp_amd/lib/libeasylp_hip_$v.so"; fi
  ELP_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c4_$v -o run -- python3 "$R/bench.py" $Q > "$R/gpurun_out/c4_$v.json" 2> "$R/gpurun_out/c4_$v.err" || { echo "c4 $v failed"; tail -5 "$R/gpurun_out/c4_$v.err"; exit 5; }
  python3 "$R/tools/c4_kernels.py" "$(find /tmp/c4_$v -name '*kernel_trace.csv' | head -1)" 2000 > "$R/gpurun_out/c4k_$v.txt"
  cp "$(find /tmp/c4_$v -name '*kernel_stats.csv' | head -1)" "$R/gpurun_out/c4_kernel_stats_$v.csv"
  echo "== $v"; head -6 "$R/gpurun_out/c4k_$v.txt"
  python3 -c "import json;d=json.load(open('$R/gpurun_out/c4_$v.json'));s=d['scaling_config'];print('$v', s['iterations_to_optimal'], round(s['time_to_optimal_s'],3), s['objective'])"
  rm -rf /tmp/c4_$v
done
