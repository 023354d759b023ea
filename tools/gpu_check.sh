#!/bin/bash
# One GPU-box session: parity tests, smoke, the bench line exactly as the
# driver runs it (`bench.py --gpus 1 --steps 20 --warmup 5`), then the
# profiles committed under profiles/:
#   * rocprofv3 --kernel-trace --stats of the same timed region (the same 25
#     full solves, without the secondary configs: every solve is identical, so
#     the per-kernel averages are the timed window's);
#   * a separate PMC pass (FETCH_SIZE) over the same command for the pricing
#     kernel's HBM traffic per launch (timed dispatches only);
#   * a per-iteration timeline over iterations [100, 1100) of one solve.
# Traces go to /tmp on the box (too large to bring back); summaries to gpurun_out/.
# Each GPU step has its own time limit; a crash / fault / timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r02}
SKIP_TESTS=${SKIP_TESTS:-0}
STEPS=${STEPS:-20}
WARM=${WARM:-5}
TMP=/tmp/elp_prof_$TAG
mkdir -p "$TMP"
# heartbeat: single GPU tests and solves can run minutes without printing;
# every step below has its own time limit
(while sleep 30; do date +%T >> "$OUT/hb_$TAG.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$OUT/host_$TAG.txt"

if [ "$SKIP_TESTS" = "0" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --durations=25 --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu_$TAG.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed rc=$?"; cat "$OUT/smoke_$TAG.log"; exit 3; }
cat "$OUT/smoke_$TAG.log"
fi

timeout -k 10 600 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_$TAG.err"; exit 4; }
cat "$OUT/bench_$TAG.json"

REG="--steps $STEPS --warmup $WARM --c4 0 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0 --host-c4 0 --c2 0 --small 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$TMP/kt" -o run -- python3 "$ROOT/bench.py" $REG > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_bench_$TAG.err" || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof_bench_$TAG.err"; exit 5; }
cp "$(find "$TMP/kt" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats_$TAG.csv"
python3 "$ROOT/tools/window_stats.py" "$(find "$TMP/kt" -name '*kernel_trace.csv' | head -1)" "$OUT/prof_bench_$TAG.json" > "$OUT/window_stats_$TAG.json" && cat "$OUT/window_stats_$TAG.json"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_price --output-format csv -d "$TMP/pmc" -o run -- python3 "$ROOT/bench.py" $REG > "$OUT/pmc_bench_$TAG.json" 2> "$OUT/pmc_bench_$TAG.err" || { echo "rocprof pmc failed rc=$?"; tail -20 "$OUT/pmc_bench_$TAG.err"; exit 6; }
python3 "$ROOT/tools/pmc_traffic.py" "$(find "$TMP/pmc" -name '*counter_collection.csv' | head -1)" "$OUT/pmc_bench_$TAG.json" > "$OUT/pmc_traffic_$TAG.json" && cat "$OUT/pmc_traffic_$TAG.json"
WIN="--steps 0 --warmup 0 --window 1 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-input 0 --host-c4 0 --c2 0 --small 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$TMP/tl" -o run -- python3 "$ROOT/bench.py" $WIN > "$OUT/tl_bench_$TAG.json" 2>&1 || { echo "rocprof timeline failed"; exit 7; }
python3 "$ROOT/tools/timeline.py" "$(find "$TMP/tl" -name '*kernel_trace.csv' | head -1)" 100 1000 > "$OUT/timeline_$TAG.txt" && cat "$OUT/timeline_$TAG.txt"
# the sparse 20000 x 100000 LPs: probe times, then the per-kernel
# stats of the phase-1 (dual simplex) solve
timeout -k 10 300 python3 "$ROOT/tools/sparse_probe.py" > "$OUT/sparse_probe_$TAG.txt" 2>&1 && cat "$OUT/sparse_probe_$TAG.txt" || { echo "sparse probe failed"; exit 8; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$TMP/sp" -o run -- python3 "$ROOT/tools/sparse_probe.py" kkt_20000x100000 > "$OUT/sparse_prof_$TAG.txt" 2>&1 || { echo "sparse rocprof failed"; exit 9; }
cp "$(find "$TMP/sp" -name '*kernel_stats.csv' | head -1)" "$OUT/sparse_kernel_stats_$TAG.csv"
# ... and of the feasible-start (primal) solve
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$TMP/spf" -o run -- python3 "$ROOT/tools/sparse_probe.py" kkt_feasible_20000x100000 > "$OUT/feasible_prof_$TAG.txt" 2>&1 || { echo "feasible rocprof failed"; exit 10; }
cp "$(find "$TMP/spf" -name '*kernel_stats.csv' | head -1)" "$OUT/feasible_kernel_stats_$TAG.csv"
# the resident small-LP solver: Klee-Minty and the per-stage counters
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$TMP/km" -o run -- python3 "$ROOT/tools/resident_km.py" > "$OUT/resident_prof_$TAG.txt" 2>&1 || { echo "resident rocprof failed"; exit 11; }
cp "$(find "$TMP/km" -name '*kernel_stats.csv' | head -1)" "$OUT/resident_kernel_stats_$TAG.csv"
rm -rf "$TMP"
echo done
