#!/bin/bash
# One GPU-box session: parity tests, smoke, the full bench line, then the
# profiles committed under profiles/: a rocprofv3 kernel trace + stats of the
# bench's timed window only (no run to optimality, no secondary configs), the
# per-iteration timeline of that trace, and a separate PMC pass (FETCH_SIZE)
# for the pricing kernel's HBM traffic over the same window.
# Each GPU step has its own time limit; a crash / fault / timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-1000}
SKIP_TESTS=${SKIP_TESTS:-0}
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$OUT/host_$TAG.txt"

if [ "$SKIP_TESTS" = "0" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu_$TAG.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed rc=$?"; cat "$OUT/smoke_$TAG.log"; exit 3; }
cat "$OUT/smoke_$TAG.log"
fi

timeout -k 10 400 python bench.py --steps "$STEPS" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_$TAG.err"; exit 4; }
cat "$OUT/bench_$TAG.json"

WIN="--steps $STEPS --warmup 100 --no-cpu --no-optimal --c4 0 --sparse 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$ROOT/bench.py" $WIN > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_bench_$TAG.err" || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof_bench_$TAG.err"; exit 5; }
python3 "$ROOT/tools/timeline.py" $(find "$OUT/prof_$TAG" -name "*kernel_trace.csv") 100 "$STEPS" > "$OUT/timeline_$TAG.txt" && cat "$OUT/timeline_$TAG.txt"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_price --output-format csv -d "$OUT/pmc_$TAG" -o run -- python3 "$ROOT/bench.py" $WIN --profile-price 0 > "$OUT/pmc_bench_$TAG.json" 2> "$OUT/pmc_bench_$TAG.err" || { echo "rocprof pmc failed rc=$?"; tail -20 "$OUT/pmc_bench_$TAG.err"; exit 6; }
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_$TAG/run_counter_collection.csv" "$OUT/pmc_bench_$TAG.json" 100 "$STEPS" > "$OUT/pmc_traffic_$TAG.json" && cat "$OUT/pmc_traffic_$TAG.json"
echo done
