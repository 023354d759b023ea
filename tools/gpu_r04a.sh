#!/bin/bash
# r04 session A: the GPU tests, then VERDICT r03 #2 -- an interleaved A/B of
# the r02 tree (abtree/r02: 1df1ffb's sources and bench, built here), HEAD and
# HEAD with the deferred plan in trailing pricing workgroups (ELP_TRAIL_APPLY=1,
# r02's layout) on the C3 timed region, each with a rocprofv3 kernel trace of
# the same region; then the driver's exact bench command.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
(while sleep 30; do date +%T >> "$O/hb_r04a.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$O/host_r04a.txt"
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --durations=25 --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu_r04a.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu_r04a.log"; [ $rc -ne 0 ] && exit $rc
fi
Q="--steps 10 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0"
QH="$Q --host-input 0 --highs 0"
run() {  # tag dir env...
  local tag=$1 dir=$2; shift 2
  local args="$Q"; [ "$dir" = "$R" ] && args="$QH"
  (cd "$dir" && env "$@" timeout -k 10 300 python -u bench.py $args > "$O/ab_$tag.json" 2> "$O/ab_$tag.err") || { echo "bench $tag failed"; tail -5 "$O/ab_$tag.err"; exit 4; }
  python -c "import json;d=json.loads(open('$O/ab_$tag.json').read().splitlines()[-1]);r=d['roofline'];w=d['steady_state'];print('$tag', round(d['value']), 'it/s ms/solve', round(d['ms_per_step'],2), 'price us', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3), 'window us/it', round(w['us_per_iteration'],2), 'w.price', round(w['price_avg_launch_us'],2))"
}
for i in 1 2 3; do
  run r02_$i "$R/abtree/r02" X=0
  run head_$i "$R" X=0
  run trail_$i "$R" ELP_TRAIL_APPLY=1
done
REG="--steps 10 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --window 0"
cd /tmp && export TMPDIR=/tmp
prof() {  # tag dir env...
  local tag=$1 dir=$2; shift 2
  local args="$REG"; [ "$dir" = "$R" ] && args="$REG --host-input 0 --highs 0"
  rm -rf /tmp/kt_$tag
  (cd "$dir" && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$tag -o run -- python3 bench.py $args > "$O/prof_$tag.json" 2> "$O/prof_$tag.err") || { echo "rocprof $tag failed"; tail -5 "$O/prof_$tag.err"; exit 5; }
  cp "$(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats_r04a_$tag.csv"
  python3 "$R/tools/window_stats.py" "$(find /tmp/kt_$tag -name '*kernel_trace.csv' | head -1)" "$O/prof_$tag.json" > "$O/window_stats_r04a_$tag.json" && cat "$O/window_stats_r04a_$tag.json"
  rm -rf /tmp/kt_$tag
}
prof r02 "$R/abtree/r02" X=0
prof head "$R" X=0
prof trail "$R" ELP_TRAIL_APPLY=1
cd "$R"
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_r04a.json" 2> "$O/bench_r04a.err" || { echo "bench failed rc=$?"; tail -20 "$O/bench_r04a.err"; exit 6; }
python -c "import json;d=json.loads(open('$O/bench_r04a.json').read().splitlines()[-1]);print({k:d[k] for k in ('value','time_to_optimal_s','time_to_optimal_hbm_s')}, d['roofline']['avg_launch_us'], d['roofline']['frac']); print(json.dumps(d.get('cpu_baseline_highs'))[:1500])"
echo done
