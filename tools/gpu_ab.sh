#!/bin/bash
# Interleaved A/B of library variants / source trees on the C3 timed region
# (same session, same box), each optionally followed by a rocprofv3 kernel trace
# of the same region.  Variants: VARIANTS="tag=spec ..." where spec is
#   lib:NAME[,K=V] easylp_amd/lib/libeasylp_hip_NAME.so (ELP_LIB_PATH), extra environment
#   tree:DIR      another checkout (DIR/bench.py with its own library)
#   env:K=V[,K=V] the in-tree library under extra environment
#   base          the in-tree library as built
# ROUNDS (3) interleaved rounds; PROF=1 adds one rocprof trace per variant.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
TAG=${TAG:-ab}
(while sleep 30; do date +%T >> "$O/hb_$TAG.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
Q="--steps ${STEPS:-10} --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0"
QH="$Q --host-input 0 --highs 0"
setup() {  # spec -> DIR ARGS ENVS
  local spec=$1
  DIR="$R"; ARGS="$QH"; ENVS="X=0"
  case $spec in
    lib:*) local l=${spec#lib:}; ENVS="ELP_LIB_PATH=$R/easylp_amd/lib/libeasylp_hip_${l%%,*}.so"
           [ "$l" != "${l#*,}" ] && ENVS="$ENVS $(echo "${l#*,}" | tr ',' ' ')" ;;
    tree:*) DIR="$R/${spec#tree:}"; ARGS="$Q" ;;
    env:*) ENVS=$(echo "${spec#env:}" | tr ',' ' ') ;;
  esac
}
summ() {
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().splitlines()[-1])
r = d["roofline"]; w = d.get("steady_state") or {}
print(sys.argv[1], round(d["value"]), "it/s", "ms/solve", round(d["ms_per_step"], 2), "price(ev)",
      round(r["avg_launch_us"], 2), "window us/it", round(w.get("us_per_iteration") or 0, 2), flush=True)
EOF
}
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    tag=${v%%=*}; setup "${v#*=}"
    (cd "$DIR" && env $ENVS timeout -k 10 300 python -u bench.py $ARGS > "$O/ab_${TAG}_${tag}_$i.json" 2> "$O/ab_${TAG}_${tag}_$i.err") || { echo "bench $tag failed"; tail -5 "$O/ab_${TAG}_${tag}_$i.err"; exit 4; }
    summ "${tag}_$i" "$O/ab_${TAG}_${tag}_$i.json"
  done
done
[ "${PROF:-0}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  tag=${v%%=*}; setup "${v#*=}"
  rm -rf /tmp/kt_$tag
  (cd "$DIR" && env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$tag -o run -- python3 bench.py $ARGS --window 0 > "$O/prof_${TAG}_$tag.json" 2> "$O/prof_${TAG}_$tag.err") || { echo "rocprof $tag failed"; tail -5 "$O/prof_${TAG}_$tag.err"; exit 5; }
  cp "$(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats_${TAG}_$tag.csv"
  python3 "$R/tools/window_stats.py" "$(find /tmp/kt_$tag -name '*kernel_trace.csv' | head -1)" "$O/prof_${TAG}_$tag.json" > "$O/window_stats_${TAG}_$tag.json"
  python3 -c "
import json; d=json.load(open('$O/window_stats_${TAG}_$tag.json'))
print('$tag', 'price rocprof', round(d['k_price_avg_us_rocprof'],2), 'frac', round(d['frac_from_rocprof'],3), 'wall ms', round(d['window_wall_ms'],1), {k.split('(')[0]: round(v['avg_us'],2) for k, v in d['kernels'].items() if v['calls'] > 20000})"
  rm -rf /tmp/kt_$tag
done
