#!/bin/bash
# A/B of library variants on the sparse 20 000 x 100 000 LPs (one GPU session):
# tools/ab_sparse.sh TAG "name1 name2 ..." [rounds] -- each name is
# easylp_amd/lib/libeasylp_hip_NAME.so (tools/build_variant.sh) or "base" for
# the default library, optionally with one environment setting after "@"
# ("base@ELP_DUAL_DEFER=0"); interleaved probe rounds, then one rocprofv3
# kernel-stats pass of the phase-1 LP per variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=$1; NAMES=$2; ROUNDS=${3:-2}
LP=${LP:-kkt_20000x100000}
(while sleep 30; do date +%T >> "$OUT/hb_$TAG.txt"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
lib() { local n=${1%%@*}; if [ "$n" = base ]; then echo "$ROOT/easylp_amd/lib/libeasylp_hip.so"; else echo "$ROOT/easylp_amd/lib/libeasylp_hip_$n.so"; fi; }
envof() { case "$1" in *@*) echo "${1#*@}";; *) echo "ELP_AB_NONE=1";; esac; }
for r in $(seq 1 "$ROUNDS"); do
  for v in $NAMES; do
    echo -n "round $r $v: " | tee -a "$OUT/ab_$TAG.txt"
    env "$(envof "$v")" ELP_LIB_PATH=$(lib "$v") timeout -k 10 120 python3 tools/sparse_probe.py $LP 2>/dev/null | tee -a "$OUT/ab_$TAG.txt" || { echo "variant $v failed"; exit 3; }
  done
done
cd /tmp && export TMPDIR=/tmp
for v in $NAMES; do
  rm -rf "/tmp/ab_$v"
  export "$(envof "$v")"
  ELP_LIB_PATH=$(lib "$v") timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/ab_$v" -o run -- python3 "$ROOT/tools/sparse_probe.py" $LP > /dev/null 2>&1 || { echo "rocprof $v failed"; exit 4; }
  unset "$(envof "$v" | cut -d= -f1)"
  cp "$(find "/tmp/ab_$v" -name '*kernel_stats.csv' | head -1)" "$OUT/ab_${TAG}_$v.csv"
  echo "== $v" | tee -a "$OUT/ab_$TAG.txt"
  python3 "$ROOT/tools/kstats.py" "$OUT/ab_${TAG}_$v.csv" > "$OUT/ab_${TAG}_$v.txt"; head -12 "$OUT/ab_${TAG}_$v.txt" | tee -a "$OUT/ab_$TAG.txt"
done
echo done
