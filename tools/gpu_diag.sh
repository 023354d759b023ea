#!/bin/bash
# Latency-chain diagnostics of the C3 solve on one GPU box: in-kernel phase
# stamps (diagnostic build, ELP_STAMPS=1, workgroup 0 of k_ratio / the select
# kernel / k_ftran_zr) and a clean rocprofv3 per-iteration timeline over
# iterations [100, 1100).  Usage: tools/gpu_diag.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-diag}
S="--steps 1 --warmup 0 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0 --host-c4 0 --c4 0"
ELP_LIB_PATH="$ROOT/easylp_amd/lib/libeasylp_hip_diag.so" ELP_STAMPS=1 timeout -k 10 300 python bench.py $S \
    > "$OUT/stamps_$TAG.json" 2> "$OUT/stamps_$TAG.err" || { echo "stamps run failed"; tail -5 "$OUT/stamps_$TAG.err"; exit 6; }
grep -A2 "k_ratio stamps" "$OUT/stamps_$TAG.err"
TMP=/tmp/elp_diag_$TAG
WIN="--steps 0 --warmup 0 --window 1 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-input 0 --host-c4 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$TMP/tl" -o run -- python3 "$ROOT/bench.py" $WIN \
    > "$OUT/tl_$TAG.json" 2>&1 || { echo "rocprof timeline failed"; exit 7; }
python3 "$ROOT/tools/timeline.py" "$(find "$TMP/tl" -name '*kernel_trace.csv' | head -1)" 100 1000 > "$OUT/timeline_$TAG.txt" \
    && head -8 "$OUT/timeline_$TAG.txt"
rm -rf "$TMP"
