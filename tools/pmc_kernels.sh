#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (one counter group each) over one full
# solve of the 5000x50000 LP; summary -> gpurun_out/pmc_kernels_<tag>.json
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG=${1:-r02}
TMP=/tmp/elp_pmck_$TAG
mkdir -p "$OUT" "$TMP"
ARGS="--steps 1 --warmup 0 --no-cpu --c4 0 --sparse 0 --compare-rules 0 --window 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$TMP/f" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmck_f_$TAG.json" 2> "$OUT/pmck_f_$TAG.err" || { echo "fetch pass failed"; tail "$OUT/pmck_f_$TAG.err"; exit 5; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$TMP/w" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmck_w_$TAG.json" 2> "$OUT/pmck_w_$TAG.err" || { echo "write pass failed"; tail "$OUT/pmck_w_$TAG.err"; exit 6; }
python3 "$ROOT/tools/pmc_kernels.py" "$(find "$TMP/f" -name '*counter_collection.csv' | head -1)" \
    "$(find "$TMP/w" -name '*counter_collection.csv' | head -1)" "$OUT/pmck_f_$TAG.json" > "$OUT/pmc_kernels_$TAG.json" && cat "$OUT/pmc_kernels_$TAG.json"
rm -rf "$TMP"
