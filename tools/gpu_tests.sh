#!/bin/bash
# Run pytest node ids on the GPU box with -v -s output to gpurun_out/$TAG.log
# and a heartbeat file (a single long test prints nothing for minutes; the
# heartbeat keeps gpurun's silence detector from taking it for a hang while
# pytest's own --timeout bounds it).  Usage: tools/gpu_tests.sh TAG TIMEOUT node...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=$1; TO=$2; shift 2
(while sleep 30; do date +%T >> "gpurun_out/hb_$TAG.txt"; done) &
HB=$!
timeout -k 10 $((TO + 60)) python -u -m pytest -x -v -s --durations=15 --timeout "$TO" --timeout-method thread \
    -p no:cacheprovider "$@" > "gpurun_out/$TAG.log" 2>&1
rc=$?
kill $HB
tail -25 "gpurun_out/$TAG.log"
exit $rc
