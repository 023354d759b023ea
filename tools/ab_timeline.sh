#!/bin/bash
# Per-kernel timeline (rocprofv3 kernel trace, iterations [100, 1100) of one
# solve) for each library variant: VARIANTS="base x y".
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
for V in ${VARIANTS:-base}; do
  if [ $V = base ]; then L=$ROOT/easylp_amd/lib/libeasylp_hip.so; else L=$ROOT/easylp_amd/lib/libeasylp_hip_$V.so; fi
  rm -rf /tmp/tl_$V
  ELP_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$V -o run -- python3 $ROOT/bench.py --steps 0 --warmup 0 --window 1 --c4 0 --sparse 0 --no-cpu --compare-rules 0 > $ROOT/gpurun_out/tl_$V.json 2>&1 || { echo "fail $V"; exit 1; }
  echo "== $V"; python3 $ROOT/tools/timeline.py $(find /tmp/tl_$V -name '*kernel_trace.csv') 100 1000 | head -7
  rm -rf /tmp/tl_$V
done
