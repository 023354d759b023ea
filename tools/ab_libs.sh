#!/bin/bash
# A/B of prebuilt library variants (easylp_amd/lib/libeasylp_hip_<V>.so; "base"
# = libeasylp_hip.so) on the bench's timed window: VARIANTS="base x y base x"
# BENCH_ARGS overrides the bench arguments (default: C3 only, 2000 steps).
set -u
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 2000 --no-cpu --no-optimal --c4 0 --sparse 0"}
for V in ${VARIANTS:-base}; do
  if [ $V = base ]; then L=easylp_amd/lib/libeasylp_hip.so; else L=easylp_amd/lib/libeasylp_hip_$V.so; fi
  ELP_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { echo "fail $V"; tail gpurun_out/ab_$V.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$V.json').read().splitlines()[-1]); c=d.get('scaling_config') or {}; print('$V', round(d['value']), 'sweep us', round(d['roofline']['avg_launch_us'],2), 'frac', round(d['roofline']['frac'],3), 'c4', c.get('value'))"
done
