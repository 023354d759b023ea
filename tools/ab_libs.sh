#!/bin/bash
# A/B of prebuilt library variants (easylp_amd/lib/libeasylp_hip_<V>.so; "base"
# = libeasylp_hip.so) in one GPU session: VARIANTS="base x y base x".
# Prints the whole-solve rate (steps are full solves), the steady-state window
# (iterations [100, 1100) of one solve) and the pricing launch (HIP events).
# A variant that changes a reduction order walks another pivot path: compare
# it on the window, not on the whole solve.  BENCH_ARGS overrides the bench
# arguments (default: C3 only, 3 timed solves).
set -u
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu --c4 0 --sparse 0 --compare-rules 0"}
for V in ${VARIANTS:-base}; do
  if [ $V = base ]; then L=easylp_amd/lib/libeasylp_hip.so; else L=easylp_amd/lib/libeasylp_hip_$V.so; fi
  ELP_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { echo "fail $V"; tail gpurun_out/ab_$V.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/ab_$V.json').read().splitlines()[-1])
w = d.get('steady_state') or {}
r = d['roofline']
c = d.get('scaling_config') or {}
print('$V', 'solve', round(d['value']), 'it/s', d['final']['iterations_to_optimal'], 'its |',
      'window', round(w.get('value') or 0), 'it/s', round(w.get('us_per_iteration') or 0, 2), 'us/it',
      'price', round(w.get('price_avg_launch_us') or 0, 2), 'us |', 'solve price', round(r['avg_launch_us'], 2),
      'us frac', round(r['frac'], 3), '| c4', c.get('value'))"
done
