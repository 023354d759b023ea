#!/bin/bash
# A/B of environment settings on one library in one GPU session:
#   ENVS="ELP_LOOKAHEAD=0 - ELP_LOOKAHEAD=0 -"   ("-" = no extra setting)
# Same report as tools/ab_libs.sh.
set -u
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu --c4 0 --sparse 0 --compare-rules 0"}
i=0
for E in ${ENVS:--}; do
  i=$((i + 1))
  if [ "$E" = - ]; then EV=""; else EV="$E"; fi
  env $EV timeout -k 10 200 python bench.py $ARGS > gpurun_out/abe_$i.json 2>gpurun_out/abe_$i.err || { echo "fail $E"; tail gpurun_out/abe_$i.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/abe_$i.json').read().splitlines()[-1])
w = d.get('steady_state') or {}
r = d['roofline']
print('$E', 'solve', round(d['value']), 'it/s', d['final']['iterations_to_optimal'], 'its', round(d['ms_per_step'], 1), 'ms |',
      'window', round(w.get('value') or 0), 'it/s', round(w.get('us_per_iteration') or 0, 2), 'us/it |',
      'solve price', round(r['avg_launch_us'], 2), 'us frac', round(r['frac'], 3))"
done
