#!/bin/bash
# Does the HIP-event pricing timer perturb the timed solves, and does it agree
# with a rocprofv3 kernel trace of the same command?
set -u
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; cd $ROOT; mkdir -p gpurun_out
A="--steps 5 --warmup 1 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --window 0"
for pp in 1 0 1 0; do
  timeout -k 10 120 python bench.py $A --profile-price $pp > gpurun_out/ev_$pp.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ev_$pp.json').read().splitlines()[-1]); print('profile', $pp, round(d['value']), 'it/s', d['roofline']['avg_launch_us'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/evk -o run -- python3 $ROOT/bench.py $A > $ROOT/gpurun_out/ev_prof.json 2>/dev/null || exit 2
python3 $ROOT/tools/window_stats.py $(find /tmp/evk -name '*kernel_trace.csv') $ROOT/gpurun_out/ev_prof.json | head -8
