# A/B of the host poll interval (elp_control.sync_every) on the 5000x50000 bench, one GPU session
set -u
mkdir -p gpurun_out
for S in 32 64 128 32 64 128 32 64 128; do
  timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu --c4 0 --sparse 0 --compare-rules 0 --sync-every $S > gpurun_out/sab_$S.json 2> gpurun_out/sab_$S.err || { echo "fail $S"; tail gpurun_out/sab_$S.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/sab_$S.json').read().splitlines()[-1])
w = d.get('steady_state') or {}
print('sync $S solve', round(d['value']), 'it/s', d['final']['iterations_to_optimal'], 'its | window', round(w.get('us_per_iteration') or 0, 2), 'us/it')"
done
