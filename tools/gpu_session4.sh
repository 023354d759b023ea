set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pricing.py tests/test_gpu_lu.py::test_bump_capacity_growth tests/test_gpu_ngpu.py > gpurun_out/t4.log 2>&1
rc=$?; tail -8 gpurun_out/t4.log; [ $rc -ne 0 ] && exit $rc
Q="--steps 10 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-c4 0"
for v in bal w128 bal2; do
  if [ $v = w128 ]; then export ELP_TILE_W=128; else unset ELP_TILE_W; fi
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/b4_$v.json 2> gpurun_out/b4_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/b4_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/b4_$v.json'));r=d['roofline'];w=d['steady_state'];h=d['host_input']['c3']['best'];print('$v', round(d['value']), 'it/s tto', round(d['time_to_optimal_s'],4), 'price us', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3), 'window us/it', round(w['us_per_iteration'],2), 'host tto', round(h['time_to_optimal_s'],4), 'h2d', round(h['h2d_s'],4), round(h['h2d_GBps'] or 0,1))"
done
