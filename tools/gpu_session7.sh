# parity of the product build; C3 A/B of 128-column vs balanced packed tiles
# (interleaved, 3 each); grid-wide k_ratio stamps from the diagnostic build
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pricing.py tests/test_gpu_ngpu.py > gpurun_out/t7.log 2>&1
rc=$?; tail -3 gpurun_out/t7.log; [ $rc -ne 0 ] && exit $rc
ELP_TILE_BAL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py > gpurun_out/t7b.log 2>&1
rc=$?; tail -2 gpurun_out/t7b.log; [ $rc -ne 0 ] && exit $rc
Q="--steps 10 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-input 0"
for v in w1 b1 w2 b2 w3 b3; do
  unset ELP_TILE_BAL
  case $v in b*) export ELP_TILE_BAL=1;; esac
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/b7_$v.json 2> gpurun_out/b7_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/b7_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/b7_$v.json'));r=d['roofline'];w=d['steady_state'];print('$v', round(d['value']), 'it/s tto', round(d['time_to_optimal_s'],4), 'price us', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3), 'window us/it', round(w['us_per_iteration'],2))"
done
unset ELP_TILE_BAL
S="--steps 1 --warmup 0 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0 --c4 0"
ELP_LIB_PATH="$R/easylp_amd/lib/libeasylp_hip_diag.so" ELP_STAMPS=2 timeout -k 10 300 python bench.py $S > gpurun_out/stamps2_r03.json 2> gpurun_out/stamps2_r03.err || { echo "stamps run failed"; tail -5 gpurun_out/stamps2_r03.err; exit 6; }
grep -A2 "k_ratio stamps" gpurun_out/stamps2_r03.err
ELP_LIB_PATH="$R/easylp_amd/lib/libeasylp_hip_diag.so" ELP_STAMPS=1 timeout -k 10 300 python bench.py $S > gpurun_out/stamps1_r03.json 2> gpurun_out/stamps1_r03.err || { echo "stamps run failed"; tail -5 gpurun_out/stamps1_r03.err; exit 6; }
grep -A2 "k_ratio stamps" gpurun_out/stamps1_r03.err
