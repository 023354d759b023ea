# (0) parity of the default library (Dev by pointer); kernel-argument probe;
# (1) C3: Dev by pointer vs by value (libeasylp_hip_val.so), balanced tiles;
# (2) C4 (10000 x 500000): cached vs non-temporal pricing sweep, per-kernel
#     averages over the last 2000 iterations (rocprofv3 kernel trace);
# (3) ELP_STAMPS phase stamps at C3 and C4
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pricing.py > gpurun_out/t6.log 2>&1
rc=$?; tail -3 gpurun_out/t6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 ./tools/kernarg_probe > gpurun_out/kernarg_probe.txt 2>&1 || { echo "probe failed"; cat gpurun_out/kernarg_probe.txt; exit 3; }
cat gpurun_out/kernarg_probe.txt
Q="--steps 10 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-input 0"
for v in ptr val bal ptr2 val2; do
  unset ELP_TILE_BAL ELP_LIB_PATH
  case $v in val*) export ELP_LIB_PATH="$R/easylp_amd/lib/libeasylp_hip_val.so";; bal) export ELP_TILE_BAL=1;; esac
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/b6_$v.json 2> gpurun_out/b6_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/b6_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/b6_$v.json'));r=d['roofline'];w=d['steady_state'];print('$v', round(d['value']), 'it/s tto', round(d['time_to_optimal_s'],4), 'price us', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3), 'window us/it', round(w['us_per_iteration'],2))"
done
unset ELP_TILE_BAL ELP_LIB_PATH
cd /tmp && export TMPDIR=/tmp
Q="--steps 0 --warmup 0 --c4 1 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0"
for v in nt0 ntauto; do
  if [ $v = nt0 ]; then export ELP_SWEEP_NT=0; else unset ELP_SWEEP_NT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c4_$v -o run -- python3 "$R/bench.py" $Q > "$R/gpurun_out/c4_$v.json" 2> "$R/gpurun_out/c4_$v.err" || { echo "c4 $v failed"; tail -5 "$R/gpurun_out/c4_$v.err"; exit 5; }
  python3 "$R/tools/c4_kernels.py" "$(find /tmp/c4_$v -name '*kernel_trace.csv' | head -1)" 2000 > "$R/gpurun_out/c4k_$v.txt"
  head -8 "$R/gpurun_out/c4k_$v.txt"
  python3 -c "import json;d=json.load(open('$R/gpurun_out/c4_$v.json'));s=d['scaling_config'];print('$v', s['iterations_to_optimal'], round(s['time_to_optimal_s'],3), s['objective'])"
  rm -rf /tmp/c4_$v
done
unset ELP_SWEEP_NT
cd "$R"
S="--steps 1 --warmup 0 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0"
ELP_STAMPS=1 timeout -k 10 300 python bench.py $S --c4 1 > gpurun_out/stamps_r03.json 2> gpurun_out/stamps_r03.err || { echo "stamps run failed"; tail -5 gpurun_out/stamps_r03.err; exit 6; }
grep -A2 "k_ratio stamps" gpurun_out/stamps_r03.err
