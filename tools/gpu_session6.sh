# C4 (10000 x 500000): cached vs non-temporal pricing sweep, per-kernel
# averages over the last 2000 iterations (rocprofv3 kernel trace)
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
Q="--steps 0 --warmup 0 --c4 1 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0"
for v in ${VARIANTS:-nt0 ntauto}; do
  if [ $v = nt0 ]; then export ELP_SWEEP_NT=0; else unset ELP_SWEEP_NT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c4_$v -o run -- python3 "$R/bench.py" $Q > "$R/gpurun_out/c4_$v.json" 2> "$R/gpurun_out/c4_$v.err" || { echo "c4 $v failed"; tail -5 "$R/gpurun_out/c4_$v.err"; exit 4; }
  python3 "$R/tools/c4_kernels.py" "$(find /tmp/c4_$v -name '*kernel_trace.csv' | head -1)" 2000 > "$R/gpurun_out/c4k_$v.txt"
  head -8 "$R/gpurun_out/c4k_$v.txt"
  python3 -c "import json;d=json.load(open('$R/gpurun_out/c4_$v.json'));s=d['scaling_config'];print('$v', s['iterations_to_optimal'], round(s['time_to_optimal_s'],3), s['objective'])"
  rm -rf /tmp/c4_$v
done
unset ELP_SWEEP_NT
cd "$R"
S="--steps 1 --warmup 0 --sparse 0 --no-cpu --compare-rules 0 --window 0 --host-input 0"
ELP_STAMPS=1 timeout -k 10 300 python bench.py $S --c4 1 > gpurun_out/stamps_r03.json 2> gpurun_out/stamps_r03.err || { echo "stamps run failed"; tail -5 gpurun_out/stamps_r03.err; exit 5; }
grep -A2 "k_ratio stamps" gpurun_out/stamps_r03.err
