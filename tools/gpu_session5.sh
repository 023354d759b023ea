set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v ${PYTEST_EXTRA:-} --timeout 400 --timeout-method thread -p no:cacheprovider --durations=20 > gpurun_out/pytest_gpu_r03b.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu_r03b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03b.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_r03b.log; exit 3; }
cat gpurun_out/smoke_r03b.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 3 --warmup 1 --c4 0 --sparse 0 --host-input 0 --window 0 > gpurun_out/bench_tr2_r03b.json 2> gpurun_out/bench_tr2_r03b.err || { echo "torchrun bench failed"; tail -20 gpurun_out/bench_tr2_r03b.err; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/bench_tr2_r03b.json'));print(d['value'], d['n_gpus'], d['config']['parallelism'], d['config']['fallback'])"
