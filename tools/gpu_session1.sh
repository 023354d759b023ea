set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_c_driver.py tests/test_gpu_ngpu.py > gpurun_out/t_new.log 2>&1
rc=$?; tail -30 gpurun_out/t_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --c4 0 --sparse 0 --no-cpu --compare-rules 0 --host-c4 0 > gpurun_out/b1.json 2> gpurun_out/b1.err
rc=$?; tail -3 gpurun_out/b1.err; python -c "import json;d=json.load(open('gpurun_out/b1.json'));print(d['value'],d['time_to_optimal_s'],json.dumps(d['host_input']))"; exit $rc
