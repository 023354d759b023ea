set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_lu.py -k "fixtures or refusals" > gpurun_out/t_lu.log 2>&1
rc=$?; tail -15 gpurun_out/t_lu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_c_driver.py tests/test_gpu_ngpu.py tests/test_gpu_lu.py > gpurun_out/t_new.log 2>&1
rc=$?; tail -30 gpurun_out/t_new.log; exit $rc
