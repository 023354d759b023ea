set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/lu_probe.py kkt2k pack1k > gpurun_out/lu_probe3.txt 2>&1
cat gpurun_out/lu_probe3.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=15 > gpurun_out/pytest_gpu_r03a.log 2>&1
rc=$?; tail -40 gpurun_out/pytest_gpu_r03a.log; exit $rc
