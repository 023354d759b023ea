set -u
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_spz.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_basis.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05f.log 2>&1 || { tail -30 gpurun_out/pytest_r05f.log; exit 1; }
tail -3 gpurun_out/pytest_r05f.log
bash tools/stamps_sparse.sh r05f || exit 2
bash tools/ab_sparse.sh r05f "lpr1 base" 2 || exit 3
