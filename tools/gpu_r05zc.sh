set -u
# r05zc: the CHUZR reductions by wave (k_dual_chuzr / k_dual_row): parity, A/B against the last commit
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_bfrt_global.py tests/test_gpu_mip.py tests/test_gpu_ngpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05zc.log 2>&1 || { tail -30 gpurun_out/pytest_r05zc.log; exit 1; }
tail -3 gpurun_out/pytest_r05zc.log
bash tools/ab_sparse.sh r05zc "prev base" 2 || exit 5
