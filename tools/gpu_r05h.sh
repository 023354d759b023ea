set -u
# r05h: the 4-wave k_ftran_zr_sq without scratch, against the one-wave version (prev = c87925b)
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_spz.py tests/test_gpu_dual.py tests/test_gpu_csc.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05h.log 2>&1 || { tail -30 gpurun_out/pytest_r05h.log; exit 1; }
tail -3 gpurun_out/pytest_r05h.log
bash tools/ab_sparse.sh r05h "prev base" 2 || exit 3
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05h_feas "prev base" 2 || exit 4
