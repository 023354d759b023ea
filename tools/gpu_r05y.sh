set -u
# r05y: Newton-Schulz GEMM with 8 x 8 outputs per thread (base) against 4 x 4 (ns4)
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_parity.py tests/test_gpu_csc.py tests/test_gpu_fullsize.py tests/test_gpu_basis.py tests/test_gpu_dual.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05y.log 2>&1 || { tail -30 gpurun_out/pytest_r05y.log; exit 1; }
tail -3 gpurun_out/pytest_r05y.log
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05y_feas "ns4 base" 1 || exit 4
bash tools/ab_sparse.sh r05y "prev ns4 base" 1 || exit 5
