set -u
# r05x: the Newton-Schulz GEMM with the next chunk's operands in flight: parity suites, A/B on both
# sparse LPs against the last commit
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_csc.py tests/test_gpu_dual.py tests/test_gpu_fullsize.py tests/test_gpu_c4.py tests/test_gpu_basis.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05x.log 2>&1 || { tail -30 gpurun_out/pytest_r05x.log; exit 1; }
tail -3 gpurun_out/pytest_r05x.log
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05x_feas "prev base" 1 || exit 4
bash tools/ab_sparse.sh r05x "prev base" 1 || exit 5
