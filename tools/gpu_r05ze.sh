set -u
# r05ze: the sparse inverse update with 4 rows per workgroup (base) against one (rpw1)
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_basis.py tests/test_gpu_mip.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05ze.log 2>&1 || { tail -30 gpurun_out/pytest_r05ze.log; exit 1; }
tail -3 gpurun_out/pytest_r05ze.log
bash tools/ab_sparse.sh r05ze "rpw1 base" 2 || exit 5
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05ze_feas "rpw1 base" 1 || exit 4
