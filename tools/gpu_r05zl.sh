set -u
# r05zl: the a_F row grouping by an LDS table (bfrt_flip_lds, bfrt_flip_column) on top of r05zh: parity, A/B against the last commit, stamps
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_bfrt_global.py tests/test_gpu_mip.py tests/test_gpu_ngpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05zl.log 2>&1 || { tail -30 gpurun_out/pytest_r05zl.log; exit 1; }
tail -3 gpurun_out/pytest_r05zl.log
bash tools/ab_sparse.sh r05zl "prev base" 2 || exit 5
bash tools/stamps_sparse.sh r05zl || exit 6
grep "k_dual_bfrt" gpurun_out/stamps_r05zl.txt
grep "k_dual_bfrt a_F by" gpurun_out/stamps_r05zl.txt
