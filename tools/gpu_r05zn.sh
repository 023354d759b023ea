set -u
# r05zn: the row table in the one-wave a_F path (bfrt_flip_wave): parity, A/B against the last commit, stamps
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_bfrt_global.py tests/test_gpu_mip.py tests/test_gpu_ngpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05zn.log 2>&1 || { tail -30 gpurun_out/pytest_r05zn.log; exit 1; }
tail -3 gpurun_out/pytest_r05zn.log
bash tools/ab_sparse.sh r05zn "prev base" 2 || exit 5
bash tools/stamps_sparse.sh r05zn || exit 6
grep "k_dual_bfrt" gpurun_out/stamps_r05zn.txt
grep "k_dual_bfrt a_F by" gpurun_out/stamps_r05zn.txt
