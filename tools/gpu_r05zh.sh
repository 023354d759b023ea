set -u
# r05zh: k_dual_bfrt's fast tail without cptr's round trip (the column extent in
# the candidate record) and with the a_F clearing loads issued at launch start:
# parity, A/B against the last commit, stamps
timeout -k 10 1000 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_bfrt_global.py tests/test_gpu_mip.py tests/test_gpu_ngpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05zh.log 2>&1 || { tail -30 gpurun_out/pytest_r05zh.log; exit 1; }
tail -3 gpurun_out/pytest_r05zh.log
bash tools/ab_sparse.sh r05zh "prev base" 2 || exit 5
bash tools/stamps_sparse.sh r05zh || exit 6
grep "k_dual_bfrt" gpurun_out/stamps_r05zh.txt
