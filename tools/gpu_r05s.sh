set -u
# r05s: k_dual_bfrt's fast tail (the candidates' columns loaded during the rounds, a_F from LDS):
# parity, stamps, A/B against the last commit
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_fuzz.py tests/test_gpu_bfrt_global.py tests/test_gpu_mip.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05s.log 2>&1 || { tail -30 gpurun_out/pytest_r05s.log; exit 1; }
tail -3 gpurun_out/pytest_r05s.log
bash tools/stamps_sparse.sh r05s || exit 5
bash tools/ab_sparse.sh r05s "prev base" 1 || exit 3
