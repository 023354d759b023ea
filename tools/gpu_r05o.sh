set -u
# r05o: the one-candidate-per-lane BFRT rounds (bfrt_wave1): parity, stamps, A/B against the last
# commit; the primal CSC pricing timeline (ELP_PDBG build)
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05o.log 2>&1 || { tail -30 gpurun_out/pytest_r05o.log; exit 1; }
tail -3 gpurun_out/pytest_r05o.log
bash tools/stamps_sparse.sh r05o || exit 5
bash tools/ab_sparse.sh r05o "prev base" 1 || exit 3
bash tools/gpu_r05n.sh || exit 6
