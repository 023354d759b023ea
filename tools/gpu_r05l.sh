set -u
# r05l: the sparse rank-one inverse update (base) against the last commit (prev), ELP_SRU=0 and the
# one-entry dual pricing walk (dpb1)
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_spz.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_basis.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05l.log 2>&1 || { tail -30 gpurun_out/pytest_r05l.log; exit 1; }
tail -3 gpurun_out/pytest_r05l.log
bash tools/ab_sparse.sh r05l "prev base base@ELP_SRU=0 dpb1" 1 || exit 3
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05l_feas "prev base base@ELP_SRU=0" 1 || exit 4
