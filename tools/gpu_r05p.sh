set -u
# r05p: the sparse inverse update one workgroup per row: parity, A/B against the last commit on both
# sparse LPs, the primal CSC pricing timeline (ELP_PDBG build)
timeout -k 10 900 python -u -m pytest tests/test_gpu_spf.py tests/test_gpu_dual.py tests/test_gpu_csc.py tests/test_gpu_fuzz.py tests/test_gpu_basis.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05p.log 2>&1 || { tail -30 gpurun_out/pytest_r05p.log; exit 1; }
tail -3 gpurun_out/pytest_r05p.log
bash tools/ab_sparse.sh r05p "prev base" 1 || exit 3
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05p_feas "prev base base@ELP_SRU=0" 1 || exit 4
bash tools/gpu_r05n.sh || exit 6
