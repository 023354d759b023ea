set -u
# r05w: the zero rule in the Newton-Schulz update (chunks skipped) and the GJ pivot column kept in registers: the whole GPU suite, then the feasible-start
# LP A/B against the last commit
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05w.log 2>&1 || { tail -30 gpurun_out/pytest_r05w.log; exit 1; }
tail -3 gpurun_out/pytest_r05w.log
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05w_feas "prev base" 1 || exit 4
bash tools/ab_sparse.sh r05w "prev base" 1 || exit 5
