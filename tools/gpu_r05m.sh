set -u
# r05m: the primal CSC pricing prefetch (base) against the r04 staging loop (pf0), with and without the
# sparse inverse update; the dual BFRT's stamps without trailing update workgroups
LP=kkt_feasible_20000x100000 bash tools/ab_sparse.sh r05m_feas "base pf0 pf0@ELP_SRU=0" 1 || exit 4
bash tools/stamps_sparse.sh r05m || exit 5
