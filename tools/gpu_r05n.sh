set -u
# r05n: one pricing launch's workgroup timeline every 1000 iterations of the feasible-start LP (ELP_PDBG build)
rm -f gpurun_out/pdbg_feas.txt
ELP_PROBE_VERBOSE=2 ELP_PDBG_FILE=gpurun_out/pdbg_feas.txt ELP_PDBG_ITER=1000 ELP_LIB_PATH=$PWD/easylp_amd/lib/libeasylp_hip_pdbg.so timeout -k 10 200 python3 tools/sparse_probe.py kkt_feasible_20000x100000 || exit 3
python3 tools/pdbg_summary.py gpurun_out/pdbg_feas.txt
