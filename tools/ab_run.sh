set -u
VARIANTS="base pfq1 pfq2 nar64 pft4 nar64pfq1 base" bash tools/ab_libs.sh || exit 1
for V in base pfq1 nar64pfq1; do
  if [ $V = base ]; then L=easylp_amd/lib/libeasylp_hip.so; else L=easylp_amd/lib/libeasylp_hip_$V.so; fi
  ELP_STAMPS=1 ELP_LIB_PATH=$PWD/$L timeout -k 10 120 python bench.py --steps 0 --warmup 0 --window 1 --c4 0 --sparse 0 --no-cpu --compare-rules 0 > gpurun_out/st_$V.json 2> gpurun_out/st_$V.err || exit 2
  echo $V; grep stamps gpurun_out/st_$V.err
done
