#!/bin/bash
# Build a library variant for tools/ab_libs.sh: tools/build_variant.sh NAME "-DKNOB=V ..." [SRC_DIR]
# (SRC_DIR: another checkout of easylp_amd/csrc, e.g. an older commit's sources)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=${2:-}; SRC=${3:-$ROOT/easylp_amd/csrc}
cd "$SRC"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-result \
  -Wno-pass-failed $DEFS -I"$ROOT/easylp_amd/csrc" -o "$ROOT/easylp_amd/lib/libeasylp_hip_$NAME.so" \
  elp_api.hip elp_kernels.hip elp_comm.hip elp_resident.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$ROOT/easylp_amd/lib/libeasylp_hip_$NAME.so"
