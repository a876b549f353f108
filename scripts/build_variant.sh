#!/bin/bash
# Build a kernel-variant copy of libmam_gpu.so: scripts/build_variant.sh NAME -DMACRO=V ... -> build/libmam_gpu_NAME.so
# (load it with MAM3SLAM_GPU_LIB=build/libmam_gpu_NAME.so; the in-tree product library is untouched)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/build
C=$R/mam3slam_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-function "$@" -o $R/build/libmam_gpu_$N.so \
  $C/orb_extract.hip $C/match.hip $C/lba.hip $C/exchange.hip $C/pose.hip $C/bow.hip
echo $R/build/libmam_gpu_$N.so
