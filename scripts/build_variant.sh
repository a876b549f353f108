#!/bin/bash
# A variant of libmam_gpu.so with extra compile flags (profiling counters, tuning macros), for experiments:
#   bash scripts/build_variant.sh <name> -DMAM_LDLT_PROFILE ...  ->  variants/libmam_gpu_<name>.so
# then run with MAM3SLAM_GPU_LIB=variants/libmam_gpu_<name>.so.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/variants
C=$R/mam3slam_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -Werror=return-type "$@" \
  -o $R/variants/libmam_gpu_$N.so $C/orb_extract.hip $C/${MATCH_SRC:-match.hip} $C/lba.hip $C/exchange.hip $C/pose.hip $C/bow.hip $C/streams.hip $C/ringmap.hip
