#!/bin/bash
# Per-column timestamps of the dataflow LDL^T (MAM_LDLT_TRACE variants) and lone-window timings of library variants:
# bash scripts/gpu_ldlt_trace.sh <trace variant>... -- <timing variant>...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
tv=1
for n in "$@"; do
  if [ "$n" = "--" ]; then tv=0; continue; fi
  if [ $tv = 1 ]; then
    MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so timeout -k 10 120 python scripts/lba_bench.py --world --solves 3 > $O/lt_$n.json 2> $O/lt_$n.err || { tail -5 $O/lt_$n.err; exit 1; }
    echo "== $n"; grep ltrace $O/lt_$n.err | tail -19
  else
    bash scripts/gpu_lba_variants.sh $n || exit 1
  fi
done
