#!/bin/bash
# Fuse timing variants: base / no window scan / logf
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for V in base fz1 fz2; do
  if [ $V = base ]; then L=""; else L=$R/build/libmam_gpu_$V.so; fi
  MAM3SLAM_GPU_LIB=$L timeout -k 10 300 python scripts/fuse_bench.py --config c2 > $O/fz_$V.json 2> $O/fz_$V.err || { tail -20 $O/fz_$V.err; exit 1; }
  echo $V; cat $O/fz_$V.json
done
