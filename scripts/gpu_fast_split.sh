#!/bin/bash
# FAST phase split on one standalone 64-frame c2 launch: library variants that stop after the cell setup (fx4), the
# ROI staging (fx2), the strength map (fx16), the NMS + counts (fx8), or replace the circle test by one difference
# (fx1) — timing only, their outputs are not candidates. Usage: bash scripts/gpu_fast_split.sh [cfg]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
CFG=${1:-c2}
mkdir -p $O
cd $R
for rep in 1 2; do
for n in base fx4 fx2 fx16 fx8 fx1; do
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so timeout -k 10 120 python scripts/fast_stage.py --config $CFG > $O/fs_$n.json 2> $O/fs_$n.err || { tail -5 $O/fs_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/fs_$n.json')); print('$n', round(d['ms_per_launch']['fast'], 4))"
done
done
