#!/bin/bash
# PoseOptimization per library variant (variants/libmam_gpu_<name>.so): the pose parity tests, then the c2 pose
# bench at batch 16 (a tracking lane's launch) and batch 1. Usage: bash scripts/gpu_pose_variants.sh n1 n2 ...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for n in "$@"; do
  export MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_pose_gpu.py > $O/pv_$n.log 2>&1 || { tail -20 $O/pv_$n.log; exit 1; }
  for B in 16 1; do
    timeout -k 10 120 python scripts/pose_bench.py --config c2 --batch $B --reps 10 > $O/pv_${n}_$B.json 2> $O/pv_${n}_$B.err || { tail -5 $O/pv_${n}_$B.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/pv_${n}_$B.json')); print('$n', 'batch $B', round(d['ms_per_batch_launch'], 4), 'ms', 'its', d['iterations_per_frame'], 'trials', d['lm_trials_per_frame'])"
  done
done
