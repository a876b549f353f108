#!/bin/bash
# Lone-window LocalBundleAdjustment wall time per library variant (variants/libmam_gpu_<name>.so) and the LDL^T phase
# counters of the lprof variant. Usage: bash scripts/gpu_lba_variants.sh name1 name2 ...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for n in "$@"; do
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so timeout -k 10 200 python scripts/lba_bench.py --world --solves 10 --batch 32 > $O/var_$n.json 2> $O/var_$n.err || { tail -20 $O/var_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/var_$n.json')); print('$n', 'lone', round(d['ms_per_solve_median'],3), {k: round(v,3) for k,v in d['stage_ms_per_solve'].items()}, 'b1', round(d['device_batch_1']['ms_per_batch_median'],3), 'b32', round(d['device_batch_32']['ms_per_batch_median'],3), 'it', d['iterations'], d['trials'])"
  grep "ldlt cycles" $O/var_$n.err | tail -1
done
