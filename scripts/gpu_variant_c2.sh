#!/bin/bash
# c2 bench (no CPU baseline / side sections) for the default library and variants (VARS="name ...", built by
# scripts/build_variant.sh), plus the standalone triangulation bench for each.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for V in default ${VARS:-}; do
  if [ $V = default ]; then L=""; else L="MAM3SLAM_GPU_LIB=$PWD/variants/libmam_gpu_$V.so"; fi
  env $L timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-pose --no-sin --steps 12 > $O/var_$V.json 2> $O/var_$V.err || { tail -3 $O/var_$V.err; exit 1; }
  env $L timeout -k 10 120 python scripts/tri_bench.py --reps 10 > $O/vtri_$V.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/var_$V.json')); t=json.load(open('$O/vtri_$V.json')); print('$V', round(d['value']), 'lba', round(d['lba']['ms_per_step_wall'],2), 'tri', round(d['new_keyframes']['ms_per_step_triangulation'],3), 'tri alone', round(t['ms_median'],3), t['parity_bad_pairs'])"
done
