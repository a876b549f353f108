#!/bin/bash
# c2 bench lines per library variant (variants/libmam_gpu_<name>.so), alternated: value, ms/step and the legs alone.
# Usage: bash scripts/gpu_c2_ab.sh name1 name2 ...   (BENCH_ARGS overrides the bench flags; ROUNDS the alternations)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in "$@"; do
    MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline --no-latency} > $O/ab_${n}_$r.json 2> $O/ab_${n}_$r.err || { tail -20 $O/ab_${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_${n}_$r.json')); o=d.get('overlap', {})
print('$n', $r, round(d['value']), round(d['ms_per_step'], 3), 'track', round(o.get('tracking_only_ms_per_step', 0), 3), 'lm', round(o.get('local_mapping_only_ms_per_step', 0), 3), 'pose', round(d['stage_ms_per_step'].get('pose', 0), 3), 'parity', d.get('parity_ok'))"
  done
done
