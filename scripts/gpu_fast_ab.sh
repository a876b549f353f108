#!/bin/bash
# FAST variants: the ORB parity tests against the first variant, then c1 / c2 bench lines per variant (alternated) with
# the FAST stage time. Usage: bash scripts/gpu_fast_ab.sh name1 name2 ...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$1.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_orb_gpu.py tests/test_golden.py > $O/fab_tests.log 2>&1 || { tail -20 $O/fab_tests.log; exit 1; }
tail -1 $O/fab_tests.log
for r in 1 2; do
  for n in "$@"; do
    for C in c1 c2; do
      MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$n.so timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-latency > $O/fab_${n}_${C}_$r.json 2> $O/fab_${n}_${C}_$r.err || { tail -20 $O/fab_${n}_${C}_$r.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/fab_${n}_${C}_$r.json'))
print('$n', '$C', $r, round(d['value']), round(d['ms_per_step'], 3), 'fast', round(d['stage_ms_per_step'].get('fast', 0), 3), 'launch', round(d['roofline']['avg_launch_ms'], 4), d['roofline']['kernel'], 'parity', d.get('parity_ok'))"
    done
  done
done
