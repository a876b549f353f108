#!/bin/bash
# Round-6 session: the GPU suite, the c2 bench line, and the Schur kernel variants on the dumped ring windows.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 600 python3 bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_c2.json'))
print('c2', d['value'], d['ms_per_step'], d.get('parity_ok'), 'LM alone', d['overlap']['local_mapping_only_ms_per_step'], 'ring batch', d['ring_lba']['ms_per_batch'])
print('roofline_lba', d['roofline_lba']['avg_launch_ms'], d['roofline_lba']['frac']); print('schur', d['roofline_lba_schur'])"
for v in ${LV:-}; do
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 scripts/ring_window_replay.py variants/ring_windows.npz --mode batch --solves 8 > $O/schur_$v.log 2>&1 || { tail -5 $O/schur_$v.log; exit 1; }
  echo "$v: $(grep 'batch of' $O/schur_$v.log)"
done
timeout -k 10 120 python3 scripts/ring_window_replay.py variants/ring_windows.npz --mode batch --solves 8 > $O/schur_main.log 2>&1 && echo "main: $(grep 'batch of' $O/schur_main.log)"
