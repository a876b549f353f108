#!/bin/bash
# The default bench line (c2 headline) without and with the CPU baseline leg skipped; kernel trace of the default run.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-c2}
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $O/bench_$T.json 2> $O/bench_$T.err || { tail -20 $O/bench_$T.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open('$O/bench_$T.json'))
print('value', d['value'], 'ms/step', d['ms_per_step']); print('stage', d.get('stage_ms_per_step')); print('lba', {k: d.get('lba',{}).get(k) for k in ('ms_per_step_wall','ms_per_window_wall','trials_mean')})
print('roofline', d['roofline']); print('parity', d.get('parity'))"
