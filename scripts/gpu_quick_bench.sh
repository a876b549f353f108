#!/bin/bash
# Quick stage-time comparison of the tracking path: c1 and c2 bench lines without the CPU baseline and side sections.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-q}
mkdir -p $O
cd $R
for CFG in ${CFGS:-c1 c2}; do
  timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-latency --no-pose --no-sin --steps ${STEPS:-10} > $O/${T}_$CFG.json 2> $O/${T}_$CFG.err || { tail -5 $O/${T}_$CFG.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${T}_$CFG.json')); print('$CFG', round(d['value']), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()}, 'frac', round(d['roofline']['frac'],4), d.get('parity'))"
done
