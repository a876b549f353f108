#!/bin/bash
# c2 quick lines with LocalMapping's stage events inside the timed region (--profile-timed) and outside (default),
# alternated twice.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for V in off on; do
    F=""; [ $V = on ] && F="--profile-timed"
    timeout -k 10 300 python bench.py --config c2 $F --no-cpu-baseline --no-latency --no-pose --no-sin --steps 10 > $O/pt${V}_$rep.json 2> $O/pt${V}_$rep.err || { tail -5 $O/pt${V}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/pt${V}_$rep.json')); print('timed-events=$V rep $rep', round(d['value']), round(d['lba']['ms_per_step_wall'],3), {k: round(v,1) for k,v in d['lba']['stage_ms_total'].items()}, round(d['new_keyframes']['ms_per_step_triangulation'],3))"
  done
done
