#!/bin/bash
# c2 quick bench lines at 2 / 4 / 8 tracking lanes (--lanes), alternated twice.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for NL in 4 2 8; do
    timeout -k 10 300 python bench.py --config c2 --lanes $NL --no-cpu-baseline --no-latency --no-pose --no-sin --steps 10 > $O/lanes${NL}_$rep.json 2> $O/lanes${NL}_$rep.err || { tail -5 $O/lanes${NL}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lanes${NL}_$rep.json')); print('lanes=$NL rep $rep', round(d['value']), round(d['lba']['ms_per_step_wall'],3))"
  done
done
