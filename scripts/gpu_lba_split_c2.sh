#!/bin/bash
# c2 quick bench lines at 1 / 2 / 3 LBA stream groups (MAM_LBA_SPLIT), alternated twice.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for G in 2 1 3; do
    MAM_LBA_SPLIT=$G timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-latency --no-pose --no-sin --steps 10 > $O/split${G}_$rep.json 2> $O/split${G}_$rep.err || { tail -5 $O/split${G}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/split${G}_$rep.json')); print('G=$G rep $rep', round(d['value']), round(d['lba']['ms_per_step_wall'],3))"
  done
done
