#!/bin/bash
# Same-box A/B of the world-window LBA batch of 32 across commits: bisect/<commit>/ holds that commit's package,
# scripts and headers (git archive) with its libraries built; "." is the working tree.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/bisect
mkdir -p $O
for rep in 1 2; do
  for d in ${DIRS:-$(ls -d $R/bisect/*) $R}; do
    n=$(basename $d); [ "$d" = "$R" ] && n=head
    (cd $d && timeout -k 10 200 python3 scripts/lba_bench.py --world --batch 32 --solves 10 > $O/${n}_$rep.json 2> $O/${n}_$rep.err) || { tail -5 $O/${n}_$rep.err; exit 1; }
    python3 -c "
import json, sys; d = json.load(open('$O/${n}_$rep.json'))
print('$n', $rep, 'batch32 %.3f' % d['device_batch_32']['ms_per_batch_median'], 'batch1 %.3f' % d['device_batch_1']['ms_per_batch_median'], 'lone %.3f' % d['ms_per_solve_median'])"
  done
done
