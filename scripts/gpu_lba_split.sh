#!/bin/bash
# The standalone batch of 32 world windows with 1..4 stream groups (MAM_LBA_SPLIT), alternating, one box.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
for rep in 1 2; do
for G in 1 2 3 4; do
  MAM_LBA_SPLIT=$G timeout -k 10 200 python scripts/lba_bench.py --world --batch 32 --solves 6 > $O/split_$G.json 2> $O/split_$G.err || { tail -5 $O/split_$G.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/split_$G.json')); print('split $G', d['device_batch_32']['ms_per_batch_median'])"
done
done
