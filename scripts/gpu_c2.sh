#!/bin/bash
# c2 session: the c2 bench line (extract + match + concurrent LocalBundleAdjustment + exchange), then the LBA
# parity tests, the standalone LBA timing and its kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
bash $R/scripts/gpu_lba.sh
