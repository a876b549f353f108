#!/bin/bash
# Standalone LocalBundleAdjustment: world windows batched 32 per launch (the bench's LocalMapping leg), timings and
# a kernel trace. Usage: bash scripts/gpu_lba_prof.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-lba}
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/lba_bench.py --world --batch 32 --solves 6 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16   # what bench.py sets for itself; under rocprofv3 the profiler initialises HIP first
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$T -o run -- python3 $R/scripts/lba_bench.py --world --batch 32 --solves 4 > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
python3 - $O/prof_$T/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:24]:
    print(x["Name"][:60].ljust(60), x["Calls"].rjust(6), "%9.1f us avg" % (float(x["AverageNs"]) / 1e3), x["Percentage"][:5])
PY
