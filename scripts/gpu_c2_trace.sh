#!/bin/bash
# Kernel trace of the default c2 bench (tracking + LocalMapping concurrently): per-kernel time under load.
# Usage: bash scripts/gpu_c2_trace.sh [tag]   (BENCH_ARGS overrides the bench flags)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-c2t}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16   # what bench.py sets for itself; under rocprofv3 the profiler initialises HIP first
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$T -o run -- python3 $R/bench.py ${BENCH_ARGS:---no-cpu-baseline --steps 8 --warmup 2 --no-latency --no-pose --no-sin} > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
python3 - $O/prof_$T/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:40]:
    print(x["Name"][:60].ljust(60), x["Calls"].rjust(6), "%9.1f us avg" % (float(x["AverageNs"]) / 1e3), "%8.2f ms" % (float(x["TotalDurationNs"]) / 1e6), x["Percentage"][:5])
PY
