#!/bin/bash
# Kernel trace of one config's bench run and its leg-overlap table (scripts/timeline.py); QUEUES sets
# GPU_MAX_HW_QUEUES (default: the box's). Usage: bash scripts/gpu_overlap_trace.sh <config> <tag>
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
C=$1; T=$2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "${QUEUES:-}" ] && export GPU_MAX_HW_QUEUES=$QUEUES
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/prof_$T -o run -- python3 $R/bench.py --config $C --no-cpu-baseline --steps 12 --warmup 3 --no-latency --no-pose --no-sin --no-overlap > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
python3 $R/scripts/timeline.py $O/prof_$T/run_kernel_trace.csv > $O/timeline_$T.txt
tail -3 $O/timeline_$T.txt
