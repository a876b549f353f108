#!/bin/bash
# B=1 latency timeline: the bench at --batch 1 (its latency section replays the single-frame graph 55 times) under a
# kernel trace, then the per-frame kernel durations / gaps (scripts/profile_summary.py gaps).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --batch 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b1.json 2> $O/b1.err || exit $?
cat $O/b1.json
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_b1 -o run -- python3 $R/bench.py --batch 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof_b1.log 2>&1 || exit $?
python3 $R/scripts/profile_summary.py gaps $O/prof_b1/run_kernel_trace.csv
