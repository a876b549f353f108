#!/bin/bash
# Parity suite + one bench line (config $1, default c2) + its kernel trace. Stops at the first failing GPU step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
CFG=${1:-c2}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --config $CFG ${BENCH_ARGS:-} > $O/bench_$CFG.json 2> $O/bench_$CFG.err || { tail -20 $O/bench_$CFG.err; exit 1; }
cat $O/bench_$CFG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof_$CFG.log 2>&1 || exit 1
head -20 $O/prof_$CFG/run_kernel_stats.csv | cut -c1-160
