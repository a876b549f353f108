#!/bin/bash
# Quick loop: given pytest files (default: all gpu tests), then the c1 bench without CPU baseline and its kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
TESTS=${TESTS:-tests}
timeout -k 10 900 python -m pytest $TESTS -m gpu -q -x -p no:cacheprovider > $O/pytest_quick.log 2>&1
st=$?
echo "pytest exit $st"; tail -25 $O/pytest_quick.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_quick.json 2> $O/bench_quick.err || exit $?
cat $O/bench_quick.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_quick -o run -- python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof_quick.log 2>&1 || exit $?
head -14 $O/prof_quick/run_kernel_stats.csv | cut -c1-150
