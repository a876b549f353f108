#!/bin/bash
# Round-2 first session: GPU parity suite, the default (c2) bench line, c1, and a kernel trace of the default bench.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
st=$?
tail -5 $O/pytest_gpu.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 600 python bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
cat $O/bench_c1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_c2 -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 1
echo done
