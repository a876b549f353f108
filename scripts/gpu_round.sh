#!/bin/bash
# One GPU session: parity tests, the default bench line, a kernel-trace profile of the bench (--lanes 1 --batch 64 --no-latency:
# standalone 64-frame launches, as bench.py's serialised stage-timing pass measures them), and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass on gfx950) used for roofline.traffic.
# Stops at the first step that faults, aborts or times out (anything other than exit 0/1 from pytest).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
CFG=${1:-c1}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"; tail -5 $O/pytest_gpu.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
timeout -k 10 400 python bench.py --config $CFG > $O/bench_$CFG.json 2> $O/bench_$CFG.err || exit $?
cat $O/bench_$CFG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --lanes 1 --batch 64 --no-latency > $O/prof_$CFG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --lanes 1 --batch 64 --no-latency --steps 4 --warmup 1 > $O/pmc_fetch_$CFG.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --lanes 1 --batch 64 --no-latency --steps 4 --warmup 1 > $O/pmc_write_$CFG.log 2>&1 || exit $?
echo done
