#!/bin/bash
# LBA session: parity tests, standalone timing, kernel trace of the standalone timing.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/test_lba_gpu.py tests/test_host_api.py tests/test_exchange.py -m gpu -q -p no:cacheprovider > $O/pytest_lba.log 2>&1
st=$?
echo "pytest exit $st"; tail -15 $O/pytest_lba.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
timeout -k 10 300 python scripts/lba_bench.py --oracle > $O/lba_bench.json 2> $O/lba_bench.err || exit $?
cat $O/lba_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_lba -o run -- python3 $R/scripts/lba_bench.py --solves 10 > $O/prof_lba.log 2>&1 || exit $?
echo done
