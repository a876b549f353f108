#!/bin/bash
# Lone LocalBundleAdjustment window: parity tests of the LBA, the standalone bench (lone + batches of 1 / 32) and a
# kernel trace of lone solves summarised per solve (scripts/lone_trace.py). Usage: bash scripts/gpu_lba_lone.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-lone}
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py tests/test_kb8_gpu.py tests/test_golden.py > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
fi
timeout -k 10 300 python scripts/lba_bench.py --world --batch 32 --solves 10 --oracle > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_$T -o run -- python3 $R/scripts/lba_bench.py --world --solves 6 > $O/prof_$T.log 2>&1 || { tail -20 $O/prof_$T.log; exit 1; }
python3 $R/scripts/lone_trace.py $(find $O/prof_$T -name '*kernel_trace.csv' -print -quit) --skip 2 | tee $O/${T}_trace.txt
