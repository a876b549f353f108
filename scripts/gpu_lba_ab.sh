#!/bin/bash
# LBA parity tests against a library variant, then the lone-window / batch timings of several variants.
# Usage: bash scripts/gpu_lba_ab.sh <test-variant> name1 name2 ...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
TV=$1; shift
MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$TV.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py tests/test_kb8_gpu.py tests/test_golden.py > $O/ab_tests_$TV.log 2>&1 || { tail -30 $O/ab_tests_$TV.log; exit 1; }
tail -2 $O/ab_tests_$TV.log
bash scripts/gpu_lba_variants.sh "$@"
