#!/bin/bash
# k_struct_sort's long observation lists: the per-part cycle counts before (sortprof) and after (sortfixprof), the
# LBA / device-map parity tests on the in-tree library, and one ring window alone.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
NPZ=variants/ring_windows.npz
for v in sortfixprof; do
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 1 --solves 2 > gpurun_out/sp_$v.log 2>&1 || { tail -5 gpurun_out/sp_$v.log; exit 1; }
  echo "$v: $(grep struct_sort gpurun_out/sp_$v.log | tail -1)"
done
TESTS="tests/test_lba_gpu.py tests/test_ringmap_gpu.py" bash scripts/gpu_tests.sh || exit 1
timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 2 --solves 6 | grep single
