#!/bin/bash
# The lookahead column-chain variant (variants/libmam_gpu_la.so): the LBA parity tests through it, then the ring batch
# and lone windows (MAM_LBA_MW=2) against the in-tree library.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/la
mkdir -p $O
cd $R
NPZ=$R/variants/ring_windows.npz
L=$R/variants/libmam_gpu_${V:-la}.so
MAM3SLAM_GPU_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in $L $R/mam3slam_amd/libmam_gpu.so; do
  MAM3SLAM_GPU_LIB=$lib timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode batch --solves 8 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "$(basename $lib) $(grep 'batch of' $O/b.log)"
  MAM_LBA_MW=2 MAM3SLAM_GPU_LIB=$lib timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 2 --solves 6 > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }
  grep single $O/s.log
done
