#!/bin/bash
# Schur variants on the ring batch; one ring window alone through the column-chain form with a workgroup per column
# (MAM_LBA_MW=2) against the HBM form (the default for a lone window).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
NPZ=variants/ring_windows.npz
for v in ${LV:-}; do
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode batch --solves 8 > $O/schur_$v.log 2>&1 || { tail -5 $O/schur_$v.log; exit 1; }
  echo "$v: $(grep 'batch of' $O/schur_$v.log)"
done
for mw in 2 0; do
  MAM_LBA_MW=$mw timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 3 --solves 6 > $O/lone_$mw.log 2>&1 || { tail -5 $O/lone_$mw.log; exit 1; }
  echo "MAM_LBA_MW=$mw"; grep single $O/lone_$mw.log
done
