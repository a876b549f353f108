#!/bin/bash
# Parity of the column-chain variants (V="la la_sc1 sc1": variants/libmam_gpu_<v>.so) on the dense LBA tests, then
# their ring batch / lone window times.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/la
mkdir -p $O
cd $R
NPZ=$R/variants/ring_windows.npz
for v in ${V:-la la_sc1 sc1}; do
  L=$R/variants/libmam_gpu_$v.so
  MAM3SLAM_GPU_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py -k "dense" > $O/tests_$v.log 2>&1
  echo "$v: $(tail -1 $O/tests_$v.log)"
  MAM3SLAM_GPU_LIB=$L timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode batch --solves 8 > $O/b_$v.log 2>&1 || { tail -5 $O/b_$v.log; exit 1; }
  echo "  $(grep 'batch of' $O/b_$v.log)"
  MAM_LBA_MW=2 MAM3SLAM_GPU_LIB=$L timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 2 --solves 6 > $O/s_$v.log 2>&1 || { tail -5 $O/s_$v.log; exit 1; }
  grep single $O/s_$v.log | sed 's/^/  /'
done
