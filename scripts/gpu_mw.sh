#!/bin/bash
# The column-chain factorization (k_ldlt_mw) on the dumped ring windows (variants/ring_windows.npz): the LBA parity
# tests, then batch of 32 and one window alone with the column-chain form (default) and the HBM form (MAM_LBA_MW=0),
# and the per-phase cycle counts of the mwprof variant (scripts/build_variant.sh mwprof -DMAM_MW_PROFILE).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/mw
mkdir -p $O
cd $R
NPZ=$R/variants/ring_windows.npz
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for mode in batch single; do
  for mw in 1 0; do
    A="--mode $mode --solves 8"; [ $mode = single ] && A="$A --windows 1"
    MAM_LBA_MW=$mw timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ $A > $O/${mode}_$mw.log 2>&1 || { tail -5 $O/${mode}_$mw.log; exit 1; }
    echo "$mode MAM_LBA_MW=$mw: $(grep -E 'ms per solve' $O/${mode}_$mw.log | head -1)"
  done
done
for v in ${LV:-}; do
  for mode in batch single; do
    A="--mode $mode --solves 8"; [ $mode = single ] && A="$A --windows 1"
    MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ $A > $O/${mode}_$v.log 2>&1 || { tail -5 $O/${mode}_$v.log; exit 1; }
    echo "$mode $v: $(grep -E 'ms per solve' $O/${mode}_$v.log | head -1)"
  done
done
if [ -f $R/variants/libmam_gpu_mwprof.so ]; then
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_mwprof.so timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode batch --solves 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
  grep "mw cycles" $O/prof.log | tail -1
fi
