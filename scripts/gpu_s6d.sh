#!/bin/bash
# LBA parity tests on the round's code, then the ring batch per points-per-workgroup (MAM_LBA_PW) and batch split
# (MAM_LBA_SPLIT) on the dumped ring windows.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
NPZ=variants/ring_windows.npz
TESTS="tests/test_lba_gpu.py tests/test_ringmap_gpu.py" bash scripts/gpu_tests.sh || exit 1
for e in "X=0" "MAM_LBA_PW=4" "MAM_LBA_PW=2" "MAM_LBA_SPLIT=1" "MAM_LBA_SPLIT=4"; do
  env $e timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode batch --solves 8 > $O/pw.log 2>&1 || { tail -5 $O/pw.log; exit 1; }
  echo "$e: $(grep 'batch of' $O/pw.log)"
done
