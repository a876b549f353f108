#!/bin/bash
# smoke(), then the ring batch at 8 / 12 / 16 workgroups a dense window (variants/libmam_gpu_g<N>.so; 8 = in-tree).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for v in main g12 g16 main; do
  L=$R/mam3slam_amd/libmam_gpu.so; [ $v = main ] || L=$R/variants/libmam_gpu_$v.so
  MAM3SLAM_GPU_LIB=$L timeout -k 10 120 python3 scripts/ring_window_replay.py variants/ring_windows.npz --mode batch --solves 8 > gpurun_out/g_$v.log 2>&1 || { tail -5 gpurun_out/g_$v.log; exit 1; }
  echo "$v: $(grep 'batch of' gpurun_out/g_$v.log)"
done
