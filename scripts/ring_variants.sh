#!/bin/bash
# 32-window ring LBA batch (the dumped windows, scratch/ring_windows.npz, x8) per library variant: RV="main st64 ...";
# "main" = the in-tree build, others variants/libmam_gpu_<name>.so. Stops at the first failure.
R=$(cd "$(dirname "$0")/.." && pwd)
for v in ${RV:-main}; do
    lib=$R/variants/libmam_gpu_$v.so; [ $v = main ] && lib=$R/mam3slam_amd/libmam_gpu.so
    MAM3SLAM_GPU_LIB=$lib timeout -k 10 120 python3 -u $R/scripts/ring_window_replay.py $R/scratch/ring_windows.npz \
        --mode batch --repeat ${REPEAT:-8} --solves 10 > $R/gpurun_out/ringvar_$v.log 2>&1 || { tail -5 $R/gpurun_out/ringvar_$v.log; exit 1; }
    echo "$v $(grep 'batch of' $R/gpurun_out/ringvar_$v.log)"
done
