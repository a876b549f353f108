#!/bin/bash
# 32-window ring LBA batch (the dumped windows, scratch/ring_windows.npz, x8) per library variant: RV="main st64 ...";
# "main" = the in-tree build, "env:VAR=value" = the in-tree build with that environment, others
# variants/libmam_gpu_<name>.so. MODE=single: the lone first window instead. Stops at the first failure.
R=$(cd "$(dirname "$0")/.." && pwd)
for v in ${RV:-main}; do
    lib=$R/mam3slam_amd/libmam_gpu.so; envs=""
    case $v in
        main) ;;
        env:*) envs=${v#env:} ;;
        *) lib=$R/variants/libmam_gpu_$v.so ;;
    esac
    tag=$(echo $v | tr ':=' '__')
    if [ "${MODE:-batch}" = single ]; then args="--mode single --windows 1 --solves 12"; else args="--mode batch --repeat ${REPEAT:-8} --solves 10"; fi
    env $envs MAM3SLAM_GPU_LIB=$lib timeout -k 10 120 python3 -u $R/scripts/ring_window_replay.py $R/scratch/ring_windows.npz \
        $args > $R/gpurun_out/ringvar_$tag.log 2>&1 || { tail -5 $R/gpurun_out/ringvar_$tag.log; exit 1; }
    echo "$v $(grep -E 'batch of|single 0' $R/gpurun_out/ringvar_$tag.log)"
done
