set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for V in distprof resprof; do
MAM3SLAM_GPU_LIB=$R/build/libmam_gpu_$V.so timeout -k 10 200 python bench.py --batch 1 --lanes 1 --steps 40 --warmup 2 --no-cpu-baseline --no-latency > $O/b1_$V.json 2>$O/b1_$V.err || exit $?
tail -4 $O/b1_$V.err
done
