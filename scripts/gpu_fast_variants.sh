set -u
cd $GRAFT_REPO_ROOT
for V in default ft128 ft512; do
  if [ $V = default ]; then L=""; else L="MAM3SLAM_GPU_LIB=$PWD/variants/libmam_gpu_$V.so"; fi
  env $L timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline --no-latency --no-pose --no-sin --steps 10 > gpurun_out/fv_$V.json 2> gpurun_out/fv_$V.err || { tail -5 gpurun_out/fv_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fv_$V.json')); print('$V', round(d['value']), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
done
