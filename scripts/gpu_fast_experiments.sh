#!/bin/bash
# FAST timing experiments (variants built by scripts/build_variant.sh with -DMAM_FAST_EXPERIMENT=<bits>, see
# k_fast_cells): fx1 = trivial strength (one difference instead of the circle test), fx2 = return after the ROI
# staging, fx4 = return at once; default = the full kernel; stage pass of the c1 bench.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for CFG in ${CFGS:-c1}; do
for V in ${VARS:-default fx1 fx2 fx4}; do
  if [ $V = default ]; then L=""; else L="MAM3SLAM_GPU_LIB=$PWD/variants/libmam_gpu_$V.so"; fi
  env $L timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-latency --no-pose --no-sin --steps 6 > $O/fx_${CFG}_$V.json 2> $O/fx_${CFG}_$V.err || { tail -2 $O/fx_${CFG}_$V.err; }
  python3 -c "import json; d=json.load(open('$O/fx_${CFG}_$V.json')); print('$CFG $V fast', round(d['stage_ms_per_step']['fast'],3))" 2>/dev/null || echo "$CFG $V failed"
done
done
