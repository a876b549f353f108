#!/bin/bash
# Tracking-stage comparison of library variants (VARS="name ...", built by scripts/build_variant.sh) on c1 and c2.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for CFG in ${CFGS:-c1 c2}; do
for V in default ${VARS:-}; do
  if [ $V = default ]; then L=""; else L="MAM3SLAM_GPU_LIB=$PWD/variants/libmam_gpu_$V.so"; fi
  env $L timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-latency --no-pose --no-sin --steps 8 > $O/vt_${CFG}_$V.json 2> $O/vt_${CFG}_$V.err || { tail -3 $O/vt_${CFG}_$V.err; continue; }
  python3 -c "import json; d=json.load(open('$O/vt_${CFG}_$V.json')); p=d.get('parity',{}); print('$CFG $V', round(d['value']), {k: round(v,3) for k,v in d['stage_ms_per_step'].items() if k in ('fast','blur','describe','distribute','pyramid')}, 'exact', p.get('extract_bit_exact'))"
done
done
