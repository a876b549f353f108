#!/bin/bash
# c2 with LBA variants (LDL^T threads) + LBA parity
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_lba2.log 2>&1 || { tail -20 $O/pytest_lba2.log; exit 1; }
tail -1 $O/pytest_lba2.log
for V in base l1024 l256; do
  if [ $V = base ]; then L=""; else L=$R/build/libmam_gpu_$V.so; fi
  MAM3SLAM_GPU_LIB=$L timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-pose --no-sin > $O/c2_$V.json 2> $O/c2_$V.err || { tail -5 $O/c2_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$V.json')); print('$V', round(d['value']), round(d['ms_per_step'],3), round(d['lba']['ms_per_solve_wall'],3))"
  MAM3SLAM_GPU_LIB=$L timeout -k 10 300 python scripts/lba_bench.py > $O/lba_$V.json 2>&1 && python -c "import json; d=json.load(open('$O/lba_$V.json')); print('$V standalone', round(d['ms_per_solve_median'],3), d['stage_ms_per_solve'])"
done
