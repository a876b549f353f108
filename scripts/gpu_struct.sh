#!/bin/bash
# LBA structure-build change check: LBA / KB8 / golden / host-API parity tests, the standalone LBA bench and a quick
# c2 bench line (tracking + LocalMapping). Usage: bash scripts/gpu_struct.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-struct}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lba_gpu.py tests/test_kb8_gpu.py tests/test_golden.py > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 python scripts/lba_bench.py --world --batch 32 --solves 10 > $O/${T}_lba.json 2> $O/${T}_lba.err || { tail -20 $O/${T}_lba.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${T}_lba.json')); print('lone', round(d['ms_per_solve_median'],3), {k: round(v,3) for k,v in d['stage_ms_per_solve'].items()}, 'b1', round(d['device_batch_1']['ms_per_batch_median'],3), 'b32', round(d['device_batch_32']['ms_per_batch_median'],3), 'it', d['iterations'], d['trials'], 'diff', d['max_point_rel_diff_vs_oracle'], d['same_control_flow'])"
CFGS=c2 bash scripts/gpu_quick_bench.sh $T || exit 1
