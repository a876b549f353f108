#!/bin/bash
# k_pyr_flat output rows per thread (MAM_PYR_RQ 1 / 2 / 4): parity of the ORB tests, then the c1 / c2 pyramid stage.
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
for RQ in 2 4; do
  MAM_PYR_RQ=$RQ timeout -k 10 300 python -m pytest tests/test_orb_gpu.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pyr_t$RQ.log 2>&1 || { tail -20 gpurun_out/pyr_t$RQ.log; exit 1; }
  tail -1 gpurun_out/pyr_t$RQ.log
done
for CFG in c1 c2; do for RQ in 1 2 4; do
  MAM_PYR_RQ=$RQ timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-latency --no-pose --no-sin --steps 8 > gpurun_out/pyr_$CFG$RQ.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pyr_$CFG$RQ.json')); print('$CFG rq $RQ', round(d['value']), 'pyr', round(d['stage_ms_per_step']['pyramid'],3), d['parity']['extract_bit_exact'])"
done; done
