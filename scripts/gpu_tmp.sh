#!/bin/bash
# ORB parity, then c1 at 512 frames per step (the last frame's last row read past the caller's buffer before)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_orb_gpu.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_orb.log 2>&1
rc=$?
tail -2 $O/pytest_orb.log
[ $rc -eq 0 ] || exit $rc
for A in "--lanes 4 --batch 512" "--lanes 8 --batch 512" "--lanes 4 --batch 256"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-pose --no-sin --no-latency $A > $O/sweep.json 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sweep.json')); print('$A', round(d['value']), round(d['ms_per_step'],3))"
done
