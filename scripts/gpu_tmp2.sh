#!/bin/bash
# ORB parity + c1 bench (FAST changes)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_orb_gpu.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_orb.log 2>&1
rc=$?
tail -3 $O/pytest_orb.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-pose --no-sin > $O/c1_fast.json 2> $O/c1_fast.err || { tail -5 $O/c1_fast.err; exit 1; }
python -c "import json; d=json.load(open('$O/c1_fast.json')); print(round(d['value']), round(d['ms_per_step'],3), d['latency_ms_per_frame_b1'], {k: round(v,3) for k,v in d['stage_ms_per_step'].items()}, d['roofline']['avg_launch_ms'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --no-pose --no-sin > $O/c1_fast2.json 2> $O/c1_fast2.err || { tail -5 $O/c1_fast2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c1_fast2.json')); print(round(d['value']), round(d['ms_per_step'],3), d['latency_ms_per_frame_b1'], {k: round(v,3) for k,v in d['stage_ms_per_step'].items()}, d['roofline']['avg_launch_ms'])"
