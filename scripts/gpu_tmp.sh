set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_orb_gpu.py tests/test_golden.py tests/test_match_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1; st=$?; tail -3 $O/pt.log; [ $st -ne 0 ] && exit $st
timeout -k 10 200 python bench.py --batch 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-pose > $O/b1.json 2>$O/b1.err || exit $?
python3 -c "import json;d=json.load(open('$O/b1.json'));print('B1 lat', round(d['latency_ms_per_frame_b1'],4), {k:round(v,4) for k,v in d['stage_ms_per_step'].items()})"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-latency --no-pose > $O/b256.json 2>$O/b256.err || exit $?
python3 -c "import json;d=json.load(open('$O/b256.json'));print('B256', round(d['value']), {k:round(v,4) for k,v in d['stage_ms_per_step'].items()})"
