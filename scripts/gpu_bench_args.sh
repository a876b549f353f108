#!/bin/bash
# Runs the c1 bench once per argument set in $ARGSETS (separated by ';') and prints value + stage times.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
i=0
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
for A in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $A > $O/bench_args_$i.json 2> $O/bench_args_$i.err || { tail -5 $O/bench_args_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']),round(d['ms_per_step'],4),round(d['latency_ms_per_frame_b1'],4),{k:round(v,4) for k,v in d['stage_ms_per_step'].items()})" $O/bench_args_$i.json "$A"
done
echo done
