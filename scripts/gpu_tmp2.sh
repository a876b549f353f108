set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for cfg in "256 4" "256 8" "512 4" "512 8" "1024 8" "1024 16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --batch $1 --lanes $2 --no-cpu-baseline --no-latency --no-pose > $O/bl_$1_$2.json 2>$O/bl_$1_$2.err || { tail -3 $O/bl_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bl_$1_$2.json'));print('B $1 lanes $2', round(d['value']), round(d['ms_per_step'],3))"
done
