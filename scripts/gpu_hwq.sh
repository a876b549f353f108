set -u
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for Q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-pose --no-sin --steps 12 > gpurun_out/hwq_$Q.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/hwq_$Q.json')); print('rep $rep queues $Q', round(d['value']), round(d['lba']['ms_per_step_wall'],2))"
done; done
