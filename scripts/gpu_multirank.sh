#!/bin/bash
# The multi-rank bench path on a one-GPU box: 2 ranks on GPU 0, the LBA write-back exchange over gloo
# (MAM_BENCH_ONE_DEVICE / MAM_DIST_BACKEND); c2 (64 streams per rank) and c3 (one agent per rank).
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
export MAM_BENCH_ONE_DEVICE=1 MAM_DIST_BACKEND=gloo
timeout -k 10 400 python bench.py --gpus 2 --config c2 --batch 64 --steps 4 --warmup 2 --no-cpu-baseline --no-latency --no-pose --no-sin > gpurun_out/mr_c2.json 2> gpurun_out/mr_c2.err || { tail -20 gpurun_out/mr_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/mr_c2.json').read().strip().splitlines()[-1]); print('c2 x2', d['n_gpus'], round(d['value']), d['lba']['exchange_bytes_per_step'], d.get('parity'))"
timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 8 --warmup 2 --no-cpu-baseline --no-latency --no-pose --no-sin > gpurun_out/mr_c3.json 2> gpurun_out/mr_c3.err || { tail -20 gpurun_out/mr_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/mr_c3.json').read().strip().splitlines()[-1]); print('c3 x2', d['n_gpus'], round(d['value']), d['config']['frames_per_step_per_gpu'], d.get('parity'))"
