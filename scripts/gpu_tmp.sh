#!/bin/bash
# c2 bench with the LBA stream at the highest priority vs the default priority
set -u
O=${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out
mkdir -p $O
cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-pose > $O/c2_prio.json 2> $O/c2_prio.err || { tail -5 $O/c2_prio.err; exit 1; }
MAM_LBA_PRIORITY=0 timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-pose > $O/c2_noprio.json 2> $O/c2_noprio.err || { tail -5 $O/c2_noprio.err; exit 1; }
python - <<'PY'
import json
for f in ("c2_prio", "c2_noprio"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), d["ms_per_step"], d["lba"]["ms_per_solve_wall"])
PY
