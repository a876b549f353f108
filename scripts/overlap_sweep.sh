#!/bin/bash
# c2 bench variants for the Tracking / LocalMapping overlap: hardware queues per process (GPU_MAX_HW_QUEUES) and the
# CU split between the legs (--cu-split). One bench process per variant, each under its own time limit; the sweep
# stops at the first failing variant. VARIANTS: "queues:split ..." (default below); EXTRA: more bench flags.
set -u
OUT=gpurun_out/sweep
mkdir -p $OUT
VARIANTS=${VARIANTS:-"4:0 8:0 16:0 8:2 8:4"}
EXTRA=${EXTRA:-"--no-latency --no-pose --no-sin --no-cpu-baseline"}
for v in $VARIANTS; do
    q=${v%%:*}; s=${v##*:}
    echo "=== queues $q split $s"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 -u bench.py --cu-split $s $EXTRA > $OUT/q${q}_s${s}.json 2> $OUT/q${q}_s${s}.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v failed rc=$rc"; tail -5 $OUT/q${q}_s${s}.err; exit $rc; fi
    python3 - $OUT/q${q}_s${s}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d.get("overlap") or {}
h = d.get("host_ms_per_step") or {}
print(f"value {d['value']:.0f} ms/step {d['ms_per_step']:.3f} tr_only {o.get('tracking_only_ms_per_step', 0):.3f} "
      f"lm_only {o.get('local_mapping_only_ms_per_step', 0):.3f} mapping_solve {h.get('mapping_solve', 0):.3f} "
      f"queue_wait {h.get('queue_wait', 0):.3f}")
PY
done
