#!/bin/bash
# Single-frame ORBextractor latency per config (scripts/extract_latency.py), its kernel trace, and (when built) the
# DistributeOctTree phase counters of the -DMAM_DIST_PROFILE variant (bash scripts/build_variant.sh distprof
# -DMAM_DIST_PROFILE).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/xlat
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/scripts/extract_latency.py --out $O/latency.json > $O/latency.log 2>&1 || { cat $O/latency.log; exit 1; }
cat $O/latency.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 -u $R/scripts/extract_latency.py --reps 100 --configs ${TRACE_CONFIGS:-c1,c2} > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:30]:
    print(x["Name"][:60].ljust(60), x["Calls"].rjust(6), "%9.1f us avg" % (float(x["AverageNs"]) / 1e3), "%8.1f us min" % (float(x["MinNs"]) / 1e3), x["Percentage"][:5])
PY
if [ -f $R/variants/libmam_gpu_distprof.so ]; then
  MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_distprof.so timeout -k 10 300 python3 -u $R/scripts/extract_latency.py --reps 100 > $O/distprof.log 2>&1
  grep "distribute cycles\|^c" $O/distprof.log | head -30 || tail -5 $O/distprof.log
fi
