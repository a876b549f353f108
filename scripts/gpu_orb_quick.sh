#!/bin/bash
# ORB parity tests (a subset via TESTS=...), then the single-frame extraction latency and its kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/orbq
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_orb_gpu.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
st=$?
tail -15 $O/pytest.log
[ $st -eq 0 ] || exit $st
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/scripts/extract_latency.py --out $O/latency.json > $O/latency.log 2>&1 || { cat $O/latency.log; exit 1; }
cat $O/latency.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 -u $R/scripts/extract_latency.py --reps 50 --configs ${TRACE_CONFIGS:-c1,c2} > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print(x["Name"][:60].ljust(60), x["Calls"].rjust(6), "%9.1f us avg" % (float(x["AverageNs"]) / 1e3), "%8.1f us min" % (float(x["MinNs"]) / 1e3), "%8.1f us max" % (float(x["MaxNs"]) / 1e3))
PY
