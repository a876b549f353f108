#!/bin/bash
# BoW parity + host API + bow bench
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_bow_gpu.py tests/test_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_bow.log 2>&1
rc=$?
tail -12 $O/pytest_bow.log
[ $rc -eq 0 ] || exit $rc
for CFG in c1 c2; do
  timeout -k 10 300 python scripts/bow_bench.py --config $CFG --oracle > $O/bow_$CFG.json 2> $O/bow_$CFG.err || { tail -20 $O/bow_$CFG.err; exit 1; }
  cat $O/bow_$CFG.json
done
