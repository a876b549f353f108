#!/bin/bash
# GPU parity suite (optionally a subset: TESTS="tests/test_x.py ..."), one pytest process, per-test timeout.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
st=$?
tail -30 $O/pytest_gpu.log
exit $st
