#!/bin/bash
# Fuse / distinctive-descriptor parity, matcher regression, host API end to end
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_fuse_gpu.py tests/test_match_gpu.py tests/test_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_fuse.log 2>&1
rc=$?
tail -25 $O/pytest_fuse.log
exit $rc
