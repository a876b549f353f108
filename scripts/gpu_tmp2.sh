#!/bin/bash
# LBA (incl. merge schedule) + host API + pose
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_lba.log 2>&1
rc=$?
tail -12 $O/pytest_lba.log
exit $rc
