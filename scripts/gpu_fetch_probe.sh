#!/bin/bash
# FETCH_SIZE scale per load shape (known bytes): rocprofv3 --pmc FETCH_SIZE over scripts/fetch_probe.py
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_probe -o run -- python3 $R/scripts/fetch_probe.py > $O/fetch_probe.json 2> $O/fetch_probe.err || { tail -5 $O/fetch_probe.err; exit 1; }
python3 $R/scripts/fetch_probe_summary.py $O/pmc_probe $O/fetch_probe.json | tee $O/fetch_probe_summary.json
