set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash scripts/gpu_round.sh c1 || exit $?
bash scripts/gpu_c2.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -i "mfma\|FETCH_SIZE\|SQ_BUSY\|GRBM_GUI" $O/counters_list.txt | head -40
