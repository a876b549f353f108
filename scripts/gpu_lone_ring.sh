#!/bin/bash
# One ring window alone (the c2 north star's LBA term): the register form (MAM_LBA_REG=1) against the default, then a
# kernel trace of the default summarised per solve (scripts/lone_trace.py).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/lone
mkdir -p $O
cd $R
NPZ=$R/variants/ring_windows.npz
for reg in 1 0; do
  MAM_LBA_REG=$reg timeout -k 10 120 python3 scripts/ring_window_replay.py $NPZ --mode single --windows 4 --solves 6 > $O/reg$reg.log 2>&1 || { tail -5 $O/reg$reg.log; exit 1; }
  echo "MAM_LBA_REG=$reg"; grep single $O/reg$reg.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 $R/scripts/ring_window_replay.py $NPZ --mode single --windows 1 --solves 6 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 $R/scripts/lone_trace.py $(find $O/tr -name '*kernel_trace.csv' -print -quit) --skip 2 | tail -14
