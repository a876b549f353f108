#!/bin/bash
# The device map's LBA windows (variants/ring_windows.npz, scripts/ringmap_probe.py --dump): the batch of 32 and one
# lone window per library variant (LV="main t1024 ...": variants/libmam_gpu_<v>.so, main = the in-tree library) and
# batch split (SPLITS="1 2 4"), plus a kernel trace of the default batch.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/dense
mkdir -p $O
export TMPDIR=/tmp
NPZ=${NPZ:-$R/variants/ring_windows.npz}
for v in ${LV:-main}; do
  lib=$R/mam3slam_amd/libmam_gpu.so
  [ "$v" = main ] || lib=$R/variants/libmam_gpu_$v.so
  for sp in ${SPLITS:-2}; do
    echo "-- $v split $sp"
    MAM_LBA_SPLIT=$sp MAM3SLAM_GPU_LIB=$lib timeout -k 10 180 python3 -u $R/scripts/ring_window_replay.py $NPZ --mode batch --solves 6 > $O/b_${v}_$sp.log 2>&1 || { tail -5 $O/b_${v}_$sp.log; exit 1; }
    grep "batch of" $O/b_${v}_$sp.log
  done
  MAM3SLAM_GPU_LIB=$lib timeout -k 10 180 python3 -u $R/scripts/ring_window_replay.py $NPZ --mode single --windows 1 --solves 8 > $O/s_$v.log 2>&1 || { tail -5 $O/s_$v.log; exit 1; }
  grep "single" $O/s_$v.log
done
if [ -n "${TRACE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/scripts/ring_window_replay.py $NPZ --mode batch --solves 4 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
  python3 - $O/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(x["Name"][:60].ljust(60), x["Calls"].rjust(6), "%9.1f avg us" % (float(x["AverageNs"]) / 1e3), "%8.2f tot ms" % (float(x["TotalDurationNs"]) / 1e6))
PY
fi
