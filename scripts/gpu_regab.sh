#!/bin/bash
# The dense-window factorization forms on the dumped ring windows (variants/ring_windows.npz): register form
# (MAM_LBA_REG=1), HBM form (the default); each under a
# kernel trace, the top kernels' mean launch time printed; any other name: variants/libmam_gpu_<name>.so.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/regab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-reg reg_g0 hbm}; do
  case $v in
    reg) E="MAM_LBA_REG=1" ;;
    hbm) E="" ;;
    rprof) E="MAM_LBA_REG=1 MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_rprof.so" ;;
    *) E="MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so" ;;   # a library variant
  esac
  env $E timeout -k 10 180 python3 -u $R/scripts/ring_window_replay.py $R/variants/ring_windows.npz --mode batch --solves 6 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  echo "-- $v: $(grep 'batch of' $O/$v.log)"; grep -E "^nt |reg ldlt" $O/$v.log | tail -12
  [ -n "$E" ] && export $E
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 $R/scripts/ring_window_replay.py $R/variants/ring_windows.npz --mode batch --solves 4 > $O/tr_$v.log 2>&1 || { tail -5 $O/tr_$v.log; exit 1; }
  unset MAM_LBA_REG MAM3SLAM_GPU_LIB
  python3 - $O/tr_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("  ", x["Name"][:50].ljust(50), x["Calls"].rjust(6), "%9.1f avg us" % (float(x["AverageNs"]) / 1e3), "%8.2f tot ms" % (float(x["TotalDurationNs"]) / 1e6))
PY
done
