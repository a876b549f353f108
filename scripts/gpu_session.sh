#!/bin/bash
# One GPU session of several parts (PARTS="orb lat lone bench" by default): the ORB parity tests + the motion retry
# test, the single-frame extraction latency and its kernel trace, the lone LocalBundleAdjustment trace, a c1 bench line.
# Every step under its own time limit; the session stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/sess
mkdir -p $O
export TMPDIR=/tmp
for part in ${PARTS:-orb lat lone bench bench2}; do
  echo "=== $part"
  case $part in
    orb)
      cd $R && timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_orb_gpu.py tests/test_track_gpu.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
      st=$?; tail -12 $O/pytest.log; [ $st -eq 0 ] || exit $st ;;
    lat)
      cd /tmp && timeout -k 10 300 python3 -u $R/scripts/extract_latency.py --out $O/latency.json > $O/latency.log 2>&1 || { cat $O/latency.log; exit 1; }
      cat $O/latency.log
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_lat -o run -- python3 -u $R/scripts/extract_latency.py --reps 50 --configs c1,c2 > $O/prof_lat.log 2>&1 || { tail -20 $O/prof_lat.log; exit 1; }
      python3 - $O/prof_lat/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(x["Name"][:58].ljust(58), x["Calls"].rjust(6), "%8.1f avg" % (float(x["AverageNs"]) / 1e3), "%8.1f min" % (float(x["MinNs"]) / 1e3), "%8.1f max" % (float(x["MaxNs"]) / 1e3))
PY
      ;;
    sweep)
      # single-frame extraction under implementation switches (env), c1 and c2, and the DistributeOctTree phase profile
      cd /tmp
      for v in "MAM_ORB_FORK=0" "MAM_PYR_BANDS=0" "MAM_PYR_BANDS=16" "MAM_PYR_BANDS=32" "MAM_ORB_FORK=0 MAM_PYR_BANDS=0" "MAM_FAST_CHUNKS=1" ${SWEEP_EXTRA:-}; do
        echo "-- $v"; env $v timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 100 --configs c1,c2 2>&1 | grep '^c'
      done
      if [ -f $R/variants/libmam_gpu_d2prof.so ]; then
        MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_d2prof.so timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 100 --configs c1,c2 > $O/d2prof.log 2>&1
        grep "d2prof" $O/d2prof.log | awk '!seen[$2 $3 $4]++' | head -24
      fi ;;
    pyr)
      # single-launch pyramid phase profile (cycles per workgroup) per band count, c1 and c2
      cd /tmp
      for nb in ${PYR_BANDS:-8 16 32 64}; do
        echo "-- MAM_PYR_BANDS=$nb"
        MAM_PYR_BANDS=$nb MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_pyrprof.so timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 60 --configs c1,c2 > $O/pyrprof_$nb.log 2>&1 || { tail -5 $O/pyrprof_$nb.log; exit 1; }
        grep "^c" $O/pyrprof_$nb.log; grep "pyrprof" $O/pyrprof_$nb.log | awk '!seen[$2 $3]++'
      done ;;
    agg)
      # DistributeOctTree count-pass aggregation variants (phase profile), and the host phases of mam_orb_extract
      cd /tmp
      for v in ${AGG_VARIANTS:-agg0 agg1 agg2 d2prof}; do
        echo "-- $v"
        MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 100 --configs c1,c2 > $O/agg_$v.log 2>&1 || { tail -5 $O/agg_$v.log; exit 1; }
        grep "^c" $O/agg_$v.log; grep "d2prof" $O/agg_$v.log | awk '!seen[$2 $3 $4]++' | grep -E " l0:| l7:"
      done
      ;;
    hostprof)
      cd /tmp
      for v in ${HOSTPROF_ENVS:-MAM_ORB_ZERO_COPY_OUT=1}; do
        echo "-- $v"
        env $v MAM_ORB_HOST_PROFILE=1 timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 400 --configs c1,c2 > $O/hostprof.log 2>&1 || { tail -5 $O/hostprof.log; exit 1; }
        grep -E "^c|orb host" $O/hostprof.log | awk '!seen[$1 $2 $3]++'
      done ;;
    ldlt)
      # the dataflow LDL^T of the lone window: per-column timestamps (MAM_LDLT_TRACE) and cycles per phase
      cd /tmp
      for v in ${LT_VARIANTS:-ltrace}; do
        echo "-- $v"
        MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_$v.so timeout -k 10 120 python3 $R/scripts/lba_bench.py --world --solves 3 > $O/lt_$v.json 2> $O/lt_$v.err || { tail -5 $O/lt_$v.err; exit 1; }
        grep -E "ltrace|ldlt cycles" $O/lt_$v.err | tail -${LT_COLS:-20}
      done ;;
    lbavar)
      # lone-window solve per library variant (LBA_VARIANTS: variants/libmam_gpu_<name>.so; "main" = the in-tree build)
      cd /tmp
      for v in ${LBA_VARIANTS:-main}; do
        lib=$R/variants/libmam_gpu_$v.so; [ $v = main ] && lib=$R/mam3slam_amd/libmam_gpu.so
        MAM3SLAM_GPU_LIB=$lib timeout -k 10 120 python3 $R/scripts/lba_bench.py --world --solves 12 > $O/lbavar_$v.json 2> $O/lbavar_$v.err || { tail -5 $O/lbavar_$v.err; exit 1; }
        python3 -c "
import json; d=json.loads(open('$O/lbavar_$v.json').read())
print('$v', 'median %.4f min %.4f' % (d['ms_per_solve_median'], d['ms_per_solve_min']), {k: round(v, 4) for k, v in d['stage_ms_per_solve'].items()})"
      done ;;
    sweep2)
      # DistributeOctTree phase profile per workgroup width; batch stage times with / without the FAST chunks
      cd /tmp
      for nt in 256 512 1024; do
        echo "-- MAM_DIST_NT=$nt"
        MAM_DIST_NT=$nt MAM3SLAM_GPU_LIB=$R/variants/libmam_gpu_d2prof.so timeout -k 10 120 python3 -u $R/scripts/extract_latency.py --reps 60 --configs c1,c2 > $O/d2prof_$nt.log 2>&1
        grep "^c" $O/d2prof_$nt.log; grep "d2prof" $O/d2prof_$nt.log | awk '!seen[$2 $3 $4]++' | grep -E " l0:| l1:| l7:"
      done
      cd $R
      for v in "MAM_FAST_CHUNKS=0" "MAM_FAST_CHUNKS=1"; do
        for cfg in c1 c2; do
          env $v timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pose --no-sin --no-overlap > $O/sw2_$cfg.json 2> $O/sw2_$cfg.err || { tail -5 $O/sw2_$cfg.err; exit 1; }
          python3 -c "
import json; d=json.loads(open('$O/sw2_$cfg.json').read().strip().splitlines()[-1])
print('$v $cfg', 'value %.0f' % d['value'], {k: round(v, 3) for k, v in d['stage_ms_per_step'].items() if k in ('fast', 'distribute', 'pyramid')}, d['roofline']['avg_launch_ms'])"
        done
      done ;;
    lone)
      cd /tmp && timeout -k 10 300 python3 $R/scripts/lba_bench.py --world --solves 10 > $O/lone_bench.json 2> $O/lone_bench.err || { tail -20 $O/lone_bench.err; exit 1; }
      head -c 600 $O/lone_bench.json; echo
      timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_lone -o run -- python3 $R/scripts/lba_bench.py --world --solves 6 > $O/prof_lone.log 2>&1 || { tail -20 $O/prof_lone.log; exit 1; }
      python3 $R/scripts/lone_trace.py $O/prof_lone/run_kernel_trace.csv --skip 2 | tee $O/lone_trace.txt | tail -30 ;;
    bench|bench2)
      cfg=c1; [ $part = bench2 ] && cfg=c2
      cd $R && timeout -k 10 600 python3 bench.py --config $cfg ${BENCH_ARGS:-} > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'parity_ok', d.get('parity_ok'))
print('latency', d.get('latency')); print('north_star', {k: v for k, v in (d.get('north_star') or {}).items() if k != 'note'})
print('stage', d.get('stage_ms_per_step')); print('overlap', d.get('overlap')); print('pose', (d.get('pose_optimization') or {}).get('ms_single_frame_launch'))" ;;
  esac
done
