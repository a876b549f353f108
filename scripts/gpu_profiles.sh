#!/bin/bash
# The measurement session behind profiles/<round>/ (copied there by `python scripts/collect_profiles.py <round>`), in
# three parts that each fit one gpurun call:
#   lba    LocalBundleAdjustment: standalone bench (lone window + batches of 1 / 32, oracle-timed), kernel trace of the
#          batch of 32, its FP64-MFMA counter pass (-> lba_mfma_f64.json, read by bench.py's roofline_lba) and the
#          FETCH / WRITE / L2-hit / SQ passes (scripts/gpu_lba_pmc.sh)
#   bench  the c1 / c2 / c3 / c4 bench lines (default flags, CPU baseline on), the c2 line with the world windows, the
#          standalone PoseOptimization, SearchInNeighbors, ComputeBoW and batched SearchForTriangulation benches and the
#          PoseOptimization counters (scripts/gpu_pose_pmc.sh)
#   pmc    per config c1 / c2: kernel trace of standalone 64-frame launches with FETCH_SIZE, WRITE_SIZE and SQ/GRBM
#          passes (scripts/gpu_fast_pmc.sh -> traffic_cN.json, read by bench.py's roofline), and the default c2 bench
#          command under a kernel trace (its stage-pass launches vs the line's roofline: roofline_check.py)
# Usage: bash scripts/gpu_profiles.sh <round> <part>. Stops at the first step that fails, faults or times out.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
RND=${1:?round}
PART=${2:?part}
mkdir -p $O
cd $R
# (the box default GPU_MAX_HW_QUEUES, as the driver runs bench.py)
case $PART in
lba)
  timeout -k 10 300 python scripts/lba_bench.py --world --batch 32 --oracle > $O/lba_bench.json 2> $O/lba_bench.err || { tail -5 $O/lba_bench.err; exit 1; }
  cat $O/lba_bench.json
  bash scripts/gpu_lba_pmc.sh ${RND}lba || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/pmc_${RND}lba -o run -- python3 $R/scripts/lba_bench.py --world --batch 32 --solves 3 > $O/pmc_${RND}lba.log 2>&1 || { tail -5 $O/pmc_${RND}lba.log; exit 1; }
  # the timed leg's windows: the 32 windows of one c2 LocalMapping run on the device map (scripts/ringmap_probe.py
  # --dump, a GPU run; dumped first when absent; variants/ is git-ignored) through scripts/ring_window_replay.py under a
  # kernel trace and the FP64-MFMA pass bench.py's roofline_lba reads
  NPZ=$R/variants/ring_windows.npz
  [ -f $NPZ ] || { mkdir -p $R/variants; timeout -k 10 300 python3 $R/scripts/ringmap_probe.py --runs 8 --dump $NPZ > $O/ring_dump.log 2>&1; } || { tail -5 $O/ring_dump.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${RND}lba_ring -o run -- python3 $R/scripts/ring_window_replay.py $NPZ --mode batch --solves 6 > $O/${RND}lba_ring.log 2>&1 || { tail -5 $O/${RND}lba_ring.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/pmc_${RND}lba_ring -o run -- python3 $R/scripts/ring_window_replay.py $NPZ --mode batch --solves 3 > $O/pmc_${RND}lba_ring.log 2>&1 || { tail -5 $O/pmc_${RND}lba_ring.log; exit 1; }
  ;;
bench)
  for CFG in c1 c2 c3 c4; do
    timeout -k 10 600 python bench.py --config $CFG > $O/bench_$CFG.json 2> $O/bench_$CFG.err || { tail -5 $O/bench_$CFG.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$CFG.json')); print('$CFG', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d.get('parity_ok'))"
  done
  ;;
bench2)
  # the world-window leg beside the headline (--lm-windows world: the synthetic map's 50-KF windows)
  timeout -k 10 600 python bench.py --config c2 --lm-windows world > $O/bench_c2_world.json 2> $O/bench_c2_world.err || { tail -5 $O/bench_c2_world.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c2_world.json')); print('c2 world', d['value'], d['ms_per_step'], d.get('parity_ok'))"
  timeout -k 10 300 python scripts/tri_bench.py > $O/tri_bench.json 2> $O/tri_bench.err || exit 1
  timeout -k 10 300 python scripts/pose_bench.py --config c2 --oracle > $O/pose_c2.json 2> $O/pose_c2.err || exit 1
  timeout -k 10 300 python scripts/fuse_bench.py --config c2 --oracle > $O/fuse_c2.json 2> $O/fuse_c2.err || exit 1
  timeout -k 10 300 python scripts/bow_bench.py --config c2 --oracle > $O/bow_c2.json 2> $O/bow_c2.err || exit 1
  bash scripts/gpu_pose_pmc.sh ${RND}pose || exit 1
  ;;
pmc)
  bash scripts/gpu_fast_pmc.sh ${RND}c1 c1 > $O/pmc_${RND}c1.out || exit 1
  bash scripts/gpu_fast_pmc.sh ${RND}c2 c2 > $O/pmc_${RND}c2.out || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_${RND}default_c2 -o run -- python3 $R/bench.py --config c2 > $O/bench_traced_c2.json 2> $O/prof_${RND}default_c2.log || { tail -5 $O/prof_${RND}default_c2.log; exit 1; }
  python3 $R/scripts/roofline_check.py $O/prof_${RND}default_c2/run_kernel_trace.csv $O/bench_traced_c2.json > $O/roofline_check_c2.json || exit 1
  cat $O/roofline_check_c2.json
  ;;
*)
  echo "part: lba | bench | bench2 | pmc"; exit 2 ;;
esac
echo done
