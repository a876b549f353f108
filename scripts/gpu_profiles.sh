#!/bin/bash
# Full measurement session (the files committed under profiles/): GPU parity tests, the c1 and c2 bench lines,
# kernel traces of standalone 64-frame launches (--lanes 1 --batch 64, as bench.py's serialised stage-timing pass
# measures them), FETCH_SIZE / WRITE_SIZE passes for roofline.traffic (they do not fit one PMC pass on gfx950), the
# B=1 timeline, the standalone LocalBundleAdjustment with its kernel trace and an FP64-MFMA counter pass, and the
# PoseOptimization, SearchInNeighbors (Fuse) and ComputeBoW benches with their kernel traces. Stops at the first step that fails, faults or times out.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for CFG in c1 c2; do
  timeout -k 10 600 python bench.py --config $CFG > $O/bench_$CFG.json 2> $O/bench_$CFG.err || { tail -5 $O/bench_$CFG.err; exit 1; }
  cat $O/bench_$CFG.json
done
timeout -k 10 300 python scripts/lba_bench.py --oracle > $O/lba_bench.json 2> $O/lba_bench.err || exit 1
cat $O/lba_bench.json
timeout -k 10 300 python scripts/pose_bench.py --config c1 --oracle > $O/pose_c1.json 2> $O/pose_c1.err || exit 1
timeout -k 10 300 python scripts/pose_bench.py --config c2 --oracle > $O/pose_c2.json 2> $O/pose_c2.err || exit 1
timeout -k 10 300 python scripts/fuse_bench.py --config c2 --oracle > $O/fuse_c2.json 2> $O/fuse_c2.err || exit 1
timeout -k 10 300 python scripts/bow_bench.py --config c2 --oracle > $O/bow_c2.json 2> $O/bow_c2.err || exit 1
cd /tmp && export TMPDIR=/tmp
for CFG in c1 c2; do
  A="--config $CFG --no-cpu-baseline --lanes 1 --batch 64 --no-latency --no-pose --no-sin"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$CFG -o run -- python3 $R/bench.py $A > $O/prof_$CFG.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$CFG -o run -- python3 $R/bench.py $A --steps 4 --warmup 1 > $O/pmc_fetch_$CFG.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$CFG -o run -- python3 $R/bench.py $A --steps 4 --warmup 1 > $O/pmc_write_$CFG.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_b1 -o run -- python3 $R/bench.py --batch 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-pose --no-sin > $O/prof_b1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_lba -o run -- python3 $R/scripts/lba_bench.py --solves 10 > $O/prof_lba.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_lba -o run -- python3 $R/scripts/lba_bench.py --solves 5 > $O/pmc_lba.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_pose -o run -- python3 $R/scripts/pose_bench.py --config c1 --reps 10 > $O/prof_pose.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_fuse -o run -- python3 $R/scripts/fuse_bench.py --config c2 --reps 10 > $O/prof_fuse.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_bow -o run -- python3 $R/scripts/bow_bench.py --config c2 --reps 10 > $O/prof_bow.log 2>&1 || exit 1
echo done
