#!/bin/bash
# Full measurement session (round 2; the files committed under profiles/r02/ come from it, copied by
# scripts/collect_profiles.py): the GPU parity suite; the c1 / c2 / c3 bench lines (default flags, CPU baseline on);
# standalone LocalBundleAdjustment (oracle-timed), PoseOptimization, SearchInNeighbors, ComputeBoW and batched
# SearchForTriangulation benches; per config c1 / c2 a kernel trace of standalone 64-frame launches (the launch shape
# bench.py's stage pass times) with FETCH_SIZE, WRITE_SIZE and SQ/GRBM passes (scripts/gpu_fast_pmc.sh ->
# traffic_cN.json); a kernel trace of the default c2 bench (tracking and LocalMapping concurrently); the LBA kernel
# trace and its FP64-MFMA counter pass. Stops at the first step that fails, faults or times out.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for CFG in c1 c2 c3; do
  timeout -k 10 600 python bench.py --config $CFG > $O/bench_$CFG.json 2> $O/bench_$CFG.err || { tail -5 $O/bench_$CFG.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$CFG.json')); print('$CFG', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 python scripts/lba_bench.py --world --batch 32 --oracle > $O/lba_bench.json 2> $O/lba_bench.err || exit 1
timeout -k 10 300 python scripts/tri_bench.py > $O/tri_bench.json 2> $O/tri_bench.err || exit 1
timeout -k 10 300 python scripts/pose_bench.py --config c2 --oracle > $O/pose_c2.json 2> $O/pose_c2.err || exit 1
timeout -k 10 300 python scripts/fuse_bench.py --config c2 --oracle > $O/fuse_c2.json 2> $O/fuse_c2.err || exit 1
timeout -k 10 300 python scripts/bow_bench.py --config c2 --oracle > $O/bow_c2.json 2> $O/bow_c2.err || exit 1
bash scripts/gpu_fast_pmc.sh r02c1 c1 > $O/pmc_r02c1.out || exit 1
bash scripts/gpu_fast_pmc.sh r02c2 c2 > $O/pmc_r02c2.out || exit 1
bash scripts/gpu_c2_trace.sh r02c2load > $O/prof_r02c2load.out || exit 1
cd /tmp && export TMPDIR=/tmp
for CFG in c1 c2; do   # the default bench command under a kernel trace: its stage-pass launches vs bench.py's roofline
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_r02default_$CFG -o run -- python3 $R/bench.py --config $CFG > $O/bench_traced_$CFG.json 2> $O/prof_r02default_$CFG.log || { tail -5 $O/prof_r02default_$CFG.log; exit 1; }
  python3 $R/scripts/roofline_check.py $O/prof_r02default_$CFG/run_kernel_trace.csv $O/bench_traced_$CFG.json > $O/roofline_check_$CFG.json || exit 1
  cat $O/roofline_check_$CFG.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_r02lba -o run -- python3 $R/scripts/lba_bench.py --world --batch 32 --solves 4 > $O/prof_r02lba.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/pmc_r02lba -o run -- python3 $R/scripts/lba_bench.py --world --batch 32 --solves 3 > $O/pmc_r02lba.log 2>&1 || exit 1
echo done
