#!/bin/bash
# Counters of k_pose_opt on the standalone c2 batch of 256 frames (scripts/pose_bench.py --no-single): kernel trace,
# then one rocprofv3 --pmc pass (VALU busy and the FP64 instruction mix), summarised by scripts/pmc_kernels.py.
# Usage: bash scripts/gpu_pose_pmc.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-posepmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="$R/scripts/pose_bench.py --config c2 --no-single --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${T}_trace -o run -- python3 $A > $O/${T}_trace.log 2>&1 || { tail -5 $O/${T}_trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/${T}_s -o run -- python3 $A > $O/${T}_s.log 2>&1 || { tail -5 $O/${T}_s.log; exit 1; }
python3 $R/scripts/pmc_kernels.py $O/${T}_trace $O/${T}_s --match pose --json $O/${T}.json
