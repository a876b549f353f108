#!/bin/bash
# Counters of the LBA kernels on the standalone batch of 32 world windows: kernel trace, then one rocprofv3 --pmc pass
# per counter group (FETCH_SIZE; WRITE_SIZE; TCC hit/miss; SQ + GRBM), summarised by scripts/pmc_kernels.py.
# Usage: bash scripts/gpu_lba_pmc.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-lbapmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
A="$R/scripts/lba_bench.py --world --batch 32 --solves 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${T}_trace -o run -- python3 $A > $O/${T}_trace.log 2>&1 || { tail -5 $O/${T}_trace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/${T}_f -o run -- python3 $A > $O/${T}_f.log 2>&1 || { tail -5 $O/${T}_f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/${T}_w -o run -- python3 $A > $O/${T}_w.log 2>&1 || { tail -5 $O/${T}_w.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d $O/${T}_h -o run -- python3 $A > $O/${T}_h.log 2>&1 || { tail -5 $O/${T}_h.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/${T}_s -o run -- python3 $A > $O/${T}_s.log 2>&1 || { tail -5 $O/${T}_s.log; exit 1; }
python3 $R/scripts/pmc_kernels.py $O/${T}_trace $O/${T}_f $O/${T}_w $O/${T}_h $O/${T}_s --match lba --json $O/${T}.json
