#!/bin/bash
# FAST / blur / describe under rocprofv3: kernel trace, FETCH_SIZE and WRITE_SIZE passes, and an SQ + GRBM pass (VALU
# activity vs wave cycles) of standalone 64-frame c1 launches; one pass per counter group (gfx950 slot limits).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${1:-fast}
CFG=${2:-c1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16   # what bench.py sets for itself; under rocprofv3 the profiler initialises HIP first
A="--config $CFG --no-cpu-baseline --lanes 1 --batch 64 --no-latency --no-pose --no-sin --steps 4 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$T -o run -- python3 $R/bench.py $A > $O/prof_$T.log 2>&1 || { tail -5 $O/prof_$T.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmcf_$T -o run -- python3 $R/bench.py $A > $O/pmcf_$T.log 2>&1 || { tail -5 $O/pmcf_$T.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmcw_$T -o run -- python3 $R/bench.py $A > $O/pmcw_$T.log 2>&1 || { tail -5 $O/pmcw_$T.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/pmcs_$T -o run -- python3 $R/bench.py $A > $O/pmcs_$T.log 2>&1 || { tail -5 $O/pmcs_$T.log; exit 1; }
python3 $R/scripts/pmc_summary.py $O/prof_$T $O/pmcf_$T $O/pmcw_$T $O/pmcs_$T --traffic $O/traffic_$CFG.json > $O/pmc_$T.json && cat $O/pmc_$T.json
