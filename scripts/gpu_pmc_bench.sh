#!/bin/bash
# SQ counter pass over the c1 bench (kernel-level instruction mix / stall picture)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT} -f csv -d $O/pmc_sq -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS:-} > $O/pmc_sq.log 2>&1 || exit $?
echo done
