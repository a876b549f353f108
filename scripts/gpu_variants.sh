#!/bin/bash
# Variant comparison: parity tests on the product library, then the c1 bench (stage times) for the product and
# each build/libmam_gpu_<V>.so in $VARIANTS; optional SQ counters (PMC="...") for the product.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
TESTS=${TESTS:-tests/test_orb_gpu.py tests/test_golden.py}
timeout -k 10 900 python -m pytest $TESTS -m gpu -q -x -p no:cacheprovider > $O/pytest_var.log 2>&1
st=$?
echo "pytest exit $st"; tail -5 $O/pytest_var.log
if [ $st -ne 0 ]; then exit $st; fi
for V in prod ${VARIANTS:-}; do
  if [ $V = prod ]; then LIBV=""; else LIBV=$R/build/libmam_gpu_$V.so; fi
  MAM3SLAM_GPU_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_var_$V.json 2> $O/bench_var_$V.err || exit $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']),{k:round(v,4) for k,v in d['stage_ms_per_step'].items()})" $O/bench_var_$V.json $V
done
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  for V in prod ${PMC_VARIANTS:-}; do
    if [ $V = prod ]; then LIBV=""; else LIBV=$R/build/libmam_gpu_$V.so; fi
    MAM3SLAM_GPU_LIB=$LIBV timeout -k 10 300 rocprofv3 --pmc $PMC -f csv -d $O/pmc_var_$V -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_var_$V.log 2>&1 || exit $?
    echo "== $V"; python3 $R/scripts/pmc_table.py $O/pmc_var_$V/run_counter_collection.csv | grep -E "${PMC_GREP:-k_}" | cut -c1-400
  done
fi
echo done
