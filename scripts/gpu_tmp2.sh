set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_all.log 2>&1; st=$?; tail -5 $O/pt_all.log; [ $st -ne 0 ] && exit $st
timeout -k 10 400 python bench.py > $O/bench_c1.json 2>$O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
cat $O/bench_c1.json
