set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for A in "--lanes 1 --batch 256" "--lanes 4 --batch 256 --no-graph" "--lanes 4 --batch 256"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/ptry_$i -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 $A > $O/ptry_$i.log 2>&1
  st=$?
  echo "$A -> $st"
  if [ $st -ne 0 ]; then grep -m3 -i "error" $O/ptry_$i.log; exit $st; fi
done
