#!/bin/bash
# Round-6 GPU session parts (PARTS="probe3 probe4 dense tests"), each step under its own limit, stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/s6
mkdir -p $O
export TMPDIR=/tmp
cd $R
for part in ${PARTS:-probe3 probe4 dense tests}; do
  echo "=== $part"
  case $part in
    probe3)
      timeout -k 10 400 python3 -u scripts/ringmap_probe.py --config c3 --batch 2 --runs 40 --check > $O/probe_c3.log 2>&1 || { tail -5 $O/probe_c3.log; exit 1; }
      grep '"run": 3[5-9]' $O/probe_c3.log | cut -c1-330; grep same_control $O/probe_c3.log ;;
    probe4)
      timeout -k 10 400 python3 -u scripts/ringmap_probe.py --config c4 --batch 8 --runs 40 --check > $O/probe_c4.log 2>&1 || { tail -5 $O/probe_c4.log; exit 1; }
      grep '"run": 3[5-9]' $O/probe_c4.log | cut -c1-330; grep same_control $O/probe_c4.log ;;
    probe2)
      timeout -k 10 400 python3 -u scripts/ringmap_probe.py --config c2 --runs 10 --check > $O/probe_c2.log 2>&1 || { tail -5 $O/probe_c2.log; exit 1; }
      grep '"run": [6-9]' $O/probe_c2.log | cut -c1-330; grep same_control $O/probe_c2.log ;;
    dump)
      mkdir -p variants
      timeout -k 10 400 python3 -u scripts/ringmap_probe.py --config c2 --runs 8 --check --dump variants/ring_windows.npz > $O/probe_dump.log 2>&1 || { tail -5 $O/probe_dump.log; exit 1; }
      grep same_control $O/probe_dump.log | cut -c1-400; cp variants/ring_windows.npz $O/ ;;
    regab)
      for reg in 1 0; do
        echo "-- MAM_LBA_REG=$reg"
        MAM_LBA_REG=$reg timeout -k 10 180 python3 -u scripts/ring_window_replay.py variants/ring_windows.npz --mode batch --solves 6 > $O/regab_$reg.log 2>&1 || { tail -5 $O/regab_$reg.log; exit 1; }
        grep -v "^window" $O/regab_$reg.log
      done ;;
    dense)
      LV="${LV:-main t1024 b8}" SPLITS="${SPLITS:-1 2 4}" bash scripts/gpu_lba_dense.sh || exit 1 ;;
    tests)
      bash scripts/gpu_tests.sh || exit 1 ;;
    bench)
      timeout -k 10 800 python3 -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], d.get('parity_ok'), d.get('invalid'))
print('lba', {k: d['lba'].get(k) for k in ('points_per_window','opt_keyframes','edges_per_window','ms_per_step_span')})
print('overlap', d.get('overlap')); print('north_star', {k: d.get('north_star',{}).get(k) for k in ('ratio','lba_lone_window_ms_gpu','lba_window_ms_cpu')})" ;;
  esac
done
