#!/bin/bash
# Same-box A/B of the c2 bench line at LBA batch splits 2 (default) and 4 (MAM_LBA_SPLIT).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
for sp in ${SPLITS:-2 4}; do
  MAM_LBA_SPLIT=$sp timeout -k 10 600 python3 bench.py --config c2 --no-cpu-baseline > $O/bench_c2_split$sp.json 2> $O/bench_c2_split$sp.err || { tail -5 $O/bench_c2_split$sp.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_c2_split$sp.json'))
print('split $sp', round(d['value']), round(d['ms_per_step'], 2), d.get('parity_ok'), 'LM alone', round(d['overlap']['local_mapping_only_ms_per_step'], 2), 'tracking alone', round(d['overlap']['tracking_only_ms_per_step'], 2))"
done
