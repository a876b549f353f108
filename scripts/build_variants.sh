#!/bin/bash
# Several libmam_gpu.so variants in parallel: bash scripts/build_variants.sh "name1:-DFLAG -DX=1" "name2:..." ...
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
pids=()
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}
  bash $R/scripts/build_variant.sh $n $f > /tmp/variant_$n.log 2>&1 &
  pids+=($!)
done
st=0
for p in "${pids[@]}"; do wait $p || st=1; done
exit $st
