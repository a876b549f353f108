#!/bin/bash
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o $R/variants/libfetch_probe.so $R/scripts/fetch_probe.hip
