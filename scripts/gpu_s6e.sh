#!/bin/bash
# The deferred-flag lookahead variant and the point-kernel occupancy variant on the ring batch (parity + time), then the
# profiles' pmc part.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
V="${V:-defer ps3 rdy rdydefer}" bash scripts/gpu_la2.sh || exit 1
timeout -k 10 120 python3 scripts/ring_window_replay.py variants/ring_windows.npz --mode batch --solves 8 > gpurun_out/main_b.log 2>&1 && echo "main: $(grep 'batch of' gpurun_out/main_b.log)"
bash scripts/gpu_profiles.sh r06 pmc
