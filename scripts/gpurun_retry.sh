#!/bin/bash
# gpurun with retries while no box could be prepared (exit 3: nothing ran, nothing charged). Any other exit status
# (including a failure of the command itself) is returned at once. Usage: scripts/gpurun_retry.sh <log> <timeout> <cmd>
log=$1; to=$2; shift 2
for i in $(seq 1 ${GPURUN_ATTEMPTS:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  st=$?
  echo "exit $st (attempt $i)" >> "$log"
  [ $st -ne 3 ] && exit $st
  sleep 60
done
exit 3
