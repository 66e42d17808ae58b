#!/bin/bash
# Run one GPU step with its own time limit; stop the whole call on a fault/timeout
# (exit codes other than 0 = pass and 1 = test failures).
# usage: scripts/gpu_step.sh NAME SECONDS cmd...
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc"
tail -n 25 "gpurun_out/$name.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[$name] fault/timeout (rc=$rc): stopping"
  exit 99
fi
exit 0
