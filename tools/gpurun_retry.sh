#!/bin/bash
# Dev helper: run one gpurun call; if the pool reports a transient infrastructure failure (no box was
# acquired, nothing ran on a GPU), wait and submit the same call again, at most 6 times.  A call that
# ran and failed is never resubmitted.  Usage: tools/gpurun_retry.sh <timeout-s> '<command>' <logfile>
T=$1; CMD=$2; LOG=$3
for i in 1 2 3 4 5 6; do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then sleep 60; continue; fi
  exit $rc
done
exit 3
