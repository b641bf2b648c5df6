#!/bin/bash
# gpurun with retries ONLY while no box / slot is free (exit 3: nothing ran, nothing charged).
# Any other exit (success, a failing command, a refusal) ends it. Usage: gpu_retry.sh LOG TIMEOUT 'CMD'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  echo "exit $rc (attempt $i)" >> "$LOG"
  [ $rc -ne 3 ] && exit $rc
  sleep 75
done
exit 3
