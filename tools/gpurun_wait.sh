#!/bin/bash
# Submit one gpurun call, resubmitting ONLY while the pool has no free box / slot (exit code 3 or a
# "transient" status: nothing ran, nothing was charged).  Any run that reached the box -- pass or
# fail -- ends the loop.  Usage: tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    sleep 90
    continue
  fi
  echo "gpurun rc=$rc" >> "$LOG"
  exit $rc
done
