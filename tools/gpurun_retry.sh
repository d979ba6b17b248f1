#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free box (exit 3: nothing ran,
# nothing charged) -- a call that ran is never repeated.  usage: tools/gpurun_retry.sh <log> <limit-s> <cmd>
LOG=$1; LIM=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $LIM -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient rc=None charged=0.0s" $LOG; then exit $rc; fi
  sleep 150
done
exit $rc
