#!/bin/bash
# gpurun with retries while the pool has no free slot / box (those attempts run nothing and charge nothing)
# usage: scripts/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  timeout $((TO + 1200)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  if grep -q "retry in\|no free box\|are busy\|status=transient" $LOG; then sleep 120; else break; fi
done
tail -40 $LOG
