#!/bin/bash
# Submit one gpurun command, resubmitting only while the pool has no free box (gpurun exit 3: nothing
# ran, nothing charged). Any other outcome (success, failure, refusal) ends the loop.
# usage: gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && grep -qv "no free box\|slot(s) on this pod are busy" "$LOG" && ! grep -q "status=transient" "$LOG" && exit $rc
  grep -q "status=transient" "$LOG" || exit $rc
  sleep 150
done
