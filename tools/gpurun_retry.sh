#!/bin/bash
# Re-submit a gpurun call while the pool has no free slot (status=transient / exit 3: nothing ran,
# nothing charged).  Any other outcome — success or failure of the command — ends the loop.
#   usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then sleep 90; continue; fi
  exit $rc
done
exit 3
