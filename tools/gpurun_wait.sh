#!/bin/bash
# Run one gpurun call, re-submitting it only while the pool reports that no box was acquired
# (busy slots, a box that failed while being prepared, back-off): nothing ran and nothing was
# charged in those cases.  Any call that reached the box is never repeated.
#   usage: tools/gpurun_wait.sh LOGFILE TIMEOUT 'command'
LOG=$1
TO=$2
shift 2
for attempt in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "stopped responding while being prepared\|slot(s) on this pod are busy\|backing off\|no box\|no free box\|taken away by the GPU service" "$LOG" &&
     ! grep -q "status=ok" "$LOG"; then
    echo "attempt $attempt: no box ($(grep -o 'status=[a-z]*' "$LOG" | head -1)); waiting" >&2
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
