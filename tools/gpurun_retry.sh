#!/bin/bash
# gpurun with a wait-and-retry while no GPU box is free (gpurun exit 3, or an infrastructure
# event that took the box before the command ran: nothing ran, nothing charged).  A command that
# ran -- whatever its exit status -- is never started again.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; tmo=$2; shift 2
for try in $(seq 1 ${GPURUN_TRIES:-30}); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "[retry] no box (try $try, rc=$rc); waiting" >> "$log.retries"
    sleep ${GPURUN_WAIT:-240}
    continue
  fi
  exit $rc
done
exit 3
