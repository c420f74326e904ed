#!/bin/bash
# Run one gpurun command, waiting while the pool has no free box or slot (nothing ran, nothing charged: exit 3 or a
# "transient" status).  A command that ran (any other outcome) is never repeated.
#   scripts/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    echo "[wait] attempt $i: no box ($(grep -o 'retry in [0-9]*s' "$LOG" | head -1)); sleeping" >> "$LOG.wait"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
