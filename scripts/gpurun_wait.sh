#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free box / back-off (status=transient with
# nothing run and nothing charged).  A call that ran on a box (any exit status) is never re-submitted.
# usage: scripts/gpurun_wait.sh TIMEOUT 'command'
T=$1
shift
for i in $(seq 1 ${MAX_TRIES:-60}); do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient rc=None charged=0.0s\|status=transient rc=None charged=Nones"; then
    echo "[wait] attempt $i: no box ($(echo "$out" | grep -o 'no free box\|backing off\|stopped responding' | head -1)); sleeping" >&2
    sleep 90
    continue
  fi
  echo "$out" | grep -v "^\[gpurun\] every call"
  exit $rc
done
echo "[wait] gave up after ${MAX_TRIES:-60} attempts" >&2
exit 3
