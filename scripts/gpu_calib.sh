#!/bin/bash
# FETCH_SIZE calibration (scripts/calib_fetch.hip): timings, then one FETCH_SIZE pass and one WRITE_SIZE-free pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/calib_fetch > gpurun_out/calib_times.json || exit $?
cat gpurun_out/calib_times.json
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_pmc -o run -- ./scripts/calib_fetch > gpurun_out/calib_pmc.log 2>&1 || exit $?
find gpurun_out/calib_pmc -name '*counter_collection.csv' -exec cp {} gpurun_out/calib_fetch_counters.csv \;
echo calib-ok
