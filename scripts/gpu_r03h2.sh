#!/bin/bash
# The corruption-rows knobs' parity: the record-major row pass (MH_CR_COLS=0) and the row pass on its own stream
# (MH_CR_ROWS_OVERLAP=1), each under the GPU corruption tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MH_CR_COLS=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_r03h2_rows.log 2>&1 || { tail -30 gpurun_out/pytest_r03h2_rows.log; exit 1; }
tail -1 gpurun_out/pytest_r03h2_rows.log
MH_CR_ROWS_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_r03h2_ov.log 2>&1 || { tail -30 gpurun_out/pytest_r03h2_ov.log; exit 1; }
tail -1 gpurun_out/pytest_r03h2_ov.log
