#!/bin/bash
# One row set on the writer stream (the default) and two with the overlapped row stream: GPU corruption tests for
# both, and a corrupt bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_r03k2.log 2>&1 || { tail -30 gpurun_out/pytest_r03k2.log; exit 1; }
tail -1 gpurun_out/pytest_r03k2.log
MH_CR_ROWS_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_r03k2_ov.log 2>&1 || { tail -30 gpurun_out/pytest_r03k2_ov.log; exit 1; }
tail -1 gpurun_out/pytest_r03k2_ov.log
timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_r03k2.json 2>gpurun_out/bench_r03k2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03k2.json')); print('cr', round(d['value']/1e9,3), round(d['ms_per_step'],2))"
