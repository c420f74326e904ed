#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
mkdir -p gpurun_out/$T
MH_MEASURE_LANE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "single_pass or batched_units_vs_oracle" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -2
TAG=$T REPS=3 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'main:' 'lane:MH_MEASURE_LANE=1'
