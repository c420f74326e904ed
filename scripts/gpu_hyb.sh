#!/bin/bash
# parity of the chained and single-pass emission paths, then a same-box A/B of the emit modes on the WGS line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "single_pass or chr1_unit_fastq or batched_units_vs_oracle" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -2
TAG=$T REPS=2 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'm0: -- --emit-mode 0' 'm2: -- --emit-mode 2' 'm3: -- --emit-mode 3'
