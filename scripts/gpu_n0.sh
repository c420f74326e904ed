#!/bin/bash
# parity of the packed start nodes (measure pass), the measure pass alone, then A/B against the previous library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "single_pass or chr1_unit or batched_units or forced_fallbacks or e2e_single or unit_vs_oracle or distributed or emit_prepare or ranges" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -2
bash scripts/gpu_iso.sh $T 2>&1 | grep -E "emit_measure|emit_tiles|perm_chase|done" || exit 1
TAG=$T REPS=3 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'new:' 'base:MH_LIB=mitty_amd/_lib/v_base/libmitty_hip.so'
