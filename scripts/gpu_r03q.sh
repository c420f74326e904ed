#!/bin/bash
# Permutation sort with 9/10/11 key bits per onesweep pass: parity + WGS A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03q}
for b in 9 10 11; do
  MH_SORT_BITS=$b timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chr1_templates or batched_units or templates_vs_oracle" > gpurun_out/pytest_${T}_b$b.log 2>&1
  echo "bits $b pytest rc=$?"; tail -1 gpurun_out/pytest_${T}_b$b.log
done
for rep in 1 2; do
  for b in 0 9 10 11; do
    MH_SORT_BITS=$b timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_b${b}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_b${b}_$rep.json')); print('wgs bits $b rep $rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), {k: d['stage_ms'][k] for k in ('sample_permutation','emit_write') if k in d['stage_ms']})"
  done
done
