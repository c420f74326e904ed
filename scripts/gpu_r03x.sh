#!/bin/bash
# Corruption rows before the writer (MH_CR_ROWS=1; the row pass on its own stream beside the previous writer, or
# MH_CR_ROWS_SAME=1 on the writer stream): GPU parity under the knob, then chr1-corrupt A/B and a WGS check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03x}
MH_CR_ROWS=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -3 gpurun_out/pytest_${T}.log
for p in 0 1 s 0 1 s; do
  if [ $p = s ]; then E="MH_CR_ROWS=1 MH_CR_ROWS_SAME=1"; else E="MH_CR_ROWS=$p"; fi
  env $E timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_cr$p.json 2>gpurun_out/bench_${T}_cr$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_cr$p.json')); print('chr1 corrupt rows=$p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
