#!/bin/bash
# Corruption rows on their own stream: the row pass's grid (MH_CR_ROWS_GRID workgroups of 512 threads) A/B on the
# chr1 corrupt bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03z}
for g in 512 256 128 384 256 512; do
  MH_CR_ROWS=1 MH_CR_ROWS_GRID=$g timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_g$g.json 2>gpurun_out/bench_${T}_g$g.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_g$g.json')); print('chr1 corrupt rows grid=$g', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
