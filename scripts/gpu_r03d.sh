#!/bin/bash
# Writer phase costs: the chr1 bench with writer phases skipped (MH_EW_DBG bits; timing only), writers mostly alone
# (MH_STAGE_WAIT=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03d}
for d in 0 1 2 8 16 9 25 0; do
  MH_STAGE_WAIT=1 MH_EW_DBG=$d timeout -k 10 200 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_d$d.json 2> gpurun_out/bench_${T}_d$d.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_d$d.json')); print('dbg $d', round(d['ms_per_step'],2), 'writer ms', round(d['roofline']['avg_launch_ms'],3), 'frac', round(d['roofline']['frac'],3))"
done
