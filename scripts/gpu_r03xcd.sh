#!/bin/bash
# Writer chunk stores XCD-aware tile order (MH_EW_DBG=1024) A/B on the WGS and chr1 benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03xcd}
for v in 0 1024 0 1024; do
  MH_EW_DBG=$v timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wgs$v.json 2>gpurun_out/bench_${T}_wgs$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs$v.json')); print('wgs dbg=$v', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3))"
done
for v in 0 1024 0 1024; do
  MH_EW_DBG=$v timeout -k 10 200 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_chr1$v.json 2>gpurun_out/bench_${T}_chr1$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_chr1$v.json')); print('chr1 dbg=$v', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3))"
done
