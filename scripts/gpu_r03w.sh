#!/bin/bash
# Two tiles per 512-thread writer workgroup (MH_EW_PAIR=1): GPU parity under the knob, then WGS and chr1-corrupt A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03w}
MH_EW_PAIR=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -3 gpurun_out/pytest_${T}.log
for p in 0 1 0 1; do
  MH_EW_PAIR=$p timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wgs$p.json 2>gpurun_out/bench_${T}_wgs$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs$p.json')); print('wgs pair=$p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), d['roofline']['frac'])"
done
for p in 0 1; do
  MH_EW_PAIR=$p timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_cr$p.json 2>gpurun_out/bench_${T}_cr$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_cr$p.json')); print('chr1 corrupt pair=$p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
