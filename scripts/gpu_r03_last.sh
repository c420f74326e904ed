#!/bin/bash
# Last check of the committed tree: GPU suite, smoke, and short WGS and corrupt bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_last.log 2>&1 || { tail -30 gpurun_out/pytest_last.log; exit 1; }
tail -1 gpurun_out/pytest_last.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_last.log 2>&1 || { tail -20 gpurun_out/smoke_last.log; exit 1; }
tail -1 gpurun_out/smoke_last.log
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_last_wgs.json 2>gpurun_out/bench_last_wgs.err || exit $?
timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_last_cr.json 2>gpurun_out/bench_last_cr.err || exit $?
for f in wgs cr; do python3 -c "import json; d=json.load(open('gpurun_out/bench_last_$f.json')); print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['roofline']['traffic_source'])"; done
