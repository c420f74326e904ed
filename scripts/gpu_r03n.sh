#!/bin/bash
# WGS default trace after the emission-set change; writer LDS A/B (staged seams vs 4 KB less LDS), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03n}
for rep in 1 2 3; do
  for d in 0 256; do
    MH_EW_DBG=$d timeout -k 10 300 python -u bench.py --workload chr1 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_chr1_d${d}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_chr1_d${d}_$rep.json')); print('chr1 d$d rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  done
done
for rep in 1 2; do
  for d in 0 256; do
    MH_EW_DBG=$d timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wgs_d${d}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_d${d}_$rep.json')); print('wgs d$d rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${T}wgs -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prof_bench_${T}wgs.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
KT=$(find gpurun_out/prof/${T}wgs -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/gaps_${T}wgs.txt 2>&1; head -50 gpurun_out/gaps_${T}wgs.txt
