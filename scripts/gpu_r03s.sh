#!/bin/bash
# Lookahead pipeline (next batch's sort queued before this batch's writers, writers gated on it): parity, WGS A/B,
# trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03s}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lookahead or batched_units or pipelined or writer_gate" > gpurun_out/pytest_${T}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log
[ $rc -le 1 ] || exit $rc
[ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/pytest_${T}.log | head; exit 1; }
for rep in 1 2; do
  for pl in batch lookahead; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --pipeline $pl > gpurun_out/bench_${T}_${pl}_$rep.json 2>gpurun_out/bench_${T}_${pl}_$rep.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_${pl}_$rep.json')); print('wgs $pl rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/${T}la -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-e2e --pipeline lookahead > gpurun_out/prof_bench_${T}la.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
KT=$(find gpurun_out/prof/${T}la -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/gaps_${T}la.txt 2>&1; head -45 gpurun_out/gaps_${T}la.txt
