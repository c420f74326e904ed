#!/bin/bash
# Corruption fast path (full 15-base blocks without per-base guards, v_bitop3 Philox) + lookahead pipeline: parity
# of both, then A/B lines (corrupt chr1 MH_CR_DBG=0/1; WGS batch/lookahead).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03t}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "corrupt or philox or lookahead or batched_units or pipelined or writer_gate" > gpurun_out/pytest_${T}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for d in 0 1; do
    MH_CR_DBG=$d timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_cr${d}_$rep.json 2>gpurun_out/bench_${T}_cr${d}_$rep.err || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/bench_${T}_cr${d}_$rep.json') if l.startswith('{')][-1]; print('corrupt dbg$d rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['stage_ms'].get('emit_corrupt'))"
  done
done
for pl in batch lookahead; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --pipeline $pl > gpurun_out/bench_${T}_${pl}.json 2>gpurun_out/bench_${T}_${pl}.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_${pl}.json')); print('wgs $pl', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}cr -o run -- \
  python3 bench.py --workload chr1 --corrupt --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_${T}cr.log 2>&1 || exit $?
find gpurun_out/prof_${T}cr -name '*kernel_stats.csv' -exec cp {} gpurun_out/${T}_cr_kernel_stats.csv \;
head -12 gpurun_out/${T}_cr_kernel_stats.csv | cut -c1-200
