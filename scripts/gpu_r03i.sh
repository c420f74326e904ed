#!/bin/bash
# File-order bits written by the compaction store (no k_file_order launch): sampling/FASTQ parity, WGS bench A/B-free
# line (two repeats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03i}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wgs.py -m gpu -x -q --timeout 600 --timeout-method thread -k "templates or unit or e2e or wgs or batched or pipelined or lookahead or philox_sampling or chr1" > gpurun_out/pytest_${T}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log
[ $rc = 0 ] || { grep -E "Error|assert|Fail" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$rep.json 2>gpurun_out/bench_${T}_$rep.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$rep.json')); print('wgs rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
