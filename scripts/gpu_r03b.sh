#!/bin/bash
# WGS batch-size sweep (sampling batches vs writer overlap), the packing test, and the gloo --gpus 2 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "packing or fifo or gz" > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
for bd in 16e6 64e6 150e6 400e6; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws $bd > gpurun_out/bench_${T}_bd$bd.json 2> gpurun_out/bench_${T}_bd$bd.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${T}_bd$bd.json')); print('$bd', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['config']['batches_rank0'], d['stage_ms'].get('emit_write'), d['stage_ms'].get('sample'))"
done
MH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2_$T.json 2> gpurun_out/bench2_$T.err || exit $?
echo bench2-ok
