#!/bin/bash
# WGS pipeline sweep (sampling batches vs writer overlap; phased sampling), the packing / FIFO tests, and the gloo
# --gpus 2 rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "packing or fifo or gz" > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('$n', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['config']['batches_rank0'], round(d['roofline']['frac'],3), d['stage_ms'].get('emit_write'), d['stage_ms'].get('sample'))"
}
run bd32 || exit $?
run bd128 --batch-draws 128e6 || exit $?
run ph --pipeline phased || exit $?
run phs --pipeline phased-sync || exit $?
run phs64 --pipeline phased-sync --batch-draws 64e6 || exit $?
MH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2_$T.json 2> gpurun_out/bench2_$T.err || exit $?
echo bench2-ok
