#!/bin/bash
# Round 3, first GPU pass: the GPU suite (incl. the WGS-plan parity test, FIFO and packing tests), then the default
# bench (30x WGS, N = 1), a gloo rehearsal of --gpus 2 on the one GPU, and the chr1 workload for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03a}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
echo bench-ok
MH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2_$T.json 2> gpurun_out/bench2_$T.err || exit $?
echo bench2-ok
timeout -k 10 200 python -u bench.py --workload chr1 --no-e2e --no-cpu-baseline > gpurun_out/bench_chr1_$T.json 2> gpurun_out/bench_chr1_$T.err || exit $?
echo done
