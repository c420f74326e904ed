#!/bin/bash
# BGZF stored-when-larger fix + GPU suite; chr1 end to end split (plain, gz on GPU, gz on host); WGS kernel trace and
# the writer-stream gaps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03h}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload chr1 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${T}_chr1.json 2> gpurun_out/bench_${T}_chr1.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_chr1.json')); print(json.dumps(d['end_to_end']))"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${T}wgs -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 > gpurun_out/prof_bench_${T}wgs.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
KT=$(find gpurun_out/prof/${T}wgs -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/gaps_${T}wgs.txt 2>&1; head -60 gpurun_out/gaps_${T}wgs.txt
