#!/bin/bash
# Round-3 record: full GPU suite; the default bench line (30x WGS, N = 1, CPU baselines, end to end); its rocprofv3
# kernel trace + stats and writer gaps; chr1, corrupt and tumor/normal lines; a 2-rank gloo rehearsal of --gpus 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
T=${TAG:-r03f}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/final/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_$T.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench_$T.json 2> gpurun_out/final/bench_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/final/bench_$T.json')); print('default', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
timeout -k 10 300 python -u bench.py --workload chr1 --no-cpu-baseline > gpurun_out/final/bench_chr1_$T.json 2>/dev/null || exit $?
timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --no-cpu-baseline --no-e2e > gpurun_out/final/bench_corrupt_$T.json 2>/dev/null || exit $?
timeout -k 10 400 python -u bench.py --tumor-normal --steps 3 --warmup 1 > gpurun_out/final/bench_tn_$T.json 2>/dev/null || exit $?
MH_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/bench2_$T.json 2> gpurun_out/final/bench2_$T.err || exit $?
for f in bench_chr1 bench_corrupt bench_tn bench2; do python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/final/${f}_$T.json') if l.startswith('{')][-1]; print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],2))"; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_$T -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/final/prof_bench_$T.log 2>&1 || exit $?
KT=$(find gpurun_out/final/prof_$T -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/final/gaps_$T.txt 2>&1
gzip -f "$KT"
echo done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_cr_$T -o run -- \
  python3 bench.py --workload chr1 --corrupt --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/final/prof_cr_bench_$T.log 2>&1 || exit $?
gzip -f gpurun_out/final/prof_cr_$T/run_kernel_trace.csv
echo done corrupt stats
