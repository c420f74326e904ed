#!/bin/bash
# 16 emission buffer sets (the host no longer waits for a batch's writers): GPU suite, WGS sync/async A/B, a
# kernel + HIP API trace of the WGS step (host waits lined up with the writer gaps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log
[ $rc -le 1 ] || exit $rc
for ae in "" "--async-emit"; do
  n=${ae:+ae}; n=${n:-sync}
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 $ae > gpurun_out/bench_${T}_wgs_$n.json 2>gpurun_out/bench_${T}_wgs_$n.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_$n.json')); print('wgs $n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
timeout -k 10 400 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${T}_chr1.json 2>gpurun_out/bench_${T}_chr1.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_${T}_chr1.json')); e=d['end_to_end']
print('chr1', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))
for k in ('gz','gz_host'): print(k, round(e[k]['seconds'],3), e[k]['gz_bytes'], e[k]['split_s'])
print('plain', round(e['seconds'],3), e['split_s'])"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/prof/${T}wgs -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 > gpurun_out/prof_bench_${T}wgs.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
KT=$(find gpurun_out/prof/${T}wgs -name '*kernel_trace.csv' | head -1)
HT=$(find gpurun_out/prof/${T}wgs -name '*hip_api_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/gaps_${T}wgs.txt 2>&1; head -30 gpurun_out/gaps_${T}wgs.txt
python3 scripts/host_waits.py "$HT" "$KT" 0.5 > gpurun_out/hostwaits_${T}wgs.txt 2>&1; head -60 gpurun_out/hostwaits_${T}wgs.txt
gzip -f "$HT"
