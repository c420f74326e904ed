#!/bin/bash
# WGS with the asynchronous emission path (no host round trip per unit); its trace; chr1 end to end with the faster
# device deflate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03k}
for ae in "" "--async-emit"; do
  n=${ae:+ae}; n=${n:-sync}
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 $ae > gpurun_out/bench_${T}_wgs_$n.json 2>gpurun_out/bench_${T}_wgs_$n.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_$n.json')); print('wgs $n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${T}wgs -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 --async-emit > gpurun_out/prof_bench_${T}wgs.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
KT=$(find gpurun_out/prof/${T}wgs -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > gpurun_out/gaps_${T}wgs.txt 2>&1; head -24 gpurun_out/gaps_${T}wgs.txt
timeout -k 10 400 python -u bench.py --workload chr1 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${T}_chr1.json 2> gpurun_out/bench_${T}_chr1.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_${T}_chr1.json')); e=d['end_to_end']
print('chr1', round(d['value']/1e9,3), round(d['ms_per_step'],2))
for k in ('gz','gz_host'): print(k, round(e[k]['seconds'],3), e[k]['gz_bytes'], e[k]['split_s'])
print('plain', round(e['seconds'],3), e['split_s'])"
