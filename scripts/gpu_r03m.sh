#!/bin/bash
# Chunked device-BGZF D2H (mh_output_bgzf_range): GPU suite, chr1 end to end (plain / gz on GPU / gz on host), WGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${T}_chr1.json 2>gpurun_out/bench_${T}_chr1.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_${T}_chr1.json')); e=d['end_to_end']
print('chr1', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))
for k in ('gz','gz_host'): print(k, round(e[k]['seconds'],3), e[k]['gz_bytes'], e[k]['split_s'])
print('plain', round(e['seconds'],3), e['split_s'])"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 > gpurun_out/bench_${T}_wgs.json 2>gpurun_out/bench_${T}_wgs.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs.json')); print('wgs', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
MH_WRITER_GATE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batched_units or pipelined or writer_gate or chr1_templates" > gpurun_out/pytest_${T}_gate.log 2>&1
echo "gate pytest rc=$?"; tail -1 gpurun_out/pytest_${T}_gate.log
for cfg in "0 -1" "0 3" "0 5" "1 -1"; do
  set -- $cfg
  n=bd$1_g$2
  bd=64e6; [ "$1" = 1 ] && bd=32e6
  if [ "$2" = "-1" ]; then G=""; else G="MH_WRITER_GATE=$2"; fi
  timeout -k 10 300 env $G python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --batch-draws $bd > gpurun_out/bench_${T}_$n.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('wgs $n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
