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
MH_EW_DBG=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "unit_vs_oracle_2mbp or chr1_unit_fastq or emit_slices or async_emission" > gpurun_out/pytest_${T}_d256.log 2>&1
echo "d256 pytest rc=$?"; tail -1 gpurun_out/pytest_${T}_d256.log
for d in 0 256; do
  MH_EW_DBG=$d timeout -k 10 300 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_d$d.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_d$d.json')); print('d$d', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
for cfg in "32e6 0" "64e6 0" "64e6 2" "64e6 3" "128e6 3"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws $1 --batch-ramp $2 > gpurun_out/bench_${T}_wgs_$1_$2.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_$1_$2.json')); print('wgs bd $1 ramp $2', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), d['config']['batches_rank0'])"
done
