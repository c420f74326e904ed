#!/bin/bash
# Unaligned ds_read_b128 in the writer, device BGZF: GPU suite, chr1 + WGS benches (barrier A/B), gz end to end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "bgzf" > gpurun_out/pytest_${T}_bgzf.log 2>&1
echo "bgzf rc=$?"; grep -E "passed|failed" gpurun_out/pytest_${T}_bgzf.log | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log
[ $rc -le 1 ] || exit $rc
run() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('$n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3), {k: d['stage_ms'][k] for k in list(d['stage_ms'])[:6]}, d.get('end_to_end'))"
}
C1="python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline"
run chr1 $C1 || exit $?
run chr1_b64 MH_EW_DBG=64 $C1 --no-e2e || exit $?
run wgs python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 || exit $?
run chr1_d128 MH_EW_DBG=128 $C1 --no-e2e || exit $?
run chr1_d4 MH_EW_DBG=4 $C1 --no-e2e || exit $?
run chr1_d1 MH_EW_DBG=1 $C1 --no-e2e || exit $?
