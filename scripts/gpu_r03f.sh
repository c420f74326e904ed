#!/bin/bash
# After removing the writer's tile loop (VGPRs back to 59): chr1 and WGS benches, barrier A/B, phase costs, and the
# FETCH_SIZE calibration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03f}
run() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('$n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3), {k: d['stage_ms'][k] for k in list(d['stage_ms'])[:8]})"
}
C1="python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e"
run chr1 $C1 || exit $?
run chr1_sw MH_STAGE_WAIT=1 $C1 || exit $?
run chr1_sw_b64 MH_STAGE_WAIT=1 MH_EW_DBG=64 $C1 || exit $?
run chr1_sw_d1 MH_STAGE_WAIT=1 MH_EW_DBG=1 $C1 || exit $?
run wgs python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
run wgs_bd64 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 || exit $?
bash scripts/gpu_calib.sh || exit $?
