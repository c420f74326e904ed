#!/bin/bash
# Epoch look-back scans + batch-wide permutation: the GPU suite, then the WGS bench (batch / phased-sync), the chr1
# bench, and the writer's launch-only floor (MH_EW_DBG=32).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$T.log
[ $rc -eq 0 ] || exit $rc
run() {   # name, env..., bench args after --
  local n=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('$n', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3), {k: d['stage_ms'][k] for k in list(d['stage_ms'])[:8]})"
}
run wgs python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
run wgs_phs python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --pipeline phased-sync || exit $?
run chr1 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
run chr1_unitperm MH_PERM_UNIT=1 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
run d32 MH_STAGE_WAIT=1 MH_EW_DBG=32 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
for k in 4 6 8; do
  run p$k MH_STAGE_WAIT=1 MH_EW_PERSIST=$k python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
done
run p0 MH_STAGE_WAIT=1 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
run b64 MH_STAGE_WAIT=1 MH_EW_DBG=64 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
