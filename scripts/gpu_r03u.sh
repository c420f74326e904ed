#!/bin/bash
# Corruption pass A/B: phased full-block path on 512-thread workgroups (default) vs 1024 threads vs the guarded path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03u}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "corrupt or philox" > gpurun_out/pytest_${T}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in "512 0" "1024 0" "512 1"; do
    set -- $v
    MH_CR_THR=$1 MH_CR_DBG=$2 timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$1_$2_$rep.json 2>gpurun_out/bench_${T}_$1_$2_$rep.err || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/bench_${T}_$1_$2_$rep.json') if l.startswith('{')][-1]; print('corrupt thr$1 dbg$2 rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['stage_ms'].get('emit_corrupt'))"
  done
done
