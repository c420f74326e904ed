#!/bin/bash
# Pointer jumping on the permutation chains before the batch chase (MH_PERM_JUMP=R rounds): GPU suite under R = 3,
# then WGS A/B (R = 0, 2, 3) with the permutation stage's time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03j2}
MH_PERM_JUMP=3 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for r in 0 2 3 0 2 3; do
  MH_PERM_JUMP=$r timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$r.json 2>gpurun_out/bench_${T}_$r.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$r.json')); sm=d.get('stage_ms') or {}; print('wgs jump=$r', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), 'perm', sm.get('sample_permutation'))"
done
