#!/bin/bash
# WGS writer gate at 0/1/2 (the next batch's sort runs alone before a batch's writers); corruption passes beside the
# writers (MH_CR_OVERLAP): parity + configs[2] bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03o}
MH_CR_OVERLAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "corrupt or philox or async_emission or emit_slices" > gpurun_out/pytest_${T}_cro.log 2>&1
echo "cr-overlap pytest rc=$?"; tail -1 gpurun_out/pytest_${T}_cro.log
for g in -1 0 1 2; do
  if [ "$g" = "-1" ]; then G=""; else G="MH_WRITER_GATE=$g"; fi
  timeout -k 10 300 env $G python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_g$g.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_g$g.json')); print('wgs gate $g', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
for cro in 0 1; do
  for pc in 0; do
    MH_CR_OVERLAP=$cro timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_cr$cro.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_cr$cro.json')); print('corrupt overlap $cro', round(d['value']/1e9,3), round(d['ms_per_step'],2), {k: d['stage_ms'][k] for k in list(d['stage_ms'])[:5]})"
  done
done
MH_CR_OVERLAP=1 MH_CR_PER_CU=2 timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_cr1pc2.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_cr1pc2.json')); print('corrupt overlap 1 per_cu 2', round(d['value']/1e9,3), round(d['ms_per_step'],2))"
