#!/bin/bash
# qname rows padded to an odd dword stride (LDS banks): parity + chr1/WGS A/B against the old multiple-of-16 stride.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03r}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "unit_vs_oracle or chr1_unit_fastq or emit_slices or async_emission or e2e or corrupt" > gpurun_out/pytest_${T}.log 2>&1
echo "pytest rc=$?"; tail -1 gpurun_out/pytest_${T}.log
for rep in 1 2 3; do
  for q in 0 4; do
    MH_EW_QPAD=$q timeout -k 10 300 python -u bench.py --workload chr1 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_chr1_q${q}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_chr1_q${q}_$rep.json')); print('chr1 qpad $q rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  done
done
for rep in 1 2; do
  for q in 0 4; do
    MH_EW_QPAD=$q timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wgs_q${q}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_q${q}_$rep.json')); print('wgs qpad $q rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  done
done
