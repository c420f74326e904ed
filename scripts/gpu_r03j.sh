#!/bin/bash
# 256-thread onesweep sort (MH_SORT_SMALL) parity + WGS/chr1 A/B; device BGZF kernel rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03j}
MH_SORT_SMALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "chr1_templates or batched_units or templates_vs_oracle or pipelined or bgzf or fifos_and_gz or unit_vs_oracle or chr1_unit_fastq or emit_slices or async_emission" > gpurun_out/pytest_${T}_ss.log 2>&1
echo "sort-small pytest rc=$?"; tail -1 gpurun_out/pytest_${T}_ss.log
for ss in 0 1; do
  MH_SORT_SMALL=$ss timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 > gpurun_out/bench_${T}_wgs_ss$ss.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_ss$ss.json')); print('wgs ss$ss', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
  MH_SORT_SMALL=$ss timeout -k 10 300 python -u bench.py --workload chr1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_chr1_ss$ss.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_chr1_ss$ss.json')); print('chr1 ss$ss', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${T}gz -o run -- python3 scripts/bgzf_rate.py --mb 1024 --reps 3 > gpurun_out/bgzf_rate_${T}.log 2>&1 || exit $?
grep '^{' gpurun_out/bgzf_rate_${T}.log
python3 scripts/kstats.py $(find gpurun_out/prof/${T}gz -name "*kernel_stats.csv" | head -1) 3 2>&1 | head -8
