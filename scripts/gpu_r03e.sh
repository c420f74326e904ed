#!/bin/bash
# Corruption rows as the default (position-major row pass on the writer stream, seams stored by the seam pass):
# GPU suite + smoke on the defaults, the in-place pass (MH_CR_ROWS=0) under the corrupt tests, chr1-corrupt A/B,
# kernel stats, and a WGS check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03e}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
MH_CR_ROWS=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}_inplace.log 2>&1 || { tail -40 gpurun_out/pytest_${T}_inplace.log; exit 1; }
tail -2 gpurun_out/pytest_${T}_inplace.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${T}.log 2>&1 || { tail -20 gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
for p in 1 0 ov 1 0 ov; do
  case $p in 1) E="MH_CR_ROWS=1";; 0) E="MH_CR_ROWS=0";; ov) E="MH_CR_ROWS_OVERLAP=1";; esac
  env $E timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$p.json 2>gpurun_out/bench_${T}_$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$p.json')); print('chr1 corrupt $p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --workload chr1 --corrupt --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${T}_prof.json 2>gpurun_out/${T}_prof.err || exit $?
python3 - gpurun_out/prof_${T}/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:5]:
  print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wgs.json 2>gpurun_out/bench_${T}_wgs.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs.json')); print('wgs', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
