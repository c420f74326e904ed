#!/bin/bash
# Position-major corruption rows (k_cr_cols, MH_CR_ROWS=1): GPU parity under the knob, chr1-corrupt A/B against the
# in-place pass and the record-major row pass, then kernel stats of the rows mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03c}
MH_CR_ROWS=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -2 gpurun_out/pytest_${T}.log
for p in 0 c cs r 0 c cs; do
  case $p in 0) E="MH_CR_ROWS=0";; c) E="MH_CR_ROWS=1";; cs) E="MH_CR_ROWS=1 MH_CR_ROWS_SAME=1";; r) E="MH_CR_ROWS=1 MH_CR_COLS=0";; esac
  env $E timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$p.json 2>gpurun_out/bench_${T}_$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$p.json')); print('chr1 corrupt $p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
MH_CR_ROWS=1 MH_CR_ROWS_SAME=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --workload chr1 --corrupt --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${T}_prof.json 2>gpurun_out/${T}_prof.err || exit $?
python3 - gpurun_out/prof_${T}/run_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
  print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
