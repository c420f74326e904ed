#!/bin/bash
# Kernel times of the corruption rows mode (MH_CR_ROWS=1) on the chr1 corrupt bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
MH_CR_ROWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03y -o run -- python3 bench.py --workload chr1 --corrupt --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r03y.json 2>gpurun_out/r03y.err || exit $?
f=$(find gpurun_out/prof_r03y -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
  print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), round(float(r['TotalDurationNs'])/1e6,1))
PY
