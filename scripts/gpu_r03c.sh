#!/bin/bash
# rocprofv3 kernel stats of the WGS bench: phased-sync (sampling alone, then writers) and the default batch pipeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
T=${TAG:-r03c}
for v in phased-sync batch; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${T}_$v -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --pipeline $v > gpurun_out/prof_bench_${T}_$v.log 2>&1 || exit $?
  KS=$(find gpurun_out/prof/${T}_$v -name "*kernel_stats.csv" | head -1)
  cp "$KS" gpurun_out/${T}_${v}_kernel_stats.csv
  python3 scripts/kstats.py "$KS" 25 > gpurun_out/${T}_${v}_kstats.txt 2>&1
  KT=$(find gpurun_out/prof/${T}_$v -name '*kernel_trace.csv' | head -1)
  gzip -c "$KT" > gpurun_out/${T}_${v}_kernel_trace.csv.gz
  rm -rf gpurun_out/prof/${T}_$v
  echo "$v done"
done
