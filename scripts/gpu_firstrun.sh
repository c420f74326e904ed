#!/bin/bash
# The first bench process on a fresh box runs slow (1.38 vs 1.6 G/s in three calls); is a longer warm-up inside the
# process enough?  First run: --warmup 40; then the default warm-up twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/firstrun
mkdir -p $O
i=0
for w in 40 2 2; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 8 --warmup $w --no-cpu-baseline --no-e2e > $O/run$i.json 2> $O/run$i.err || exit $?
  python3 scripts/bsum.py $O/run$i.json "run$i warmup=$w" || true
done
echo done
