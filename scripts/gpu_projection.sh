#!/bin/bash
# The N-GPU projection: rank 0's share of the N-rank LPT plan timed alone on this GPU (--plan-share 0/N), N = 2, 4, 8,
# beside the N = 1 line.  A projection, not a scaling measurement (the driver's 8-GPU run is that).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/projection
mkdir -p $O
for n in 1 2 4 8; do
  if [ $n -eq 1 ]; then extra=""; else extra="--plan-share 0/$n"; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e $extra > $O/n$n.json 2> $O/n$n.err || exit $?
  python3 scripts/bsum.py $O/n$n.json n$n || true
done
echo done
