#!/bin/bash
# Development measurement of the WGS line: bench (prime pass, 8 steps after 4 warm-up), then its kernel statistics
# under rocprofv3 (3 steps).  Extra arguments go to both bench runs.   bash scripts/gpu_dev.sh TAG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/dev_$TAG
mkdir -p $O
timeout -k 10 420 python -u bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-e2e "$@" > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json "$TAG" || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-prime "$@" > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python3 scripts/bsum.py $O/bench_prof.json "$TAG prof" || true
python3 scripts/kstats.py $(ls $O/prof/*kernel_stats.csv | head -1) 4 22
echo done
