#!/bin/bash
# One bench line (the metric, CPU baseline legs, end to end) and a short rocprofv3 kernel-statistics run of the same
# workload: bash scripts/gpu_bench_base.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-base}
mkdir -p $O
timeout -k 10 480 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 scripts/bsum.py $O/bench.json || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python3 scripts/bsum.py $O/bench_prof.json prof || true
