#!/bin/bash
# The single-pass writer against the two-pass path: each alone (every kernel serialised) and on the line (rocprofv3
# kernel statistics beside the sampling side).   bash scripts/gpu_fused_diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
bash scripts/gpu_iso.sh ${T}_fu || exit $?
bash scripts/gpu_iso.sh ${T}_tp --emit-mode 2 || exit $?
O=gpurun_out/line_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 0 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$m -o run -- \
    python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-e2e --emit-mode $m > $O/bench$m.json 2> $O/bench$m.err || exit $?
  python3 scripts/bsum.py $O/bench$m.json mode$m || true
  python3 scripts/kstats.py $(ls $O/prof$m/*kernel_stats.csv | head -1) 8 12
done
