#!/bin/bash
# gpu_iso.sh for another tree of this repository checked out under the repo root (e.g. a git worktree of an earlier
# round), so two builds' isolated kernel times come from one box:   bash scripts/gpu_iso_tree.sh DIR TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=$1; TAG=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/iso_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/$D"
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-prime "$@" > $O/bench.json 2> $O/bench.err || exit $?
python3 "$GRAFT_REPO_ROOT/scripts/kstats.py" $(ls $O/prof/*kernel_stats.csv | head -1) 3 16
echo done
