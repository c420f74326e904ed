#!/bin/bash
# A/B of this tree against another tree of the repository checked out under the root (an earlier round's worktree),
# alternating REPS times after one throwaway run (the box's first process runs slow: DESIGN.md "the first process").
#   REPS=2 bash scripts/gpu_ab_trees.sh TAG DIR [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; D=$2; shift 2
REPS=${REPS:-2}
O=$GRAFT_REPO_ROOT/gpurun_out/abt_$TAG
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-prime --no-cpu-baseline --no-e2e "$@" > $O/throwaway.json 2>&1 || exit $?
for rep in $(seq 1 $REPS); do
  for t in here other; do
    if [ $t = here ]; then cd "$GRAFT_REPO_ROOT"; else cd "$GRAFT_REPO_ROOT/$D"; fi
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-prime --no-cpu-baseline --no-e2e "$@" > $O/${t}_$rep.json 2> $O/${t}_$rep.err || exit $?
    cd "$GRAFT_REPO_ROOT"
    python3 scripts/bsum.py $O/${t}_$rep.json "$t $rep" || true
  done
done
echo done
