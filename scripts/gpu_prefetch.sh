#!/bin/bash
# word-stream prefetch: the step's last batch prefetching before its first unit vs after it, against none
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=prefetch5 REPS=4 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'pfw:' 'pfwl: -- --prefetch-last-after -1' 'nopf: -- --no-prefetch' || exit $?
