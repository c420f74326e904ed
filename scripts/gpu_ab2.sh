#!/bin/bash
# same-box A/B of emit modes 0 and 2 on the WGS line (and configs[1] chr1 once each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
TAG=$T REPS=2 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'm0: -- --emit-mode 0' 'm2: -- --emit-mode 2' || exit $?
TAG=${T}c REPS=1 BENCH_ARGS="--steps 20 --warmup 10 --workload chr1" bash scripts/gpu_ab.sh 'm0: -- --emit-mode 0' 'm2: -- --emit-mode 2'
