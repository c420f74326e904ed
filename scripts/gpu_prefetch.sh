#!/bin/bash
# prefetch placement: after unit 0 (default; the step's last batch before unit 0) vs before unit 0 in every batch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=prefetch7 REPS=4 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'def:' 'm1all: -- --prefetch-after -1' 'a1: -- --prefetch-after 1' || exit $?
