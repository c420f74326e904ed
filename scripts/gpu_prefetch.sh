#!/bin/bash
# haplotype prefetch (threaded): issued before unit 0 / after unit 0 against none
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=prefetch3 REPS=4 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'pfm1: -- --prefetch --prefetch-after -1' 'nopf:' 'pf0: -- --prefetch --prefetch-after 0' || exit $?
