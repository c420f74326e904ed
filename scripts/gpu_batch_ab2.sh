#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=batch2 REPS=2 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'b64:' 'b32: -- --batch-draws 32e6' 'b48: -- --batch-draws 48e6'
