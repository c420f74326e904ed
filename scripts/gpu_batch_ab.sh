#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=batch REPS=2 BENCH_ARGS="--steps 10 --warmup 10" bash scripts/gpu_ab.sh 'b64:' 'b96: -- --batch-draws 96e6' 'b128: -- --batch-draws 128e6'
