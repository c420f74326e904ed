#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=cr REPS=2 BENCH_ARGS="--steps 20 --warmup 10 --workload chr1 --corrupt" bash scripts/gpu_ab.sh 'new:' 'base:MH_LIB=mitty_amd/_lib/v_base/libmitty_hip.so'
bash scripts/gpu_iso.sh cr --workload chr1 --corrupt 2>&1 | grep -E "ms/step" | head -8
