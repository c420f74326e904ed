#!/bin/bash
# Round 4: the WGS line on torch's HIP runtime at N = 1 (as at N > 1) and with ramped first batches, against the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04u REPS=2 bash scripts/gpu_ab.sh 'base:' 'torchrt: -- --hip-runtime torch' 'ramp1: -- --batch-ramp 1' 'ramp2: -- --batch-ramp 2' || exit $?
echo done
