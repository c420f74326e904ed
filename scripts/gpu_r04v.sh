#!/bin/bash
# Round 4: the half-size first batch (--batch-ramp 1) against the default, three alternations; and on torch's runtime.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04v REPS=3 bash scripts/gpu_ab.sh 'base:' 'ramp1: -- --batch-ramp 1' 'ramp1t: -- --batch-ramp 1 --hip-runtime torch' || exit $?
echo done
