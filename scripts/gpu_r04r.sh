#!/bin/bash
# Round 4: what the writer's formatting costs — the nodes' loads (NOFMT2: loaded, nothing formatted) against the
# formatting (NOFMT: neither) — calibration builds, wrong bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/mitty_amd/_lib
TAG=r04r REPS=2 bash scripts/gpu_ab.sh 'base:' "nofmt2:MH_LIB=$L/v_NOFMT2/libmitty_hip.so" "nofmt:MH_LIB=$L/v_NOFMT/libmitty_hip.so" || exit $?
echo done
