#!/bin/bash
# Round 4: the writer without its reads-part formatting / without its qname heads (calibration builds, wrong bytes)
# against the product, on the WGS line: what the formatting costs per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/mitty_amd/_lib
TAG=r04p REPS=1 bash scripts/gpu_ab.sh 'base:' "nofmt:MH_LIB=$L/v_NOFMT/libmitty_hip.so" "nohead:MH_LIB=$L/v_NOHEAD/libmitty_hip.so" || exit $?
echo done
