#!/bin/bash
# Round 4: the qname digits two per step (FMT2 build): the GPU parity file on that build, then the A/B on the WGS line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y
mkdir -p $O
V=$GRAFT_REPO_ROOT/mitty_amd/_lib/v_FMT2/libmitty_hip.so
MH_LIB=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > $O/pytest_fmt2.log 2>&1 || { tail -30 $O/pytest_fmt2.log; exit 1; }
grep -E "passed|failed" $O/pytest_fmt2.log | tail -2
TAG=r04y REPS=3 bash scripts/gpu_ab.sh 'base:' "fmt2:MH_LIB=$V" || exit $?
echo done
