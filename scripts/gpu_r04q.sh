#!/bin/bash
# Round 4: the writer with its seam chunks computed in the chunk sweep (no seam pass staging, no second barrier):
# the GPU parity file on that build, then the A/B on the WGS line and on configs[2].
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q
mkdir -p $O
V=$GRAFT_REPO_ROOT/mitty_amd/_lib/v_SEAMINLINE/libmitty_hip.so
MH_LIB=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > $O/pytest_seaminline.log 2>&1 || { tail -30 $O/pytest_seaminline.log; exit 1; }
grep -E "passed|failed" $O/pytest_seaminline.log | tail -2
TAG=r04q REPS=2 bash scripts/gpu_ab.sh 'base:' "seam:MH_LIB=$V" || exit $?
TAG=r04q_cr REPS=1 BENCH_ARGS="--workload chr1 --corrupt --steps 8 --warmup 2" bash scripts/gpu_ab.sh 'base:' "seam:MH_LIB=$V" || exit $?
echo done
