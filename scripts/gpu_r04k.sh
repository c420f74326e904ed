#!/bin/bash
# Round 4: which HIP runtime the fetch runs on (the library's /opt/rocm one, as bench.py at N=1, vs torch's, as at
# N > 1), the batch-wide tail chase (parity + A/B), and the WGS line at world size 1 over RCCL.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "async_tail" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 200 python -u scripts/calib_fetch_e2e.py > $O/calib_fetch_rocm.json 2> $O/calib_fetch_rocm.err || exit $?
cat $O/calib_fetch_rocm.json
timeout -k 10 200 python -u scripts/calib_fetch_e2e.py --torch > $O/calib_fetch_torch.json 2> $O/calib_fetch_torch.err || exit $?
cat $O/calib_fetch_torch.json
timeout -k 10 200 python -u scripts/calib_deflate.py > $O/calib_deflate.json 2> $O/calib_deflate.err || exit $?
cat $O/calib_deflate.json
timeout -k 10 200 python -u scripts/calib_deflate.py --prof > $O/calib_deflate_prof.json 2> $O/calib_deflate_prof.err || exit $?
cat $O/calib_deflate_prof.json
TAG=r04k REPS=2 bash scripts/gpu_ab.sh 'base:' 'tailbatch:MH_TAIL_CHASE=batch' 'nccl:MH_DIST_BACKEND=nccl' || exit $?
echo done
