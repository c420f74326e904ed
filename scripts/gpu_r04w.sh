#!/bin/bash
# Round 4: a batch's unit 0 measured and written before the next units are prepared (the writer stream's wait at a
# batch boundary): parity of the paths that use run_units, then the A/B against the chunked order.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "e2e or async_tail or golden or chr1 or batch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
TAG=r04w REPS=3 bash scripts/gpu_ab.sh 'unit0:' 'chunk: -- --unit0-in-chunk' || exit $?
echo done
