#!/bin/bash
# The round's record: the whole GPU suite (parity, RCCL at world size 1, the 100-unit genome plan) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -2
echo done
