#!/bin/bash
# A development call: a -k selection of the GPU suite, then (optionally) one short bench line.
#   bash scripts/gpu_dev.sh TAG 'KEXPR' [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "$2" > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'PASSED|FAILED|ERROR|passed|failed' $O/pytest.log | tail -40
[ $rc = 0 ] || { grep -E "Error|error|assert" $O/pytest.log | head -30; exit $rc; }
shift 2
if [ $# -gt 0 ]; then
  timeout -k 10 420 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/bsum.py $O/bench.json || true
fi
