#!/bin/bash
# The GPU test suite (optionally a -k expression) and the driver's smoke, each under its own time limit:
#   bash scripts/gpu_suite.sh TAG [KEXPR]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-t}
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  "${K[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -60; tail -30 gpurun_out/pytest_$TAG.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
