# Iteration check: GPU parity tests, then an interleaved A/B (VARS) of the steady-state bench
set -o pipefail
mkdir -p gpurun_out/iter
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/iter/pytest.log 2>&1 || { tail -n 40 gpurun_out/iter/pytest.log; exit 1; }
tail -n 2 gpurun_out/iter/pytest.log
bash scripts/gpu_ab.sh
