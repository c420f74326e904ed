# full GPU test suite, then the perfect and corrupt bench lines: bash scripts/gpu_full.sh TAG
mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e > gpurun_out/benchcr_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/benchcr_$TAG.log | cut -c1-400
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
