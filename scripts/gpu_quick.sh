# GPU tests + short bench (+ optional rocprofv3 kernel-trace of the bench)
# usage: bash scripts/gpu_quick.sh TAG [prof]
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -60; tail -4 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ] && [ "$rc" != 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.log
if [ "$rc" != 0 ]; then exit $rc; fi
if [ "$2" = prof ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1
  echo "rocprof rc=$?"
  find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec head -30 {} \;
fi
