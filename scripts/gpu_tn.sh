# GPU tests, the default bench line and the tumor/normal (configs[4]) bench line.  usage: bash scripts/gpu_tn.sh TAG
mkdir -p gpurun_out
TAG=${1:-tn}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -20; tail -3 gpurun_out/pytest_$TAG.log
[ "$rc" = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --tumor-normal --steps 3 --warmup 1 > gpurun_out/bench_tn_$TAG.log 2>&1
rc=$?
echo "bench tn rc=$rc"; tail -c 2500 gpurun_out/bench_tn_$TAG.log
