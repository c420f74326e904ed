# asynchronous emission: parity tests, then the bench (pipelined and synchronous) and a steady-state timeline
mkdir -p gpurun_out
TAG=${1:-async}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "async or e2e or chr1_unit or corruption_statistics or nodes or splice or templates_golden or decode or resident or pipelined" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -20; tail -30 gpurun_out/pytest_$TAG.log | grep -v PASSED | tail -25
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/b_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/b_$TAG.log | cut -c1-330
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --async-emit > gpurun_out/bs_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bs_$TAG.log | cut -c1-330
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --corrupt > gpurun_out/bc_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bc_$TAG.log | cut -c1-330
