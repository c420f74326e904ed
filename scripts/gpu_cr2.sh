# corruption tests + corrupt/perfect bench lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "corrupt or philox or slices" > gpurun_out/pytest_cr2.log 2>&1
rc=$?
grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_cr2.log | tail -40; tail -30 gpurun_out/pytest_cr2.log | grep -v PASSED
[ $rc -ne 0 ] && exit $rc
for m in "--corrupt" ""; do
  timeout -k 10 300 python -u bench.py $m --no-cpu-baseline --no-e2e --steps 6 --warmup 2 --stages > gpurun_out/b_cr2$m.log 2>&1 || exit $?
  tail -2 gpurun_out/b_cr2$m.log | cut -c1-900
done
