# philox corruption tests + corrupt bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "philox_corruption or slices or direct_writer_matches" > gpurun_out/pytest_cr3.log 2>&1
rc=$?
grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_cr3.log | tail -40; tail -30 gpurun_out/pytest_cr3.log | grep -v PASSED
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e --steps 6 --warmup 2 --stages > gpurun_out/b_cr3.log 2>&1 || exit $?
tail -2 gpurun_out/b_cr3.log | cut -c1-700
