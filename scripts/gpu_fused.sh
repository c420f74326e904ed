# emission modes of the asynchronous path: parity (asynchronous vs synchronous emission) in modes 1 and 2, then the
# bench per mode (MH_EMIT_FUSED: 1 measure + look-back writer, 2 all fused, 0 measure + scan + direct writer)
mkdir -p gpurun_out
TAG=${1:-fused}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "async or pipelined or e2e" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -20
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_$TAG.log; exit $rc; fi
MH_EMIT_FUSED=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "async" > gpurun_out/pytest2_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest2_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest2_$TAG.log
for mode in 1 0; do
  MH_EMIT_FUSED=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --async-emit > gpurun_out/b${mode}_$TAG.log 2>&1 || exit $?
  python3 scripts/bsum.py gpurun_out/b${mode}_$TAG.log mode$mode
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/bs_$TAG.log 2>&1 || exit $?
python3 scripts/bsum.py gpurun_out/bs_$TAG.log sync
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --async-emit --corrupt > gpurun_out/bc_$TAG.log 2>&1 || exit $?
python3 scripts/bsum.py gpurun_out/bc_$TAG.log corrupt-async
