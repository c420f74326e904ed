# tile-prefix writer: the whole GPU suite, then the bench (synchronous and pipelined emission, corruption)
mkdir -p gpurun_out
TAG=${1:-tiles}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/bs_$TAG.log 2>&1 || exit $?
python3 scripts/bsum.py gpurun_out/bs_$TAG.log sync
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --async-emit > gpurun_out/ba_$TAG.log 2>&1 || exit $?
python3 scripts/bsum.py gpurun_out/ba_$TAG.log async
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --corrupt > gpurun_out/bc_$TAG.log 2>&1 || exit $?
python3 scripts/bsum.py gpurun_out/bc_$TAG.log corrupt
