# GPU tests, then bench A/B of the number of sampling lanes (MH_LANES) and a kernel trace of the default
mkdir -p gpurun_out
TAG=${1:-lanes}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ "$rc" = 0 ] || exit $rc
for rep in 1 2; do
  for l in 4 2 3; do
    MH_LANES=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_l$l.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_l$l.log "lanes=$l" | cut -c1-100
  done
done
bash scripts/gpu_trace.sh ${TAG}tr > gpurun_out/${TAG}_trace.txt 2>&1; head -60 gpurun_out/${TAG}_trace.txt
