# GPU tests, a kernel trace of the gated bench, then bench A/B of the writer gate (MH_WRITER_GATE = the index of the
# first writer that waits; -1 off)
mkdir -p gpurun_out
TAG=${1:-gate}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ "$rc" = 0 ] || exit $rc
bash scripts/gpu_trace.sh ${TAG}tr > gpurun_out/${TAG}_trace.txt 2>&1; head -45 gpurun_out/${TAG}_trace.txt
for rep in 1 2; do
  for g in 2 -1 1 3; do
    MH_WRITER_GATE=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_g$g.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_g$g.log "gate=$g" | cut -c1-100
  done
done
