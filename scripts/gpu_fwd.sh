# GPU tests, then bench A/B of the mate-1 gather: the reverse-complement table (MH_HAP_RC=1) vs the forward
# haplotype complemented in registers (default).  usage: bash scripts/gpu_fwd.sh TAG
mkdir -p gpurun_out
TAG=${1:-fwd}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -20; tail -3 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then exit $rc; fi
for rep in 1 2; do
  for r in 1 0; do
    MH_HAP_RC=$r timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_rc$r.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_rc$r.log "rc=$r" | cut -c1-90
  done
done
