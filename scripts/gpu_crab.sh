# GPU tests, then the corrupt bench A/B of per-file corruption workgroups (MH_CR_PERFILE=0: both files' tables)
mkdir -p gpurun_out
TAG=${1:-crab}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ "$rc" = 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    MH_CR_PERFILE=$v timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_p$v.log 2>&1 || exit $?
    python3 scripts/crsum.py gpurun_out/${TAG}_p$v.log "perfile=$v"
  done
done
