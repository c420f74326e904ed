# GPU tests, then PMC passes of k_bam_write on a small tumor/normal bench.  usage: bash scripts/gpu_bampmc.sh TAG
mkdir -p gpurun_out
TAG=${1:-bamw}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ "$rc" = 0 ] || exit $rc
bash scripts/gpu_pmc.sh $TAG k_bam_write "--tumor-normal --tn-length 10000000" || exit $?
python3 scripts/pmc_print.py $TAG
