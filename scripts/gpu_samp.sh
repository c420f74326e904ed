# sampling parity tests + perfect bench + trace timeline: bash scripts/gpu_samp.sh TAG
mkdir -p gpurun_out
TAG=${1:-samp}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  -k "template or chr1 or unit or e2e or philox_sampling" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
bash scripts/gpu_steady.sh $TAG | head -40
