# GPU tests only (optionally a -k expression): bash scripts/gpu_tests.sh TAG [KEXPR]
mkdir -p gpurun_out
TAG=${1:-t}
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread "${K[@]}" \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -80; tail -40 gpurun_out/pytest_$TAG.log
exit $rc
