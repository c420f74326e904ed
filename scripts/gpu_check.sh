mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
if [ "$rc" = 0 ] || [ "$rc" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
  timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
  echo "smoke/bench rc=$?"
  tail -n 5 gpurun_out/smoke.log gpurun_out/bench.log
fi
