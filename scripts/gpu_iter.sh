# Iteration check: GPU parity tests, decode pass diagnostics, steady-state bench
set -o pipefail
mkdir -p gpurun_out/iter
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/iter/pytest.log 2>&1 && \
MH_DEC_VERBOSE=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/iter/diag.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/iter/bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 3 gpurun_out/iter/pytest.log
grep decode gpurun_out/iter/diag.log | tail -n 3
python3 -c "import json;d=json.loads(open('gpurun_out/iter/bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['stage_ms'])"
