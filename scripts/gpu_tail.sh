# Decode-tail check: template parity at several tail cutoffs, then the steady-state bench per cutoff
set -o pipefail
mkdir -p gpurun_out/tail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k templates \
  --timeout 200 --timeout-method thread > gpurun_out/tail/pytest.log 2>&1 || { tail -n 30 gpurun_out/tail/pytest.log; exit 1; }
tail -n 2 gpurun_out/tail/pytest.log
for t in ${TAILS:-32768 65536 131072}; do
  echo -n "tail $t: "
  MH_DEC_TAIL=$t MH_DEC_VERBOSE=1 timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/tail/b$t.log 2>&1 || exit 1
  grep decode gpurun_out/tail/b$t.log | tail -n 1 | tr '\n' ' '
  python3 -c "import json;d=json.loads(open('gpurun_out/tail/b$t.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),d['stage_ms']['sample_shuffle_decode'])"
done
