# Parity subset + A/B bench of an env switch + kernel trace: bash scripts/gpu_ab2.sh TAG "ENV=VAL" [KEXPR]
mkdir -p gpurun_out
TAG=${1:-ab}
ALT=${2:-MH_EMIT_SLOTS=1}
KEXPR=${3:-"unit_vs_oracle or e2e or chr1 or corruption or slices or pipelined or batched or god_aligner_from"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  -k "$KEXPR" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_new$k.log 2>&1 || exit $?
  env $ALT timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_alt$k.log 2>&1 || exit $?
  python3 - "$TAG" "$k" <<'PY'
import json, sys
for v in ('new', 'alt'):
    d = json.loads(open('gpurun_out/bench_{}_{}{}.log'.format(sys.argv[1], v, sys.argv[2])).read().strip().split('\n')[-1])
    print(v, round(d['value'] / 1e9, 4), 'G/s', round(d['ms_per_step'], 2), 'ms  writer', round(d['roofline']['avg_launch_ms'], 3),
          'ms frac', round(d['roofline']['frac'], 3), {k: d['stage_ms'][k] for k in ('emit_measure', 'emit_write', 'sample', 'splice') if k in d['stage_ms']})
PY
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1
echo "rocprof rc=$?"
python3 scripts/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 12 14
