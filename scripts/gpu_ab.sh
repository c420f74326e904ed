# Interleaved A/B of env settings on the steady-state bench (VARS = space-separated KEY=VAL settings, X=0 = default)
mkdir -p gpurun_out/ab
cd "$GRAFT_REPO_ROOT"
for rep in ${REPS:-1 2}; do
  for v in ${VARS}; do
    echo -n "$v: "
    env $v timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline 2>/dev/null > gpurun_out/ab/o.log || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab/o.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),d['stage_ms']['sample_shuffle_decode'])"
  done
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  env $PROF timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/prof.log 2>&1
  grep -h "decode" gpurun_out/ab/prof/*stats.csv | cut -c1-160
fi
