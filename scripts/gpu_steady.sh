# Steady-state bench (more steps) and a kernel trace of it
set -o pipefail
mkdir -p gpurun_out/steady
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/steady/bench10.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/steady/trace -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/steady/trace.log 2>&1
rc=$?
echo "rc=$rc"
python3 -c "import json;d=json.loads(open('gpurun_out/steady/bench10.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
