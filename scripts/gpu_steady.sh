# Steady-state bench and a kernel trace (+ stats) of it: bash scripts/gpu_steady.sh TAG
set -o pipefail
TAG=${1:-steady}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/$TAG/trace.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && exit $rc
T=$(find gpurun_out/$TAG/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$T" k_resolve full > gpurun_out/$TAG/timeline.txt
head -45 gpurun_out/$TAG/timeline.txt
tail -1 gpurun_out/$TAG/trace.log | cut -c1-300
