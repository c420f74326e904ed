# rocprofv3 kernel-trace summary of the default bench (kernel trace only; PMC passes are separate runs)
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof/$TAG -name '*stats*' | head
tail -2 gpurun_out/prof_bench_$TAG.log
