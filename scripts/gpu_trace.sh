# rocprofv3 kernel trace + stats of the default bench (8 timed steps), then the step timeline and the per-kernel
# summary.  usage: bash scripts/gpu_trace.sh TAG [bench args...]
set -o pipefail
mkdir -p gpurun_out/prof
TAG=${1:-tr}; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e "$@" > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ "$rc" = 0 ] || exit $rc
python3 scripts/bsum.py gpurun_out/prof_bench_$TAG.log "$TAG" | cut -c1-100
KT=$(find gpurun_out/prof/$TAG -name '*kernel_trace.csv' | head -1)
python3 scripts/tl_detail.py "$KT" > gpurun_out/timeline_$TAG.txt 2>&1; cat gpurun_out/timeline_$TAG.txt
python3 scripts/kstats.py $(find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1) 10 2>&1 | head -30
