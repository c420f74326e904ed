# round profile: PMC passes of the writer, then kernel-trace runs of the bench (synchronous and pipelined emission)
TAG=${1:-r02q}
bash scripts/gpu_pmc.sh $TAG k_emit_tiles || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in sync async; do
  A=""; [ $mode = async ] && A="--async-emit"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG}_$mode -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e $A > gpurun_out/prof_${TAG}_$mode.log 2>&1 || exit $?
  python3 scripts/bsum.py gpurun_out/prof_${TAG}_$mode.log $mode
done
