# Shuffle-decode diagnostics: queued chunks per pass by log2(start), then a kernel trace of one bench step
set -o pipefail
mkdir -p gpurun_out/dec
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
MH_DEC_VERBOSE=2 MH_DEC_BATCH=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/dec/diag.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dec/trace -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/dec/trace.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 3 gpurun_out/dec/diag.log
