# Round-end check: full GPU suite, bench lines (perfect, corrupt), a 2-rank rehearsal of the N>1 plan, kernel stats
mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e > gpurun_out/benchcr_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/benchcr_$TAG.log | cut -c1-300
MH_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --genome-scale 0.05 \
  > gpurun_out/bench2_$TAG.log 2>&1 || exit $?
grep '"metric"' gpurun_out/bench2_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
echo prof ok
timeout -k 10 400 python -u bench.py --tumor-normal --steps 3 --warmup 1 > gpurun_out/benchtn_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/benchtn_$TAG.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_proftn -o run -- \
  python3 bench.py --tumor-normal --steps 2 --warmup 1 > gpurun_out/${TAG}_proftn.log 2>&1 || exit $?
echo proftn ok
