# GPU tests (subset or all), the default bench (N=1 with end-to-end + CPU baseline legs), and a 2-rank rehearsal of
# the multi-GPU genome plan on one GPU (gloo, scaled-down genome): bash scripts/gpu_bench_full.sh TAG [KEXPR]
mkdir -p gpurun_out
TAG=${1:-full}
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread "${K[@]}" \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_$TAG.log
if [ "$rc" != 0 ]; then exit $rc; fi
MH_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --genome-scale 0.1 \
  > gpurun_out/bench2_$TAG.log 2>&1
echo "bench2 rc=$?"; tail -c 1500 gpurun_out/bench2_$TAG.log
