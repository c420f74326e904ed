mkdir -p gpurun_out
TAG=${1:-h}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  -k "corrupt or slices or e2e or distributed" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ "$rc" != 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e > gpurun_out/benchcr_$TAG.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/benchcr_$TAG.log').read().strip().split('\n')[-1])
print('corrupt', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step'],2), 'ms writer', round(d['roofline']['avg_launch_ms'],3))"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().split('\n')[-1])
print('perfect', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step'],2), 'ms writer', round(d['roofline']['avg_launch_ms'],3), 'e2e', d['end_to_end'])"
MH_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --genome-scale 0.1 \
  > gpurun_out/bench2_$TAG.log 2>&1
echo "bench2 rc=$?"; tail -c 1200 gpurun_out/bench2_$TAG.log
