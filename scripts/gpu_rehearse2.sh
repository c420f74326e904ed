#!/bin/bash
# The N = 2 bench path rehearsed on one GPU: two ranks under torch.distributed.run, gloo for the count all-reduce
# (RCCL needs a GPU per rank), the metric's workload dealt by LPT.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rehearse2
mkdir -p $O
MH_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
  > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python3 scripts/bsum.py $O/bench2.json rehearse2 || true
echo done
