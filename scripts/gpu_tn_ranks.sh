#!/bin/bash
# configs[4] across ranks rehearsed on one GPU (gloo ranks sharing it) and the one-GPU line beside it:
#   bash scripts/gpu_tn_ranks.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tnr}
mkdir -p $O
export MH_DIST_BACKEND=gloo
timeout -k 10 300 python -u bench.py --tumor-normal --gpus 2 --steps 3 --warmup 1 --tn-length 20000000 \
  > $O/tn2.json 2> $O/tn2.err || { tail -20 $O/tn2.err; exit 1; }
cat $O/tn2.json | cut -c1-600
timeout -k 10 300 python -u bench.py --tumor-normal --gpus 3 --steps 2 --warmup 1 --tn-genome --genome-scale 0.01 \
  > $O/tn3g.json 2> $O/tn3g.err || { tail -20 $O/tn3g.err; exit 1; }
cat $O/tn3g.json | cut -c1-600
