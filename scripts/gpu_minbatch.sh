#!/bin/bash
# Batches per rank at N = 8 and N = 4 (rank 0's LPT share alone, --plan-share): --min-batches 1, 2, 3, 4 (default 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/minbatch
mkdir -p $O
for share in ${SHARES:-0/8 0/4}; do
  for mb in ${MBS:-4 2 3 1}; do
    tag=$(echo $share | tr / _)_mb$mb
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --plan-share $share \
      --min-batches $mb > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('$O/$tag.json') if l.startswith('{')][-1]; print('$tag', round(d['value']/1e9,4), round(d['ms_per_step'],2), d['config'].get('batches_rank0'))"
  done
done
echo done
