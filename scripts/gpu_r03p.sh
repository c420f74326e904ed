#!/bin/bash
# Scaling projection: rank 0's share of the N-rank LPT plan timed alone on this GPU (N = 2, 4, 8), with at least 4
# batches per rank (default) and with one batch per rank (the old sizing at N = 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03p}
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_n1.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_n1.json')); print('N=1', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['config']['batches_rank0'])"
for n in 2 4 8; do
  for mb in 4 1; do
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --plan-share 0/$n --min-batches $mb > gpurun_out/bench_${T}_n${n}_mb$mb.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_n${n}_mb$mb.json')); print('rank0 of $n mb$mb', round(d['value']/1e9,3), round(d['ms_per_step'],2), d['config']['batches_rank0'], d['projection'])"
  done
done
for sw in 1 0; do
  MH_SORT_WAIT=$sw timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_sw$sw.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_sw$sw.json')); print('wgs sort-wait $sw', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
