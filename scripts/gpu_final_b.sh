#!/bin/bash
# Round record, part B: configs[4] (default and chr1-size), configs[2] corrupt, configs[1] chr1, the device deflate's
# kernel statistics, the RCCL N = 1 line, and the N-GPU projection (rank 0's share, ratios against this call's N = 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_b
mkdir -p $O
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --no-cpu-baseline --no-e2e > $O/corrupt.json 2> $O/corrupt.err || exit $?
python3 scripts/bsum.py $O/corrupt.json corrupt || true
timeout -k 10 300 python -u bench.py --workload chr1 --no-cpu-baseline --no-e2e > $O/chr1.json 2> $O/chr1.err || exit $?
python3 scripts/bsum.py $O/chr1.json chr1 || true
MH_DIST_BACKEND=nccl timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-e2e > $O/bench_nccl.json 2> $O/bench_nccl.err || exit $?
python3 scripts/bsum.py $O/bench_nccl.json nccl || true
for n in 1 2 4 8; do
  if [ $n -eq 1 ]; then extra=""; else extra="--plan-share 0/$n"; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e $extra > $O/proj_n$n.json 2> $O/proj_n$n.err || exit $?
  python3 scripts/bsum.py $O/proj_n$n.json proj_n$n || true
done
echo done
