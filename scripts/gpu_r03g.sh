#!/bin/bash
# Corruption pass defaults on one box: fast full-block path (MH_CR_DBG=0) or guarded per-base path (1), at 1024 or 512
# threads per workgroup (MH_CR_THR), alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03g}
for rep in 1 2; do
  for v in "1024 0" "1024 1" "512 0" "512 1"; do
    set -- $v
    MH_CR_THR=$1 MH_CR_DBG=$2 timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$1_$2_$rep.json 2>gpurun_out/bench_${T}_$1_$2_$rep.err || exit $?
    python3 scripts/crsum.py gpurun_out/bench_${T}_$1_$2_$rep.json "thr=$1 dbg=$2 rep$rep"
  done
done
