#!/bin/bash
# Why does the first bench process on a fresh box run slow?  Arm given as $1:
#   sleep  — the box idles (no GPU use) for $2 seconds first, then the bench without the HBM prime pass
#   none   — the bench without the prime pass straight away
#   inproc — the prime pass inside the first bench process (scripts/inproc_prime_bench.py)
#   arena  — the first bench process with MH_ARENA_GB=$2 (the library's device blocks carved from one big block)
#   (round 5 also ran `contig`: the library's buffers >= 64 MiB from hipExtMallocWithFlags(hipDeviceMallocContiguous):
#   1.15 / 1.28 G/s, slower in both processes — gpurun_out/fresh_contig, profiles/r05/fresh/)
# then a second bench process (no prime) as the warm reference.  Each line records rocm-smi's memory use before it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fresh_$1
mkdir -p $O
date +%s.%N > $O/t0
(rocm-smi --showmemuse --showuse --json > $O/smi0.json 2>&1 || true)
if [ "$1" = sleep ]; then
  for i in $(seq 1 $(( $2 / 10 ))); do sleep 10; (rocm-smi --showmemuse --showuse --json > $O/smi_sleep_$i.json 2>&1 || true); echo "slept $((i*10))"; done
fi
for i in 1 2; do
  if [ "$1" = inproc ] && [ $i = 1 ]; then B="scripts/inproc_prime_bench.py"; else B=bench.py; fi
  E=""; if [ "$1" = arena ] && [ $i = 1 ]; then E="MH_ARENA_GB=$2"; fi
  env $E timeout -k 10 300 python -u $B --steps 8 --warmup 2 --no-prime --no-cpu-baseline --no-e2e > $O/run$i.json 2> $O/run$i.err || exit $?
  python3 scripts/bsum.py $O/run$i.json "run$i" || true
done
echo done
