#!/bin/bash
# Why does the first bench process on a fresh box run slow?  Arm given as $1 (one arm per gpurun call, so that its
# first bench is the call's first GPU process); every bench runs without the priming pass (--no-prime):
#   none    — straight away
#   inproc  — scripts/prime_hbm.py's pass (most of the HBM in 1 GiB blocks, written, freed) inside the first bench
#             process (scripts/inproc_prime_bench.py; PRIME_WRITE=0: allocated and freed, not written)
#   sleep   — the box idles $2 seconds first
#   cpuspin — 16 host processes spin $2 seconds first (no GPU use)
# Round 5 also ran library variants (since removed): the buffers carved from one 250-271 GiB block, the free HBM
# reserved in one block and released, every new block zeroed, hipDeviceMallocContiguous — DESIGN.md "the first
# process" has the numbers.  Then a second bench process as the warm reference.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fresh_$1
mkdir -p $O
date +%s.%N > $O/t0
(rocm-smi --showmemuse --showuse --json > $O/smi0.json 2>&1 || true)
E="${ARM_ENV:-}"
if [ "$1" = cpuspin ]; then   # the host's cores busy for $2 seconds first (no GPU use)
  grep MHz /proc/cpuinfo | head -4 > $O/cpumhz_before.txt
  python3 -c "
import multiprocessing as mp, time
def spin(t):
  e = time.time() + t
  while time.time() < e: pass
with mp.Pool(16) as p: p.map(spin, [float($2)] * 16)
"
  grep MHz /proc/cpuinfo | head -4 > $O/cpumhz_after.txt
fi
if [ "$1" = sleep ]; then
  for i in $(seq 1 $(( $2 / 10 ))); do sleep 10; echo "slept $((i*10))"; done
fi
for i in 1 2; do
  if [ "$1" = inproc ] && [ $i = 1 ]; then B="scripts/inproc_prime_bench.py"; else B=bench.py; fi
  env $E timeout -k 10 300 python -u $B --steps 8 --warmup 2 --no-prime --no-cpu-baseline --no-e2e > $O/run$i.json 2> $O/run$i.err || exit $?
  python3 scripts/bsum.py $O/run$i.json "run$i" || true
done
echo done
