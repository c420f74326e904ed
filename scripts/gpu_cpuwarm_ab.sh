#!/bin/bash
# The first-process question on one box (DESIGN.md "the first process"): run A after the host's cores spin 15 s, then
# 60 s idle, run B cold, then run C warm.  bash scripts/gpu_cpuwarm_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cpuwarm_$1
mkdir -p $O
spin() {
  python3 -c "
import multiprocessing as mp, time
def spin(t):
  e = time.time() + t
  while time.time() < e: pass
with mp.Pool(16) as p: p.map(spin, [float($1)] * 16)
"
}
run() {
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-prime --no-cpu-baseline --no-e2e > $O/$1.json 2> $O/$1.err || exit $?
  python3 scripts/bsum.py $O/$1.json "$1" || true
}
spin 15 && run A_spun
for i in 1 2 3 4 5 6; do sleep 10; echo "idle $((i*10))"; done
run B_cold
run C_warm
echo done
