#!/bin/bash
# Clock trace around a first and a second bench process (the fresh-box question, DESIGN.md "the first process"):
# rocm-smi's clocks, power and activity sampled every second into gpurun_out/clk_TAG/trace.txt while the box idles
# IDLE seconds, then runs bench (no arena) twice.   bash scripts/gpu_clock_trace.sh TAG IDLE
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/clk_$1
mkdir -p $O
( while true; do
    echo "t=$(date +%s.%N)"
    rocm-smi --showclocks --showpower --showuse --showmemuse 2>/dev/null | grep -E "sclk|mclk|fclk|socclk|Power|use" | head -12
    sleep 1
  done ) > $O/trace.txt 2>&1 &
SP=$!
sleep ${2:-10}
for i in 1 2; do
  echo "run$i start $(date +%s.%N)" >> $O/marks.txt
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-prime --no-cpu-baseline --no-e2e > $O/run$i.json 2> $O/run$i.err || { kill $SP; exit 1; }
  echo "run$i end $(date +%s.%N)" >> $O/marks.txt
  python3 scripts/bsum.py $O/run$i.json "run$i" || true
done
kill $SP
echo done
