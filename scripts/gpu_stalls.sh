#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/host_stalls.py --steps 10 --warmup 10 --no-cpu-baseline --no-e2e > gpurun_out/stalls.json 2> gpurun_out/stalls.txt || { tail -20 gpurun_out/stalls.txt; exit 1; }
python3 scripts/bsum.py gpurun_out/stalls.json stalls | cut -c1-120
