#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mem
timeout -k 10 420 python -u bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-e2e > gpurun_out/mem/n1.json 2> gpurun_out/mem/n1.err || { tail -5 gpurun_out/mem/n1.err; exit 1; }
python3 scripts/bsum.py gpurun_out/mem/n1.json n1 | cut -c1-80
python3 -c "import json; d=json.load(open('gpurun_out/mem/n1.json')); print('peak GiB', d['device_peak_gib'])"
bash scripts/gpu_rehearse2.sh && bash scripts/gpu_projection.sh
