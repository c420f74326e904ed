#!/bin/bash
# Where the corruption pass's time goes: timing-only knobs (MH_CR_DBG 2 no stores, 4 no base loads, 8 no Philox,
# 16 the item loop alone) on the chr1 corrupt bench; the bytes are wrong under every knob but 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03v}
for v in 0 2 4 8 6 14 16 0; do
  MH_CR_DBG=$v timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$v.json 2>gpurun_out/bench_${T}_$v.err || exit $?
  python3 scripts/crsum.py gpurun_out/bench_${T}_$v.json "dbg=$v"
done
for c in 8 7 6; do
  MH_WRITER_CUS=$c timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_wcu$c.json 2>gpurun_out/bench_${T}_wcu$c.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wcu$c.json')); print('wgs writer_cus=$c', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
