#!/bin/bash
# Position-major corruption rows: knob A/B on the chr1 corrupt bench (all MH_CR_ROWS=1): register budget for 8 waves
# (MH_CR_COLS_MW=8), templates per workgroup (MH_CR_COLS_PER), seams stored by the seam pass (MH_EW_DBG=256).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03d}
for p in c mw8 p2k p8k s256 c mw8 p8k s256; do
  case $p in c) E="X=0";; mw8) E="MH_CR_COLS_MW=8";; p2k) E="MH_CR_COLS_PER=2048";; p8k) E="MH_CR_COLS_PER=8192";; s256) E="MH_EW_DBG=256";; esac
  env MH_CR_ROWS=1 $E timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$p.json 2>gpurun_out/bench_${T}_$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$p.json')); print('chr1 corrupt rows $p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
