#!/bin/bash
# k_cr_cols one triple draw at a time (MH_CR_COLS_G3=1, with MH_CR_COLS_MW=8: 61 VGPRs, 8 waves/SIMD): corruption
# tests under the knob, then chr1-corrupt A/B against the default, and kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03i2}
MH_CR_COLS_G3=1 MH_CR_COLS_MW=8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "corrupt or Corrupt" --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1 || { tail -30 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for p in d g3 g38 d g3 g38; do
  case $p in d) E="X=0";; g3) E="MH_CR_COLS_G3=1";; g38) E="MH_CR_COLS_G3=1 MH_CR_COLS_MW=8";; esac
  env $E timeout -k 10 200 python -u bench.py --workload chr1 --corrupt --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_${T}_$p.json 2>gpurun_out/bench_${T}_$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_$p.json')); print('chr1 corrupt $p', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3), 'rows', round(d['corrupt_pass']['avg_launch_ms'],3))"
done
