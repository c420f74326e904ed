#!/bin/bash
# parity of the single-pass writer, then it alone (serialised) and on the line: bash scripts/gpu_fused_diag2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "single_pass or chr1_unit_fastq or batched_units_vs_oracle" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -2
bash scripts/gpu_iso.sh ${T}_fu "$@" || exit $?
O=gpurun_out/line_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof0 -o run -- \
  python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/bench0.json 2> $O/bench0.err || exit $?
python3 scripts/bsum.py $O/bench0.json mode0 || true
python3 scripts/kstats.py $(ls $O/prof0/*kernel_stats.csv | head -1) 8 12
