#!/bin/bash
# Round 4, first call: parity of the new paths (asynchronous batch tail, hand-written permutation sort, writer
# variants, multi-token deflate parse, RCCL at world size 1), the WGS bench line, the writer and D2H calibrations,
# the first A/B arms and a kernel trace.  (scripts/gpu_r04d.sh: the full-size verify and the other arms.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "async_tail or philox_corruption or direct_writer_matches or e2e or templates_golden or templates_vs_oracle or batched_units or forward_haplotype or writer_variants or writer_gate_pipelined or scan_timeout or bgzf or fifos_and_gz or god_aligner_from_device or tumor_normal_mix or unit_vs_oracle_2mbp" \
  tests/test_gpu_rccl.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['cpu_baseline']; r=d['roofline']; print('cpu', c['value'], c['cores'], c['sample']); print('read_only_frac', r['read_only_frac'], 'span', d['span_ms'])" || true
timeout -k 10 120 ./scripts/calib_writer > $O/calib_writer.json || exit $?
cat $O/calib_writer.json
timeout -k 10 120 python3 scripts/calib_d2h.py > $O/calib_d2h.json || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 120 python3 scripts/calib_d2h.py >> $O/calib_d2h.json || exit $?
cat $O/calib_d2h.json
TAG=r04c REPS=1 bash scripts/gpu_ab.sh 'base:' 'synctail: -- --sync-tail' 'lsd:MH_SORT=lsd' 'fwd:MH_HAP_FWD=1' || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit $?
KT=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > $O/gaps.txt 2>&1; tail -32 $O/gaps.txt
gzip -f "$KT"
echo done
