#!/bin/bash
# Round 4: the writer gate on a batch's last D writers (MH_WRITER_GATE_TAIL=D) against the default, on the WGS line,
# in alternation; then a kernel trace of the default for the writer-stream gaps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "forward_haplotype or philox_corruption_vs_numpy or writer_gate_pipelined" > /tmp/r04b_pytest.log 2>&1; rc=$?; tail -3 /tmp/r04b_pytest.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 120 ./scripts/calib_writer > $O/calib_writer.json || exit $?
cat $O/calib_writer.json
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > $O/b_$tag.json 2> $O/b_$tag.err || return $?
  python3 -c "import json; d=json.load(open('$O/b_$tag.json')); r=d['roofline']; print('$tag', round(d['value']/1e9,4), round(d['ms_per_step'],2), 'writer', round(r['avg_launch_ms'],3))"
}
for rep in 1 2; do
  run base$rep MH_X=0 || exit $?
  run fwd$rep MH_HAP_FWD=1 || exit $?
  for D in 2 4 6; do run tail${D}_$rep MH_WRITER_GATE_TAIL=$D || exit $?; done
  run fwdtail4_$rep MH_HAP_FWD=1 MH_WRITER_GATE_TAIL=4 || exit $?
done
for o in copy; do
  env timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --unit-order $o > $O/b_order_$o.json 2>/dev/null || exit $?
  MH_HAP_FWD=1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --unit-order $o > $O/b_order_fwd_$o.json 2>/dev/null || exit $?
  for t in order_$o order_fwd_$o; do python3 -c "import json; d=json.load(open('$O/b_$t.json')); r=d['roofline']; print('$t', round(d['value']/1e9,4), round(d['ms_per_step'],2), 'writer', round(r['avg_launch_ms'],3))"; done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit $?
KT=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/wgs_gaps.py "$KT" > $O/gaps.txt 2>&1; tail -30 $O/gaps.txt
gzip -f "$KT"
echo done
