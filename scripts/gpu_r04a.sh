#!/bin/bash
# Round 4, first call: the new GPU tests (RCCL world 1, scan fault report), the default bench line (WGS CPU baseline,
# read-only frac), the full-size --verify step, the nccl bench at N = 1, and the writer's phase costs on WGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rccl.py tests/test_gpu_parity.py::test_scan_timeout_is_reported tests/test_gpu_parity.py::test_device_bgzf_round_trip > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['cpu_baseline']; r=d['roofline']; print('cpu', c['value'], c['cores'], c['sample']); print('read_only_frac', r['read_only_frac'], 'span', d['span_ms'])"
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; tail -2 $O/verify.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/verify.json')); print('verify', d['verify'])"
MH_DIST_BACKEND=nccl timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_nccl.json 2> $O/bench_nccl.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_nccl.json')); print('nccl', d['value']/1e9, d['config']['collective_backend'], d['config']['world_size_seen'])"
for dbg in 1 8 16 9 17 24 25 32; do
  MH_EW_DBG=$dbg timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $O/dbg_$dbg.json 2> $O/dbg_$dbg.err || exit $?
  python3 -c "import json; d=json.load(open('$O/dbg_$dbg.json')); r=d['roofline']; print('dbg $dbg', round(d['value']/1e9,3), round(d['ms_per_step'],1), 'writer ms', round(r['avg_launch_ms'],3))"
done

timeout -k 10 120 ./scripts/calib_writer > $O/calib_writer.json || exit $?
cat $O/calib_writer.json
echo done
