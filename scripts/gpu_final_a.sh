#!/bin/bash
# Round record, part A: the default bench line (metric, CPU baseline legs, end to end), its kernel statistics under
# rocprofv3, and the full-size byte check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_a
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "
import json; d = json.load(open('$O/bench.json')); e = d['end_to_end']
print('e2e', round(e['seconds'], 3), round(e['value'] / 1e6, 1), 'gz', round(e['gz']['seconds'], 3), round(e['gz']['value'] / 1e6, 1))
print('cpu', json.dumps(d['cpu_baseline'])[:400])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python3 scripts/bsum.py $O/bench_prof.json prof || true
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/verify.err; exit $rc; }
python3 -c "import json; d=json.load(open('$O/verify.json')); v=d['verify']; print('verify', v['units'], v['units_equal'], v['templates'])"
echo done
