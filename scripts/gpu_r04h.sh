#!/bin/bash
# Round 4: the deflate parse after the walk-only extension (parity + rate), the tumor/normal step's regression
# (async vs sync tail, a kernel trace), the chr1 line with its end-to-end leg in a fresh process, the full-size
# verify.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "bgzf or fifos_and_gz or god_aligner or tumor_normal_mix or e2e" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bgzf -o run -- \
  python3 scripts/bgzf_rate.py --mb 1024 --reps 3 > $O/bgzf_rate.json 2>&1 || exit $?
tail -1 $O/bgzf_rate.json; grep -h "k_bgzf_blocks" $(find $O/bgzf -name '*kernel_stats.csv') | cut -d, -f1-4
timeout -k 10 300 python -u bench.py --tumor-normal --steps 4 --warmup 1 > $O/tn_async.json 2> $O/tn_async.err || exit $?
timeout -k 10 300 python -u bench.py --tumor-normal --steps 4 --warmup 1 --sync-tail > $O/tn_sync.json 2> $O/tn_sync.err || exit $?
python3 -c "
import json
for k in ('async', 'sync'):
  d = json.load(open('$O/tn_%s.json' % k)); print('tn', k, round(d['ms_per_step'], 2), d['bam_file_gpu']['seconds'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tnprof -o run -- \
  python3 bench.py --tumor-normal --steps 3 --warmup 1 > $O/tnprof.log 2>&1 || exit $?
timeout -k 10 420 python -u bench.py --workload chr1 --steps 8 --warmup 2 --no-cpu-config0 > $O/chr1.json 2> $O/chr1.err || exit $?
python3 -c "
import json; d = json.load(open('$O/chr1.json')); e = d.get('end_to_end') or {}
print('chr1', d['value'], d['ms_per_step']); print('e2e', e.get('seconds'), e.get('split_s'), e.get('stages_ms', {}).get('output_d2h'))
g = e.get('gz') or {}; print('gz', g.get('seconds'), g.get('split_s'), {k: v for k, v in (g.get('stages_ms') or {}).items() if 'bgzf' in k})"
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; tail -2 $O/verify.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/verify.json')); print('verify', d['verify'])"
echo done
