#!/bin/bash
# The round's record: the bench line (metric, CPU baseline, end to end), its kernel statistics under rocprofv3, the
# full-size byte check, configs[1] / [2] / [4] lines, the device deflate's kernel statistics, the RCCL N = 1 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_bench
mkdir -p $O
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "
import json; d = json.load(open('$O/bench.json')); e = d['end_to_end']
print('e2e', round(e['seconds'], 3), round(e['value'] / 1e6, 1), 'gz', round(e['gz']['seconds'], 3), round(e['gz']['value'] / 1e6, 1))
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python3 scripts/bsum.py $O/bench_prof.json prof || true
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/verify.err; exit $rc; }
python3 -c "import json; d=json.load(open('$O/verify.json')); v=d['verify']; print('verify', v['units'], v['units_equal'], v['templates_kept'])"
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
timeout -k 10 300 python -u bench.py --workload chr1 --corrupt --no-cpu-baseline --no-e2e > $O/corrupt.json 2> $O/corrupt.err || exit $?
python3 scripts/bsum.py $O/corrupt.json corrupt || true
timeout -k 10 300 python -u bench.py --workload chr1 --no-cpu-baseline --no-e2e > $O/chr1.json 2> $O/chr1.err || exit $?
python3 scripts/bsum.py $O/chr1.json chr1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bgzf -o run -- \
  python3 scripts/bgzf_rate.py --mb 1024 --reps 3 > $O/bgzf_rate.json 2>&1 || exit $?
python3 -c "
import csv, glob
for r in csv.DictReader(open(glob.glob('$O/bgzf/*kernel_stats.csv')[0])):
  if 'bgzf' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 1), 'ms')"
MH_DIST_BACKEND=nccl timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-e2e > $O/bench_nccl.json 2> $O/bench_nccl.err || exit $?
python3 scripts/bsum.py $O/bench_nccl.json nccl || true
echo done
