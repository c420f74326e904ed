#!/bin/bash
# Round 4: NUMA-local staging (e2e parity + the e2e leg), the deflate rate with pass 2 replaying pass 1's tokens,
# the configs[4] line, and the writer's PMC passes on the WGS line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "e2e or fifos_and_gz or god_aligner or bgzf or tumor_normal" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "
import json; d = json.load(open('$O/bench.json')); e = d['end_to_end']
print('e2e', round(e['seconds'], 3), round(e['value'] / 1e6, 1), e['split_s'], e['stages_ms'].get('output_d2h'))
g = e['gz']; print('gz', round(g['seconds'], 3), round(g['value'] / 1e6, 1), g['split_s'], {k: v for k, v in g['stages_ms'].items() if 'bgzf' in k})"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bgzf -o run -- \
  python3 scripts/bgzf_rate.py --mb 1024 --reps 3 > $O/bgzf_rate.json 2>&1 || exit $?
python3 -c "
import csv, glob
for r in csv.DictReader(open(glob.glob('$O/bgzf/*kernel_stats.csv')[0])):
  if 'bgzf' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 1), 'ms')"
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
bash scripts/gpu_pmc.sh r04wgs k_emit_tiles r04_wgs wgs 150 3095693981 || exit $?
echo done
