#!/bin/bash
# Round 4: the deflate parse with aligned word loads and reused hashes, pass 2 with packed codes and token loads a
# step ahead (parity, phase clocks); the device block cache (the e2e leg after the WGS steps); configs[4].
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "bgzf or gz or god_aligner or e2e or tumor_normal or async_tail" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 200 python -u scripts/calib_deflate.py > $O/calib_deflate.json 2> $O/calib_deflate.err || exit $?
cat $O/calib_deflate.json
timeout -k 10 200 python -u scripts/calib_deflate.py --prof > $O/calib_deflate_prof.json 2> $O/calib_deflate_prof.err || exit $?
cat $O/calib_deflate_prof.json
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
python3 -c "
import json; d = json.load(open('$O/bench.json')); e = d['end_to_end']
print('e2e', round(e['seconds'], 3), round(e['value'] / 1e6, 1), e['split_s'], e['stages_ms'].get('output_d2h'))
g = e['gz']; print('gz', round(g['seconds'], 3), round(g['value'] / 1e6, 1), g['split_s'], {k: v for k, v in g['stages_ms'].items() if 'bgzf' in k})"
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
echo done
