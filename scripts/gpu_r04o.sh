#!/bin/bash
# Round 4: the deflate kernel with its wave index declared uniform (scalar parse walk): parity, phase clocks, the
# e2e .gz leg and configs[4]'s BAM file; the writer's phase clocks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "bgzf or gz or god_aligner or tumor_normal" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 200 python -u scripts/calib_deflate.py --prof > $O/calib_deflate_prof.json 2> $O/calib_deflate_prof.err || exit $?
cat $O/calib_deflate_prof.json
timeout -k 10 200 python -u scripts/calib_writer_phases.py > $O/calib_writer_phases.json 2> $O/calib_writer_phases.err || exit $?
cat $O/calib_writer_phases.json
timeout -k 10 300 python -u scripts/e2e_fresh.py > $O/e2e.json 2> $O/e2e.err || exit $?
cat $O/e2e.json
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
echo done
