#!/bin/bash
# configs[4]: the god-aligner parity tests, then the tumor/normal bench line twice (the BAM file leg's seconds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tn_check
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "god_aligner or tumor_normal or bgzf" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn_$rep.json 2> $O/tn_$rep.err || exit $?
  python3 -c "import json; d=json.load(open('$O/tn_$rep.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])"
done
echo done
