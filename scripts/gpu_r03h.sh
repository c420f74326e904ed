#!/bin/bash
# Device-deflated BAM (mh_bam_write_gpu): god-aligner GPU tests, then the tumor/normal bench with its BAM file legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r03h}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "god or bgzf or tumor" > gpurun_out/pytest_${T}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log
[ $rc = 0 ] || { grep -E "Error|assert|Fail" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --tumor-normal --steps 3 --warmup 1 > gpurun_out/bench_tn_${T}.json 2>gpurun_out/bench_tn_${T}.err || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/bench_tn_${T}.json') if l.startswith('{')][-1]; print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; host bam', round(d['bam_file_after_timing']['seconds'],2), 's; gpu bam', round(d['bam_file_gpu']['seconds'],3), 's', d['bam_file_gpu']['file_bytes'], 'B; with file', round(d['with_bam_file']['value']/1e6,1), 'M/s')"
