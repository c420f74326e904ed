#!/bin/bash
# Round 4: the BAI mark kernel's wave-reduced window count and the kept BAM buffers (god-aligner parity, the
# 10-step configs[4] line), the e2e fetch variants, a PMC pass on the deflate kernel, the full-size verify, and the
# default bench line with its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "god_aligner or tumor_normal or lsd_sort or async_tail or bgzf" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', round(d['ms_per_step'],2), d['value'], d['bam_file_gpu']['seconds'], d['with_bam_file']['value'])" || true
timeout -k 10 300 python3 -u scripts/calib_fetch_e2e.py > $O/calib_fetch.json 2> $O/calib_fetch.err || exit $?
cat $O/calib_fetch.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  --kernel-include-regex k_bgzf_blocks --output-format csv -d $O/pmc_bgzf -o run -- python3 scripts/bgzf_rate.py --mb 256 --reps 1 > $O/pmc_bgzf.log 2>&1
echo "pmc rc=$?"
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; tail -2 $O/verify.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/verify.json')); print('verify', d['verify'])"
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit $?
echo done
