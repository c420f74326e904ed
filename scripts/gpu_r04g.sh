#!/bin/bash
# Round 4: the GPU suite (all but the full-size WGS verify), the D2H and deflate calibrations in the e2e setting,
# the A/B arms (async tail, hand-written sort, forward-only haplotypes, writer variants, gate, unit order) and the
# corruption arms (row pass vs rows computed in the writer), the tumor/normal + BAM line, then the full-size verify.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu \
  --deselect tests/test_gpu_wgs_full.py::test_wgs_full_step_every_unit_equals_oracle > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u scripts/calib_fetch_e2e.py > $O/calib_fetch.json 2> $O/calib_fetch.err || exit $?
cat $O/calib_fetch.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bgzf -o run -- \
  python3 scripts/bgzf_rate.py --mb 1024 --reps 3 > $O/bgzf_rate.json 2>&1 || exit $?
tail -1 $O/bgzf_rate.json; grep -h "k_bgzf" $(find $O/bgzf -name '*kernel_stats.csv') | cut -c1-200
TAG=r04g REPS=2 bash scripts/gpu_ab.sh 'base:' 'lsd:MH_SORT=lsd' 'fwd:MH_HAP_FWD=1' 'lsdfwd:MH_SORT=lsd MH_HAP_FWD=1' 'synctail: -- --sync-tail' 'g4:MH_EW_GATHER4=1' 'flat:MH_EW_FLAT=1' 'tail4:MH_WRITER_GATE_TAIL=4' 'copyorder: -- --unit-order copy' || exit $?
TAG=r04gc REPS=2 BENCH_ARGS='--workload chr1 --corrupt --steps 8 --warmup 2' bash scripts/gpu_ab.sh 'rows:' 'fused:MH_CR_FUSED=1' || exit $?
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', d['value'], d['ms_per_step'], d['bam_file_gpu'], d['with_bam_file']['value'])" || true
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; tail -2 $O/verify.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/verify.json')); print('verify', d['verify'])"
echo done
