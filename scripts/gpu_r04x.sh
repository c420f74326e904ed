#!/bin/bash
# Round 4: the next batch sampled as soon as this batch's measure passes are queued (--sample-ahead): the full-size
# byte check on that order, then the A/B against the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify --sample-ahead \
  > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/verify.err; exit $rc; }
python3 -c "import json; d=json.load(open('$O/verify.json')); v=d['verify']; print('verify', v['units'], v['units_equal'])"
TAG=r04x REPS=3 bash scripts/gpu_ab.sh 'base:' 'ahead: -- --sample-ahead' || exit $?
echo done
