#!/bin/bash
# The default bench line as the first process on a fresh box, with its HBM first-touch pass; then the two-rank
# rehearsal (each rank primes its own GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/primecheck
mkdir -p $O
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/bsum.py $O/bench.json first || true
grep prime_hbm $O/bench.err || true
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['setup_s'], d['warmup'])"
echo done
