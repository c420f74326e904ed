#!/bin/bash
# A/B of environment variants on one bench line, alternating REPS times in one call.
# usage (inside gpurun): TAG=name REPS=2 BENCH_ARGS="--steps 8 --warmup 2" scripts/gpu_ab.sh 'base:' 'x:MH_LIB=path/to/other/libmitty_hip.so' ...
# Each argument is label:ENV=V ENV2=V2 (env may be empty), optionally followed by ' -- ' and extra bench arguments.  Prints value, ms/step and writer ms per run; JSON lines in
# gpurun_out/ab_$TAG/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
REPS=${REPS:-2}
BENCH_ARGS=${BENCH_ARGS:---steps 8 --warmup 2}
O=gpurun_out/ab_$TAG
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    label=${v%%:*}
    rest=${v#*:}
    envs=${rest%% -- *}
    extra=""
    [[ "$rest" == *" -- "* ]] && extra=${rest#* -- }
    env $envs timeout -k 10 300 python -u bench.py $BENCH_ARGS $extra --no-cpu-baseline --no-e2e > $O/${label}_$rep.json 2> $O/${label}_$rep.err || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('$O/${label}_$rep.json') if l.startswith('{')][-1]; r=d['roofline']; print('$label', $rep, round(d['value']/1e9,4), round(d['ms_per_step'],2), 'writer', round(r['avg_launch_ms'],4))"
  done
done
