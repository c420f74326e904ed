# A/B of an environment switch on the bench: bash scripts/gpu_ab_env.sh VAR "v1 v2 .." "bench args"
mkdir -p gpurun_out
VAR=$1; VALS=$2; ARGS=$3
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e $ARGS > gpurun_out/ab_${VAR}_$v.log 2>&1 || exit $?
  python3 scripts/bsum.py gpurun_out/ab_${VAR}_$v.log "$VAR=$v [$ARGS]"
done
