# GPU tests, then bench A/B over environment settings (each "NAME=VAL[,NAME=VAL]" or "base"), repeated twice.
# usage: bash scripts/gpu_ab_env.sh TAG "base" "MH_HAP_RC=1" ...
mkdir -p gpurun_out
TAG=${1:-ab}; shift
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E 'FAILED|ERROR' gpurun_out/pytest_$TAG.log | tail -20; tail -3 gpurun_out/pytest_$TAG.log
  if [ "$rc" != 0 ]; then exit $rc; fi
fi
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_v$i.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_v$i.log "$v" | cut -c1-100
  done
done
