# bench A/B, three rounds: usage bash scripts/gpu_ab3.sh TAG "ENV=1" ["ENV=2" ...] (base always first)
mkdir -p gpurun_out
TAG=${1:-ab}; shift
for rep in 1 2 3; do
  i=0
  for v in base "$@"; do
    i=$((i+1))
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_v$i.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_v$i.log "$v" | cut -c1-90
  done
done
