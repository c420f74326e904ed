# bench A/B of the sampling lanes (MH_LANES 2 vs 4), three rounds on one box
mkdir -p gpurun_out
TAG=${1:-lanes}
for rep in 1 2 3; do
  for l in 2 4; do
    MH_LANES=$l timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_l$l.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/${TAG}_l$l.log "lanes=$l" | cut -c1-100
  done
done
