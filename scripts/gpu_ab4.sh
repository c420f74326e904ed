# step time of the emission modes with and without the stage wait, each twice (noise on the pool is about +-3 %)
for rep in 1 2; do
  for w in 1 0; do
    MH_STAGE_WAIT=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab4_s$w.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/ab4_s$w.log "sync wait=$w" | cut -c1-80
    MH_STAGE_WAIT=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --async-emit > gpurun_out/ab4_a$w.log 2>&1 || exit $?
    python3 scripts/bsum.py gpurun_out/ab4_a$w.log "async wait=$w" | cut -c1-80
  done
done
