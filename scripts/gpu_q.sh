# quick iteration: GPU tests selected by -k "$1", then bench lines for each extra argument set ("$2", "$3", ...;
# "-" = plain bench), summarised by scripts/bsum.py
mkdir -p gpurun_out
K="$1"; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  -k "$K" > gpurun_out/pytest_q.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_q.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_q.log | head -20; exit $rc; fi
i=0
for args in "$@"; do
  i=$((i+1))
  [ "$args" = "-" ] && args=""
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e $args > gpurun_out/bq_$i.log 2>&1 || exit $?
  python3 scripts/bsum.py gpurun_out/bq_$i.log "[$args]"
done
