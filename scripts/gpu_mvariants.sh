# Timing experiments for k_emit_measure: MH_MEASURE_DBG variants (results are not valid FASTQ).
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2}; do
  MH_MEASURE_DBG=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mvar_$v.log 2>&1
  rc=$?
  echo "mvariant $v rc=$rc: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/mvar_$v.log').read().strip().splitlines()[-1]); print(d['stage_ms'].get('emit_measure'))" 2>&1)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
