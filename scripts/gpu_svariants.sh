# Timing experiments for k_mt_segments: MH_MT_DBG variants (1 no jump, 2 no twists, 4 no stores; invalid output).
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 4}; do
  MH_MT_DBG=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/svar_$v.log 2>&1
  echo "svariant $v rc=$?: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/svar_$v.log').read().strip().splitlines()[-1]); print(d['stage_ms'].get('sample_mt_segments'))" 2>&1)"
done
