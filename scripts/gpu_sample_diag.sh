# Sampler experiments: MT segment length (MH_SEG_TWISTS), k_mt_segments parts (MH_MT_DBG), decode pass trace.
mkdir -p gpurun_out
stage() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['stage_ms']; print(d['ms_per_step'], s.get('sample_mt_segments'), s.get('sample_shuffle_decode'))" 2>&1; }
for s in ${SEGS:-80 160 320 640}; do
  MH_SEG_TWISTS=$s timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/seg_$s.log 2>&1 || exit 1
  echo "seg $s: $(stage gpurun_out/seg_$s.log)"
done
for v in ${VARIANTS:-1}; do
  MH_MT_DBG=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/svar_$v.log 2>&1 || exit 1
  echo "svariant $v: $(stage gpurun_out/svar_$v.log)"
done
MH_DEC_VERBOSE=1 MH_DEC_BATCH=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dec_trace.log 2>&1 || exit 1
grep decode: gpurun_out/dec_trace.log | head -40
