# Writer-stream CU share experiments: MH_WRITER_CUS = eighths of the CUs the FASTQ writer stream may use.
mkdir -p gpurun_out
for v in ${VARIANTS:-8 6 5 4}; do
  MH_WRITER_CUS=$v timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/wcus_$v.log 2>&1 || exit 1
  echo "wcus $v: $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/wcus_$v.log | tr '\n' ' ')"
done
