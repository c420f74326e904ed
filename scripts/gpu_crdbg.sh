mkdir -p gpurun_out
for d in 0 512 1024 1536 2; do
  MH_EMIT_DBG=$d timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e --steps 4 --warmup 1 > gpurun_out/crdbg_$d.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/crdbg_$d.log').read().strip().split('\n')[-1])
print('dbg $d', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step'],2), 'ms writer', round(d['roofline']['avg_launch_ms'],3))"
done
