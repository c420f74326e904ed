mkdir -p gpurun_out
for d in 0 2; do
  MH_CR_DBG=$d timeout -k 10 300 python -u bench.py --corrupt --no-cpu-baseline --no-e2e --steps 4 --warmup 1 --stages > gpurun_out/crdbg2_$d.log 2>&1 || exit $?
  python3 -c "
import json; L=open('gpurun_out/crdbg2_$d.log').read().strip().split('\n'); d=json.loads(L[-1]); st=json.loads(L[-2])
print('dbg $d', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step'],2), 'ms corrupt', st.get('emit_corrupt'), 'write', st.get('emit_write'))"
done
