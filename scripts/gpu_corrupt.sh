# Corruption path: parity tests touching corruption, then the fused-corruption bench and the LDS-image writer alone
mkdir -p gpurun_out/configs
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "corrupt or slices" --timeout 200 \
  --timeout-method thread > gpurun_out/configs/pytest_corrupt.log 2>&1 || { tail -n 30 gpurun_out/configs/pytest_corrupt.log; exit 1; }
tail -n 1 gpurun_out/configs/pytest_corrupt.log
for v in "--corrupt" "--emit-mode 1"; do
  timeout -k 10 300 python bench.py $v --no-cpu-baseline > gpurun_out/configs/o.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/configs/o.log').read().strip().splitlines()[-1]);print('$v',round(d['value']/1e6,1),'M/s',round(d['ms_per_step'],2),'ms',d['roofline']['kernel'],round(d['roofline']['avg_launch_ms'],3),round(d['roofline']['frac'],3))"
done
