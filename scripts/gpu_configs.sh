# The other BASELINE configs on one GPU: fused BQ corruption (configs[2]) and the 2x250 model (configs[4]'s model)
mkdir -p gpurun_out/configs
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --corrupt --no-cpu-baseline > gpurun_out/configs/corrupt.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model 1kg-pcr-free --no-cpu-baseline > gpurun_out/configs/pe250.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --coverage 60 --no-cpu-baseline > gpurun_out/configs/cov60.log 2>&1 || exit 1
for f in corrupt pe250 cov60; do
  python3 -c "import json;d=json.loads(open('gpurun_out/configs/$f.log').read().strip().splitlines()[-1]);print('$f',round(d['value']/1e6,1),'M/s',round(d['ms_per_step'],2),'ms',d['roofline']['kernel'],round(d['roofline']['avg_launch_ms'],3),round(d['roofline']['frac'],3))"
done
