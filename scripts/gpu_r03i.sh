#!/bin/bash
# Write/read pattern calibration for a position-ordered writer; WGS A/B of the unstaged seams (4 KB less LDS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/calib2
T=${TAG:-r03i}
timeout -k 10 120 ./scripts/calib_scatter > gpurun_out/calib_scatter_times.json || exit $?
cat gpurun_out/calib_scatter_times.json
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib2/f -o run -- ./scripts/calib_scatter > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib2/w -o run -- ./scripts/calib_scatter > /dev/null || exit $?
python3 - << 'PY'
import csv, glob, collections
for tag in ('f', 'w'):
  fs = glob.glob('gpurun_out/calib2/%s/**/*counter_collection.csv' % tag, recursive=True)
  if not fs:
    print(tag, 'no counter csv'); continue
  acc = collections.defaultdict(list)
  for r in csv.DictReader(open(fs[0])):
    acc[(r['Kernel_Name'][:40], r.get('Grid_Size', ''), r['Counter_Name'])].append(float(r['Counter_Value']))
  for k, v in acc.items():
    print(tag, k, ['%.3e' % x for x in v[-4:]])
PY
for d in 0 256; do
  MH_EW_DBG=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --batch-draws 64e6 > gpurun_out/bench_${T}_wgs_d$d.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}_wgs_d$d.json')); print('wgs d$d', round(d['value']/1e9,3), round(d['ms_per_step'],2), 'writer', round(d['roofline']['avg_launch_ms'],3))"
done
