# HBM bytes of every kernel over one bench step (FETCH_SIZE / WRITE_SIZE passes)
mkdir -p gpurun_out/pmct
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmct/$c -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/pmct/$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for c in ('FETCH_SIZE', 'WRITE_SIZE'):
  f = glob.glob('gpurun_out/pmct/%s/**/*counter_collection.csv' % c, recursive=True)[0]
  agg = collections.Counter()
  for r in csv.DictReader(open(f)):
    if r['Counter_Name'] == c:
      agg[r['Kernel_Name'][:50]] += float(r['Counter_Value']) * 1024 * (2 if c == 'FETCH_SIZE' else 1)
  tot = sum(agg.values())
  print(c, 'total GB (2 jobs):', round(tot / 1e9, 2))
  for k, v in agg.most_common(12):
    print('  %-50s %8.2f GB' % (k, v / 1e9))
PY
