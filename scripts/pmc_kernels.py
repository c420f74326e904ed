"""Per-kernel averages of PMC counters from rocprofv3 counter_collection.csv files (dispatches of grid >= MIN only):
python scripts/pmc_kernels.py DIR [MIN_GRID]"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
mg = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 1000
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(d + '/p*/*counter_collection.csv')):
  per = collections.defaultdict(float)
  names = {}
  for r in csv.DictReader(open(p)):
    if int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0) < mg:
      continue
    k = re.sub(r'\(.*', '', r['Kernel_Name'].replace('mh::(anonymous namespace)::', '').replace('void ', ''))
    per[(k, r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
  for (k, _, c), v in per.items():
    acc[k][c].append(v)
for k in sorted(acc):
  print(k)
  for c in sorted(acc[k]):
    v = acc[k][c]
    print('   {:24s} {:16.1f}  ({} dispatches)'.format(c, sum(v) / len(v), len(v)))
