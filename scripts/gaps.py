"""Gaps and busy spans per queue over the last full step of a rocprofv3 kernel_trace.csv (step = between the last
two pairs of k_resolve launches, as scripts/timeline.py): python scripts/gaps.py CSV"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']),
              re.sub(r'\(.*', '', r['Kernel_Name'].replace('mh::(anonymous namespace)::', '').replace('void ', ''))[:40])
             for r in rows), key=lambda x: x[0])
starts = [e[0] for e in ev if 'k_resolve' in e[3]]
t0, t1 = starts[-6], starts[-4]
sel = [e for e in ev if t0 <= e[0] < t1]
print('step {:.3f} ms'.format((t1 - t0) / 1e6))
for q in sorted({e[2] for e in sel}):
  spans = []
  for s, e, _, n in sorted(x for x in sel if x[2] == q):
    if spans and s <= spans[-1][1] + 20000:   # merge gaps under 20 us
      spans[-1][1] = max(spans[-1][1], e)
      spans[-1][2].append(n)
    else:
      spans.append([s, e, [n]])
  print('queue', q)
  for s, e, names in spans:
    heavy = sorted(set(n for n in names if not n.startswith('__amd')))[:4]
    print('  {:7.3f} - {:7.3f}  ({:6.3f} ms) {} kernels: {}'.format((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6,
                                                                   len(names), ', '.join(heavy)))
