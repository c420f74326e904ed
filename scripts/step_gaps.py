"""Writer-queue idle per step (steady state) from a rocprofv3 kernel_trace.csv: the gaps between writers over the
last N steps (a step starts at its first k_resolve after a writer gap), each gap with the main-queue kernels inside.
python scripts/step_gaps.py CSV [writer_name] [steps] [ms_per_step]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
wname = sys.argv[2] if len(sys.argv) > 2 else 'k_emit_tiles'
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 4


def short(n):
  n = n.replace('mh::(anonymous namespace)::', '').replace('mh::', '').replace('void ', '')
  return re.sub(r'[(<].*', '', n)[:28]


ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']), short(r['Kernel_Name']))
            for r in rows)
ws = [e for e in ev if wname in e[3]]
wq = collections.Counter(e[2] for e in ws).most_common(1)[0][0]
# the last N steps: step k starts at the drop of its first haplotype, the first k_resolve after the previous step's
# last writer was queued... approximated by the N + 1 latest k_resolve clusters (a cluster: k_resolve launches with
# gaps below 30 ms; the batches of one step are ~30 ms apart, the clusters of consecutive steps' first batches
# include the step boundary's idle)
res = [e[0] for e in ev if e[3] == 'k_resolve']
period = float(sys.argv[4]) * 1e6 if len(sys.argv) > 4 else None
t1 = ws[-1][1]
t0 = t1 - nsteps * period if period else res[0]
busy = sorted((s, e) for s, e, q, _ in ev if q == wq and e > t0 and s < t1)
gaps, cur = [], t0
for s, e in busy:
  if s > cur:
    gaps.append((cur, s))
  cur = max(cur, e)
if cur < t1:
  gaps.append((cur, t1))
span = (t1 - t0) / 1e6
idle = sum(b - a for a, b in gaps) / 1e6
print('%d steps, %.2f ms per step; writer idle %.2f ms per step (%.1f %%), %d gaps' %
      (nsteps, span / nsteps, idle / nsteps, 100 * idle / span, len(gaps)))
for a, b in gaps:
  if b - a < 0.3e6:
    continue
  names = collections.Counter()
  for s, e, q, n in ev:
    if q != wq and min(e, b) > max(s, a):
      names['q%d %s' % (q, n)] += (min(e, b) - max(s, a)) / 1e6
  print('  %8.2f +%6.2f ms: %s' % ((a - t0) / 1e6, (b - a) / 1e6,
                                  ', '.join('%s %.2f' % x for x in names.most_common(5))))
