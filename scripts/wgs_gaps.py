"""Writer-stream idle time from a rocprofv3 kernel_trace.csv: the queue that runs k_emit_tiles, its busy union
between its first and last writer, and what ran on the other queues while it idled (kernel time by name inside the
gaps).  python scripts/wgs_gaps.py CSV [writer_kernel]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
wname = sys.argv[2] if len(sys.argv) > 2 else 'k_emit_tiles'


def short(n):
  n = n.replace('mh::(anonymous namespace)::', '').replace('void ', '')
  n = re.sub(r'rocprim::ROCPRIM_\w+::detail::trampoline_kernel<.*?(onesweep_\w+|transform|block_sort|lookback\w*)\w*.*',
             r'rocprim \1', n)
  return re.sub(r'\(.*', '', n)[:40]


ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']), short(r['Kernel_Name']))
            for r in rows)
ws = [e for e in ev if wname in e[3]]
wq = collections.Counter(e[2] for e in ws).most_common(1)[0][0]
t0, t1 = ws[0][0], ws[-1][1]
busy = sorted((s, e) for s, e, q, _ in ev if q == wq and s >= t0 and e <= t1)
gaps, cur = [], t0
for s, e in busy:
  if s > cur:
    gaps.append((cur, s))
  cur = max(cur, e)
span = (t1 - t0) / 1e6
idle = sum(b - a for a, b in gaps) / 1e6
wt = sum(e - s for s, e, q, n in ws) / 1e6
print('writer queue %d: %d writers, %.3f ms writing, span %.3f ms, idle %.3f ms (%.1f %%)' %
      (wq, len(ws), wt, span, idle, 100 * idle / span))
inside = collections.Counter()
for s, e, q, n in ev:
  if q == wq:
    continue
  for a, b in gaps:
    lo, hi = max(s, a), min(e, b)
    if hi > lo:
      inside[n] += (hi - lo) / 1e6
print('other-queue kernel time inside the writer gaps (ms):')
for n, t in inside.most_common(25):
  print('  %8.3f %s' % (t, n))
big = sorted(gaps, key=lambda g: g[0] - g[1])[:15]
print('largest gaps:')
for a, b in sorted(big):
  names = collections.Counter()
  for s, e, q, n in ev:
    if q != wq and min(e, b) > max(s, a):
      names[n] += (min(e, b) - max(s, a)) / 1e6
  print('  %9.3f +%7.3f ms: %s' % ((a - t0) / 1e6, (b - a) / 1e6,
                                   ', '.join('%s %.2f' % x for x in names.most_common(4))))
tot = collections.Counter()
for s, e, q, n in ev:
  if s >= t0 and e <= t1:
    tot[n] += (e - s) / 1e6
print('kernel time in the span by name (ms):')
for n, t in tot.most_common(25):
  print('  %8.3f %s' % (t, n))
