"""Steady-state step timeline from a rocprofv3 kernel_trace.csv: python scripts/timeline.py CSV [step_marker]
Per queue: busy time and the kernels of the last full step (between the last two k_splice-start markers)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else 'k_resolve'


def short(n):
  n = n.replace('mh::(anonymous namespace)::', '').replace('void ', '')
  n = re.sub(r'rocprim::ROCPRIM_\w+::detail::trampoline_kernel<.*?(onesweep_\w+|transform|block_sort)\w*.*', r'rocprim \1', n)
  return re.sub(r'\(.*', '', n)[:60]


ev = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']), short(r['Kernel_Name']))
             for r in rows), key=lambda x: x[0])
starts = [e[0] for e in ev if marker in e[3]]
# a step begins with the first copy's splice: take marker occurrences in pairs (2 copies per step)
if len(starts) < 6:
  print('not enough steps'); sys.exit()
t0, t1 = starts[-6], starts[-4]
sel = [e for e in ev if t0 <= e[0] < t1]
print('step window {:.3f} ms'.format((t1 - t0) / 1e6))
queues = sorted({e[2] for e in sel})
for q in queues:
  ks = [e for e in sel if e[2] == q]
  busy = sum(min(e[1], t1) - e[0] for e in ks)
  print('queue {}: {} kernels, busy {:.3f} ms'.format(q, len(ks), busy / 1e6))
agg = {}
for e in sel:
  agg.setdefault((e[2], e[3]), [0, 0])
  agg[(e[2], e[3])][0] += e[1] - e[0]
  agg[(e[2], e[3])][1] += 1
for (q, n), (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
  print('  q{} {:8.3f} ms {:4d}x  {}'.format(q, d / 1e6, c, n))
if len(sys.argv) > 3:
  for e in sel:
    print('{:9.3f} {:9.3f} q{} {}'.format((e[0] - t0) / 1e6, (e[1] - e[0]) / 1e6, e[2], e[3]))
