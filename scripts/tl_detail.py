"""Kernels of the last full step per queue from a rocprofv3 kernel_trace.csv (those over 0.1 ms, and the writers and
measure passes): python scripts/tl_detail.py CSV"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))


def short(n):
  n = n.replace('mh::(anonymous namespace)::', '').replace('void ', '')
  n = re.sub(r'rocprim::ROCPRIM_\w+::detail::trampoline_kernel<.*?(onesweep_\w+|transform|block_sort)\w*.*', r'rocprim \1', n)
  return re.sub(r'\(.*', '', n)[:40]


ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']), short(r['Kernel_Name'])) for r in rows)
st = [e[0] for e in ev if 'k_resolve' in e[3]]
t0, t1 = st[-6], st[-4]
print('step %.3f ms' % ((t1 - t0) / 1e6))
for q in sorted({e[2] for e in ev}):
  ks = [e for e in ev if e[2] == q and t0 <= e[0] < t1]
  print('queue', q)
  for e in ks:
    if e[1] - e[0] > 100000 or 'emit' in e[3] or 'mt_seg' in e[3]:
      print('  %7.3f-%7.3f %6.3f %s' % ((e[0] - t0) / 1e6, (e[1] - t0) / 1e6, (e[1] - e[0]) / 1e6, e[3]))
