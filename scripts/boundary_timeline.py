"""Kernels on every queue around a batch-boundary writer gap (1.5-4 ms) of a rocprofv3 kernel_trace.csv, 30 ms back.  usage: python scripts/boundary_timeline.py CSV"""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
  n = n.replace('mh::(anonymous namespace)::', '').replace('mh::', '').replace('void ', '')
  return re.sub(r'[(].*', '', n)[:30]
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Queue_Id']), short(r['Kernel_Name'])) for r in rows)
ws = [e for e in ev if 'k_emit_tiles' in e[3]]
gaps = [(ws[i][1], ws[i+1][0]) for i in range(len(ws)-1) if 1.5e6 < ws[i+1][0] - ws[i][1] < 4e6]
g0, g1 = gaps[-3]
print('gap %.3f ms' % ((g1-g0)/1e6))
lo = g0 - 30e6
for s, e, q, n in ev:
  if e > lo and s < g1 + 0.5e6 and (e - s) > 0.05e6:
    print('%8.3f %8.3f %6.3f q%d %s' % ((s-g0)/1e6, (e-g0)/1e6, (e-s)/1e6, q, n))
