"""Host-side waits from a rocprofv3 --hip-trace CSV: the HIP API calls longer than a threshold (synchronisations,
pageable copies, allocations), summed by function, and the longest ones with their time relative to the first
k_emit_tiles dispatch (so they can be lined up with scripts/wgs_gaps.py's writer gaps).
python scripts/host_waits.py HIP_API_TRACE_CSV KERNEL_TRACE_CSV [min_ms]"""
import collections
import csv
import sys

api = list(csv.DictReader(open(sys.argv[1])))
kt = list(csv.DictReader(open(sys.argv[2])))
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
t0 = min(int(r['Start_Timestamp']) for r in kt if 'k_emit_tiles' in r['Kernel_Name'])
tot, cnt = collections.Counter(), collections.Counter()
long_calls = []
for r in api:
  d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
  f = r.get('Function') or r.get('Operation') or r.get('Kind')
  tot[f] += d
  cnt[f] += 1
  if d >= thr:
    long_calls.append(((int(r['Start_Timestamp']) - t0) / 1e6, d, f, r.get('Thread_Id')))
print('HIP API time by function (ms, calls):')
for f, t in tot.most_common(15):
  print('  %9.3f %7d %s' % (t, cnt[f], f))
print('calls >= %.2f ms (start relative to the first writer, ms):' % thr)
for s, d, f, th in sorted(long_calls)[:400]:
  print('  %9.3f +%7.3f %s (thread %s)' % (s, d, f, th))
