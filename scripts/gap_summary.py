"""Writer-queue gaps over the last 5 steps of a rocprofv3 kernel_trace.csv, by size class.  usage: python scripts/gap_summary.py CSV"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ws = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows if 'k_emit_tiles' in r['Kernel_Name'])
g = [(ws[i+1][0] - ws[i][1]) / 1e6 for i in range(len(ws) - 1)]
# last 500 writers (5 steps)
g = g[-500:]
span = (ws[-1][1] - ws[-501][0]) / 1e6
big = [x for x in g if x > 8]
mid = [x for x in g if 0.3 < x <= 8]
small = [x for x in g if x <= 0.3]
print('span %.1f ms over 5 steps; busy %.1f' % (span, span - sum(g)))
print('gaps >8 ms: n=%d sum=%.1f; 0.3-8 ms: n=%d sum=%.1f; <=0.3: n=%d sum=%.1f' % (len(big), sum(big), len(mid), sum(mid), len(small), sum(small)))
print(sorted(mid)[-30:])
