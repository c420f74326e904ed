"""One-line summary of a bench.py log's JSON line: step time, writer launch, frac, stages."""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1])
r = d['roofline']
print(sys.argv[2] if len(sys.argv) > 2 else '', 'value %.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'],
      'writer %.3f ms' % r['avg_launch_ms'], 'frac %.3f' % r['frac'], json.dumps(d.get('stage_ms')))
