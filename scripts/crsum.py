"""One-line summary of a `bench.py --corrupt` log: step time and the corruption pass's launch time."""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1])
print(sys.argv[2] if len(sys.argv) > 2 else '', 'value %.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'],
      'corrupt %.3f ms' % d['corrupt_pass']['avg_launch_ms'], 'writer %.3f ms' % d['roofline']['avg_launch_ms'])
