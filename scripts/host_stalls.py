"""Host-side stalls of the WGS bench line: every mitty_amd._native.Context method and Engine method timed on the host
(perf_counter around the call); prints, per method, the calls and the time spent in calls over 0.5 ms, and the
longest calls with their step-relative time.  usage: python scripts/host_stalls.py [bench args...]"""
import collections
import functools
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mitty_amd import _native  # noqa: E402
from mitty_amd import engine as E  # noqa: E402



def main():
  LOG = []
  STACK = []


  def wrap(cls, name):
    f = getattr(cls, name)

    @functools.wraps(f)
    def g(*a, **k):
      t0 = time.perf_counter()
      STACK.append(name)
      try:
        return f(*a, **k)
      finally:
        STACK.pop()
        LOG.append(('/'.join(STACK + [cls.__name__ + '.' + name]), t0, time.perf_counter() - t0))
    setattr(cls, name, g)


  for cls in (_native.Context, E.Engine):
    for name, v in list(vars(cls).items()):
      if callable(v) and not name.startswith('__'):
        wrap(cls, name)

  import bench  # noqa: E402
  sys.argv = ['bench.py'] + sys.argv[1:]
  t_start = time.perf_counter()
  bench.main()
  tot = collections.defaultdict(lambda: [0, 0.0, 0.0])
  for n, t0, d in LOG:
    r = tot[n]
    r[0] += 1
    r[1] += d
    if d > 5e-4:
      r[2] += d
  print('method: calls, total s, s in calls > 0.5 ms', file=sys.stderr)
  for n, (c, s, big) in sorted(tot.items(), key=lambda kv: -kv[1][2])[:25]:
    print('  %-70s %6d %8.3f %8.3f' % (n[-70:], c, s, big), file=sys.stderr)
  print('longest calls below run_units:', file=sys.stderr)
  inner = [x for x in LOG if x[0].startswith('run_units/')]
  for n, t0, d in sorted(inner, key=lambda x: -x[2])[:30]:
    print('  %8.3f ms at %9.3f s  %s' % (d * 1e3, t0 - t_start, n[-90:]), file=sys.stderr)
  print('the last 3 steps, calls over 1 ms in time order (s from the first):', file=sys.stderr)
  t_last = [t0 for n, t0, d in LOG if n == 'Engine.drop_haplotypes'][-3]
  for n, t0, d in sorted(LOG, key=lambda x: x[1]):
    if t0 >= t_last and d > 1e-3 and n != 'Engine.run_units':
      print('  %9.3f  %8.3f ms  %s  [abs %.3f]' % ((t0 - t_last) * 1e3, d * 1e3, n[-80:], t0 * 1e3), file=sys.stderr)
  print('step starts (abs ms): ' + ' '.join('%.3f' % (t0 * 1e3) for n, t0, d in LOG if n == 'Engine.drop_haplotypes'),
        file=sys.stderr)


if __name__ == '__main__':
  main()
