"""Host-side timing of one pipelined chr1 job's calls (diagnostics for the asynchronous emission path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mitty_amd import _native, synth  # noqa: E402
from mitty_amd.engine import Engine  # noqa: E402
from mitty_amd.readmodel import get_read_model  # noqa: E402

_, model = get_read_model('hiseq-X-v2.5-Garvan.pkl')
rlen = 150
p, passes = _native.read_model_params(rlen, 30.0)
L = 249_250_621
seq = synth.contig(L, 1000)
copies = synth.copies_soa(synth.variants(seq, 2000))
units = _native.work_units(7, [2], passes)
eng = Engine(0)
eng.load_region(0, ('1', 0, L), seq)
for c in range(2):
  eng.upload_variants(0, c, copies[c])
T = {}
orig = {}


def wrap(obj, name):
  f = getattr(obj, name)

  def g(*a, **k):
    t = time.perf_counter()
    r = f(*a, **k)
    T[name] = T.get(name, 0.0) + time.perf_counter() - t
    return r
  setattr(obj, name, g)


for n in ('release_haplotype', 'reset_output', 'sample_units', 'emit_async', 'read_bound', 'use_templates'):
  wrap(eng.ctx, n)
wrap(eng, 'haplotype')
for it in range(6):
  T.clear()
  t0 = time.perf_counter()
  eng.drop_haplotypes()
  eng.ctx.reset_output()
  pend = eng.run_units([(ps, ri, cpy, s) for ps, (ri, cpy, s) in enumerate(units)], lambda r, c: copies[c], p, rlen,
                       model['cum_tlen'], 'SYN', 0, True, 'mitty', lazy=True)
  t1 = time.perf_counter()
  print('job {}: host {:.2f} ms'.format(it, (t1 - t0) * 1e3), {k: round(v * 1e3, 2) for k, v in T.items()}, flush=True)
eng.ctx.sync()
print(pend.resolve())
eng.close()
