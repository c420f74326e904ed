"""GPU diagnostics: run the golden end-to-end case and a 2 Mbp oracle unit under each emission / decode mode.
usage: python scripts/diag_modes.py CASE EMIT_MODE DECODE_MODE   (CASE: e2e | unit)"""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from mitty_amd import engine as E  # noqa: E402

case, emit_mode, dec_mode = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
_init = E.Engine.__init__


def _patched(self, *a, **k):
  _init(self, *a, **k)
  self.ctx.set_emit_mode(emit_mode)
  self.ctx.set_decode_mode(dec_mode)


E.Engine.__init__ = _patched


def first_diff(a, b):
  la, lb = a.split(b'\n'), b.split(b'\n')
  for i, (x, y) in enumerate(zip(la, lb)):
    if x != y:
      return 'line {}: got {!r} want {!r}'.format(i, x[:200], y[:200])
  return 'length {} vs {} lines'.format(len(la), len(lb))


t0 = time.time()
if case == 'e2e':
  from tests import golden_io as G
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  model = 'hiseq-X-v2.5-Garvan'
  c = G.load_json('e2e_config.json')[model]
  mod, mdl = get_read_model(model + '.pkl')
  d = tempfile.mkdtemp()
  f1, f2 = os.path.join(d, 'r1.fq'), os.path.join(d, 'r2.fq')
  readgenerate.process_multi_threaded(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], f1, f2, threads=2, seed=c['seed'])
  for f, g in ((f1, 'r1'), (f2, 'r2')):
    got, want = open(f, 'rb').read(), G.fastq_bytes('e2e_{}.{}.fq.gz'.format(model, g))
    print(case, emit_mode, dec_mode, g, 'OK' if got == want else 'DIFF ' + first_diff(got, want), flush=True)
else:
  from tests.test_gpu_parity import _unit_vs_oracle
  try:
    print(case, emit_mode, dec_mode, 'kept', _unit_vs_oracle(2_000_000, 7, 'hiseq-X-v2.5-Garvan', emit_mode=emit_mode))
  except AssertionError as e:
    print(case, emit_mode, dec_mode, 'FAIL', str(e)[:300])
print('elapsed {:.1f}s'.format(time.time() - t0), flush=True)
