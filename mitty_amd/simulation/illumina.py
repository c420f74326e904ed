"""The 'illumina' read-model plugin (reference mitty/simulation/illumina.py), backed by the GPU.

Same function names, arguments and return types as the reference module; `generate_reads` runs the MT19937-exact
sampling kernels (mh_sample_templates_span) and returns the reference's arrays; `corrupt_template` /
`corrupt_single_read` run the exact-stream corruption kernels (mh_corrupt.hip) on the caller's RandomState, which
is left exactly where the reference leaves it.
"""
import threading

import numpy as np

from mitty_amd import _native

SEED_MAX = (1 << 32) - 1

base_rot = {'A': 'CTG', 'C': 'ATG', 'T': 'ACG', 'G': 'ACT'}
phred_p = 10 ** (-np.arange(100) / 10)   # illumina.py:162, computed as the reference does

_ctx = None
_ctx_lock = threading.Lock()


def device_context():
  """Module-level device context used by the plugin-level API (created on first use, device 0)."""
  global _ctx
  with _ctx_lock:
    if _ctx is None:
      _ctx = _native.Context(0)
    return _ctx


def read_model_params(model, diploid_coverage=30.0):
  """illumina.read_model_params (illumina.py:12-40)."""
  p, passes = _native.read_model_params(model['mean_rlen'], diploid_coverage)
  return {'diploid_coverage': diploid_coverage, 'p': p, 'passes': passes, 'rlen': model['mean_rlen'],
          'cum_tlen': model['cum_tlen'], 'cum_bq_mat': model['cum_bq_mat']}


def generate_reads(model, p_min, p_max, seed=7, rng='mitty'):
  """illumina.generate_reads (illumina.py:43-58): template arrays for one (region, copy, pass).

  Returns [{'file_order': int8[m], 'pos': int64[m], 'len': uint32[m]}, {...mate 1...}].
  """
  if not (0 <= seed <= SEED_MAX):
    raise ValueError('Seed value {} is out of range 0 - {}'.format(seed, SEED_MAX))
  ctx = device_context()
  mode = _native.MH_RNG_MITTY if rng == 'mitty' else _native.MH_RNG_PHILOX
  ctx.sample_templates_span(p_min, p_max, model['p'], model['rlen'], model['cum_tlen'], seed, mode)
  fo0, pos0, pos1 = ctx.get_templates()
  rlen = model['rlen']
  return [{'file_order': fo0, 'pos': pos0, 'len': np.full(fo0.size, rlen, dtype=np.uint32)},
          {'file_order': (1 - fo0).astype(np.int8), 'pos': pos1, 'len': np.full(fo0.size, rlen, dtype=np.uint32)}]


_cx_tables = None   # the BQ tables last uploaded to the module context (kept referenced: identity is the cache key)


def _corrupt_exact(seqs, tables, corrupt_rng):
  """Reads `seqs` (one per mate, in order) corrupted with tables[i] = the mate's cum BQ matrix [max_bp, n_bq], their
  uniforms drawn from corrupt_rng's MT19937 stream as illumina.py:151-153 draws them.  Returns [(seq, bq_str)]."""
  global _cx_tables
  for sq, tb in zip(seqs, tables):
    if len(sq) > np.shape(tb)[0]:   # bq_mat[n, :] past the table (illumina.py:156)
      raise IndexError('index {} is out of bounds for axis 0 with size {}'.format(np.shape(tb)[0], np.shape(tb)[0]))
  ctx = device_context()
  pair = list(tables) + [tables[0]] * (2 - len(tables))
  if _cx_tables is None or any(a is not b for a, b in zip(_cx_tables, pair)):
    ctx.set_corruption(True, np.stack([np.asarray(t, dtype=np.float64) for t in pair]), phred_p, 0)
    _cx_tables = pair
  st = corrupt_rng.get_state()
  if st[0] != 'MT19937':
    raise TypeError('corrupt_rng must be a numpy RandomState (MT19937)')
  ctx.set_corruption_stream(_native.MH_RNG_MITTY, key=st[1], pos=int(st[2]))
  recs = [b'@r\n' + sq.encode('ascii') + b'\n+\n' + b'~' * len(sq) + b'\n' for sq in seqs]
  ctx.reset_output()
  try:
    ctx.corrupt_fastq(recs[0], recs[1] if len(recs) > 1 else None, 0)
    out = ctx.fetch_output()
  finally:
    ctx.reset_output()
  key, pos, _ = ctx.get_corruption_stream()
  corrupt_rng.set_state(('MT19937', key, pos, st[3], st[4]))
  res = []
  for k in range(len(seqs)):
    lines = out[k].split(b'\n')
    res.append((lines[1].decode('ascii'), lines[3].decode('ascii')))
  return res


def corrupt_template(model, template, corrupt_rng):
  """illumina.corrupt_template (illumina.py:113-128): [qname, seq, seq] -> [(qname, seq, bq), (qname, seq, bq)]."""
  bq_mat = model['cum_bq_mat']
  seqs = list(template[1:3])
  out = _corrupt_exact(seqs, [bq_mat[mate, :, :] for mate in range(len(seqs))], corrupt_rng)
  return [(template[0],) + o for o in out]


def corrupt_single_read(seq, bq_mat, corrupt_rng):
  """illumina.corrupt_single_read (illumina.py:140-162): (corrupted seq, BQ string)."""
  return _corrupt_exact([seq], [bq_mat], corrupt_rng)[0]
