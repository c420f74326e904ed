"""The 'illumina' read-model plugin (reference mitty/simulation/illumina.py), backed by the GPU.

Same function names, arguments and return types as the reference module; `generate_reads` runs the MT19937-exact
sampling kernels (mh_sample_templates_span) and returns the reference's arrays.
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
