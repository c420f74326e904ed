"""corrupt-reads over existing FASTQ (reference mitty/simulation/readcorrupt.py:18-118, CLI cli.py:144-157),
MI355X build.

The reference reads template after template (file 1's name + each file's sequence, readcorrupt.py:50-54), corrupts
them in `processes` workers seeded from RandomState(seed) (:31-37) with illumina.corrupt_template and writes
'@{name}\n{seq}\n+\n{bq}\n' per file (:112-114), in whatever order the workers finish.  Here the FASTQ goes to the
GPU in large chunks and every base is corrupted in parallel with the same model and the same arithmetic
(mh_corrupt.hip); output order = input order.  Word source:
  rng='mitty'  (default) the reference's single-worker stream, i.e. `processes=1`: worker 0's
               RandomState(RandomState(seed).randint(SEED_MAX)) consumed template by template — byte-identical to
               the reference's `--threads 1` output (with more workers the reference's own output depends on which
               worker dequeues which template, so `processes` only selects this one deterministic realisation)
  rng='philox' counter-based: one Philox4x32-10 draw per three bases, counted by (template, file, triple)
               (include/mitty_hip.h, mh_set_corruption), no sequential chain at all
"""
import logging
import time

import numpy as np

from mitty_amd import _native
from mitty_amd.lib.fastq_stream import FastqSink, stream_templates, write_pair

logger = logging.getLogger(__name__)

SEED_MAX = (1 << 32) - 1


def multi_process(read_module, read_model, fastq1_in, fastq1_out, fastq2_in=None, fastq2_out=None, processes=2,
                  seed=7, device=0, chunk_bytes=None, flush_bytes=1 << 30, rng='mitty'):
  """readcorrupt.multi_process; `processes` is accepted for compatibility.  Returns a stats dict."""
  if not (0 <= seed <= SEED_MAX):
    raise ValueError('Seed value {} is out of range 0 - {}'.format(seed, SEED_MAX))
  if rng not in ('mitty', 'philox'):
    raise ValueError('rng must be mitty or philox')
  if chunk_bytes is None:   # the exact stream keeps ~6.4 KB of MT words per template on the device
    chunk_bytes = (256 << 20) if rng == 'mitty' else (1 << 30)
  t0 = time.time()
  ctx = _native.Context(device)
  fps = [FastqSink(fastq1_out)] + ([FastqSink(fastq2_out)] if fastq2_in is not None and fastq2_out else [])
  try:
    ctx.set_corruption(True, read_model['cum_bq_mat'], 10 ** (-np.arange(100) / 10), seed)
    if rng == 'mitty':   # readcorrupt.py:31-37, 84: worker 0's seed is the first randint(SEED_MAX) of RandomState(seed)
      ctx.set_corruption_stream(_native.MH_RNG_MITTY, int(np.random.RandomState(seed).randint(SEED_MAX)))

    def consume(b1, b2, want, done):
      r = ctx.corrupt_fastq(b1, b2, done)
      u1, u2 = ctx.output_size()
      if u1 + u2 >= flush_bytes:
        flush()
      return r

    def flush():
      d1, d2 = ctx.fetch_output()
      write_pair(fps + [None] * (2 - len(fps)), [d1, d2])   # each file on its own thread (FIFO outputs)
      ctx.reset_output()

    n = stream_templates(fastq1_in, fastq2_in, consume, chunk_bytes)
    flush()
  finally:
    for fp in fps:
      fp.close()
    ctx.close()
  dt = time.time() - t0
  logger.debug('Processed {} templates in {:0.2f}s ({:0.2f} t/s)'.format(n, dt, n / max(dt, 1e-9)))
  return {'templates': n, 'seconds': dt}
