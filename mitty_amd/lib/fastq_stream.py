"""Chunked FASTQ (pair) streaming into the device parsers (god-aligner BAM builder, corrupt-reads).

The host reads large chunks (gzip handled as pysam.FastxFile does); the device finds the record boundaries and
reports how many bytes of each buffer it consumed (whole templates only, the same number from both files); the
rest is carried into the next call.
"""
import gzip


def _reader(fname, chunk):
  with open(fname, 'rb') as fp:
    gz = fp.read(2) == b'\x1f\x8b'
  fp = gzip.open(fname, 'rb') if gz else open(fname, 'rb')
  try:
    while True:
      b = fp.read(chunk)
      if not b:
        return
      yield b
  finally:
    fp.close()


def stream_templates(fastq1, fastq2, consume, chunk=1 << 30, limit=None):
  """consume(buf1, buf2_or_None, max_templates, t_done) -> (used1, used2, templates).  Returns the templates done."""
  r1 = _reader(fastq1, chunk)
  r2 = _reader(fastq2, chunk) if fastq2 else None
  buf1, buf2 = b'', (b'' if fastq2 else None)
  eof1 = eof2 = False
  total, stalled = 0, False
  while True:
    if not eof1 and (len(buf1) < chunk or stalled):
      nxt = next(r1, None)
      eof1 = nxt is None
      buf1 += nxt or b''
    if r2 is not None and not eof2 and (len(buf2) < chunk or stalled):
      nxt = next(r2, None)
      eof2 = nxt is None
      buf2 += nxt or b''
    done = eof1 and (r2 is None or eof2)
    if done:   # a last record without its final newline
      if buf1 and not buf1.endswith(b'\n'):
        buf1 += b'\n'
      if buf2 and not buf2.endswith(b'\n'):
        buf2 += b'\n'
    want = -1 if limit is None else limit - total
    if want == 0:
      break
    u1, u2, t = consume(buf1, buf2, want, total)
    total += t
    stalled = t == 0
    buf1 = buf1[u1:]
    if buf2 is not None:
      buf2 = buf2[u2:]
    if done and t == 0:
      break
  return total


class FastqSink:
  """Sequential FASTQ output (works with FIFOs / process substitution, examples/reads/run.sh:13-16).  A name ending
  in '.gz' gets BGZF (gzip-compatible) output, deflated on a host thread pool."""

  def __init__(self, fname, level=6, threads=8, compress=None):
    self.fp = open(fname, 'wb')
    self.gz = fname.endswith('.gz') if compress is None else compress
    self.level, self.threads = level, threads
    self.raw = 0

  def write(self, data):
    self.raw += len(data)
    if self.gz:
      from mitty_amd import _native
      data = _native.bgzf_compress(data, self.level, self.threads)
    mv = memoryview(data)
    while len(mv):
      n = self.fp.write(mv)
      mv = mv[n:]

  def close(self):
    if self.fp is None:
      return
    if self.gz:
      from mitty_amd import _native
      self.fp.write(_native.bgzf_eof())
    self.fp.close()
    self.fp = None
