"""Chunked FASTQ (pair) streaming into the device parsers (god-aligner BAM builder, corrupt-reads).

The host reads large chunks (gzip handled as pysam.FastxFile does); the device finds the record boundaries and
reports how many bytes of each buffer it consumed (whole templates only, the same number from both files); the
rest is carried into the next call.
"""
from mitty_amd.lib.openfile import open_input


class _Prefetch:
  """One input file read on its own thread into a queue of pieces (at most `max_bytes` not yet taken), so that a
  producer writing the two files of a pair (a FIFO or `<(...)` each, examples/reads/run.sh:13-16) never blocks on one
  pipe while we wait on the other: both pipes are drained as data arrives, whatever order the producer writes in
  (record by record like the reference's writer, readgenerate.py:233-253, or file by file in pieces up to
  `max_bytes`)."""

  def __init__(self, fname, piece, max_bytes):
    import collections
    import threading
    self._pieces = collections.deque()
    self._cv = threading.Condition()
    self._held = 0             # bytes read and not yet taken
    self._eof = False
    self._err = None
    self._stop = False         # close(): the reader thread closes the input and ends
    self._piece, self._max = piece, max_bytes
    self._t = threading.Thread(target=self._run, args=(fname,), daemon=True)
    self._t.start()

  def _run(self, fname):
    try:
      with open_input(fname) as fp:   # one open: FIFOs and process substitution lose no bytes
        read = getattr(fp, 'read1', fp.read)
        while True:
          with self._cv:
            while self._held >= self._max and not self._stop:
              self._cv.wait()
            if self._stop:
              break
          b = read(self._piece)   # what the pipe holds, or a whole piece of a file
          if not b:
            break
          with self._cv:
            if self._stop:
              break
            self._pieces.append(b)
            self._held += len(b)
            self._cv.notify_all()
    except BaseException as e:   # re-raised in the consumer
      self._err = e
    finally:
      with self._cv:
        self._eof = True
        self._cv.notify_all()

  def close(self):
    """Stop reading: the thread drops what it holds and closes the input (a FIFO producer then gets EPIPE instead of
    blocking on a reader that is gone).  A read already waiting on the pipe ends when the producer writes."""
    with self._cv:
      self._stop = True
      self._pieces.clear()
      self._held = 0
      self._cv.notify_all()

  def take(self, want):
    """Up to about `want` bytes: blocks until some are there, then takes what is queued.  b'' at end of file."""
    with self._cv:
      while not self._pieces and not self._eof:
        self._cv.wait()
      out, n = [], 0
      while self._pieces and n < want:
        b = self._pieces.popleft()
        out.append(b)
        n += len(b)
      self._held -= n
      self._cv.notify_all()
      if not out and self._err is not None:
        raise self._err
    return b''.join(out)


def _fill(r, buf, chunk, stalled):
  """buf topped up to `chunk` bytes (blocking until there or EOF), or by one more take when the consumer stalled."""
  parts, n = [buf], len(buf)
  while n < chunk or stalled:
    nxt = r.take(max(chunk - n, 1))
    if not nxt:
      return b''.join(parts), True
    parts.append(nxt)
    n += len(nxt)
    if stalled:
      break
  return b''.join(parts), False


def stream_templates(fastq1, fastq2, consume, chunk=1 << 30, limit=None, max_ahead=None):
  """consume(buf1, buf2_or_None, max_templates, t_done) -> (used1, used2, templates).  Returns the templates done.
  Each file is prefetched on its own thread, up to `max_ahead` bytes (default: 2 chunks, at least 1 GiB) beyond what
  the device has taken."""
  ahead = max_ahead or max(2 * chunk, 1 << 30)
  piece = min(chunk, 16 << 20)
  r1 = _Prefetch(fastq1, piece, ahead)
  r2 = _Prefetch(fastq2, piece, ahead) if fastq2 else None
  try:
    return _stream(r1, r2, consume, chunk, limit)
  finally:   # an early return (limit) or an error: the readers stop and close their inputs
    r1.close()
    if r2 is not None:
      r2.close()


def _stream(r1, r2, consume, chunk, limit):
  buf1, buf2 = b'', (b'' if r2 is not None else None)
  eof1 = eof2 = False
  total, stalled = 0, False
  while True:
    if not eof1:
      buf1, eof1 = _fill(r1, buf1, chunk, stalled)
    if r2 is not None and not eof2:
      buf2, eof2 = _fill(r2, buf2, chunk, stalled)
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


def write_pair(sinks, datas, raw_lens=None):
  """Write datas[f] to sinks[f] (None: skipped), each file on its own thread, so a reader that takes the two files in
  lockstep (pysam FastxFile pairs, `corrupt-reads` on FIFOs) never leaves us blocked on one pipe while it waits on
  the other."""
  raw_lens = raw_lens or [None] * len(sinks)
  jobs = [(s, d, r) for s, d, r in zip(sinks, datas, raw_lens) if s is not None]

  def put(s, d, r):   # r: BGZF bytes for r raw bytes (compressed on the GPU), else raw bytes
    if r is None:
      s.write(d)
    else:
      s.write_bgzf(d, r)
  if len(jobs) <= 1:
    for j in jobs:
      put(*j)
    return
  import threading
  errs = []

  def run(s, d, r):
    try:
      put(s, d, r)
    except BaseException as e:
      errs.append(e)
  ts = [threading.Thread(target=run, args=j) for j in jobs]
  for t in ts:
    t.start()
  for t in ts:
    t.join()
  if errs:
    raise errs[0]


class PairWriter:
  """Queued writes to the FASTQ sinks, one thread per file (a reader taking the two files in lockstep never leaves
  us blocked on one pipe while it waits on the other).  submit(slot, datas) returns at once; wait(slot) blocks until
  every write handed in with that staging slot is done, so its page-locked buffers can be refilled; close() drains.
  A write error is raised by the next wait() or close()."""

  def __init__(self, sinks):
    import queue
    import threading
    self.sinks = sinks
    self.q = [queue.Queue() if s is not None else None for s in sinks]
    self.errs = []
    self.pending = {}
    self.ts = [threading.Thread(target=self._run, args=(f,), daemon=True) for f in range(len(sinks))
               if sinks[f] is not None]
    for t in self.ts:
      t.start()

  def _run(self, f):
    while True:
      item = self.q[f].get()
      if item is None:
        return
      data, raw, ev = item
      try:
        if raw is None:
          self.sinks[f].write(data)
        else:
          self.sinks[f].write_bgzf(data, raw)
      except BaseException as e:   # (reported by the caller's next wait / close)
        self.errs.append(e)
      finally:
        ev.set()

  def submit(self, slot, datas, raw_lens=None):
    import threading
    raw_lens = raw_lens or [None] * len(datas)
    for f, (s, d, r) in enumerate(zip(self.sinks, datas, raw_lens)):
      if s is None or d is None:
        continue
      ev = threading.Event()
      self.pending.setdefault(slot, []).append(ev)
      self.q[f].put((d, r, ev))

  def wait(self, slot):
    for ev in self.pending.pop(slot, []):
      ev.wait()
    if self.errs:
      raise self.errs[0]

  def close(self):
    for q in self.q:
      if q is not None:
        q.put(None)
    for t in self.ts:
      t.join()
    self.pending.clear()
    if self.errs:
      raise self.errs[0]


class FastqSink:
  """Sequential FASTQ output (works with FIFOs / process substitution, examples/reads/run.sh:13-16).  A name ending
  in '.gz' gets BGZF (gzip-compatible) output, deflated on a host thread pool."""

  def __init__(self, fname, level=6, threads=8, compress=None):
    self.fp = open(fname, 'wb')
    self.gz = fname.endswith('.gz') if compress is None else compress
    self.level, self.threads = level, threads
    self.raw = 0       # bytes handed in
    self.written = 0   # bytes written (compressed when gz)

  def write(self, data):
    self.raw += len(data)
    if self.gz:
      from mitty_amd import _native
      data = _native.bgzf_compress(data, self.level, self.threads)
    self.written += len(data)
    mv = memoryview(data)
    while len(mv):
      n = self.fp.write(mv)
      mv = mv[n:]

  def write_bgzf(self, data, raw_len):
    """BGZF members compressed elsewhere (the GPU: mh_output_bgzf) for `raw_len` bytes of FASTQ."""
    assert self.gz, 'BGZF members into an uncompressed sink'
    self.raw += raw_len
    self.written += len(data)
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
