"""Open an input that may be gzip-compressed with ONE open() and no seek, so FIFOs and process substitution
(`<(...)`, examples/reads/run.sh:13-16) lose no bytes: the first two bytes are read to sniff the gzip magic and put
back in front of the stream (pysam.FastxFile / htslib hopen sniff the same way on the open handle)."""
import gzip
import io


class _Prefixed(io.RawIOBase):
  """`head` followed by the rest of `fp`."""

  def __init__(self, head, fp):
    self._head, self._fp = head, fp

  def readable(self):
    return True

  def readinto(self, b):
    if self._head:
      n = min(len(b), len(self._head))
      b[:n] = self._head[:n]
      self._head = self._head[n:]
      return n
    return self._fp.readinto(b)

  def close(self):
    if not self.closed:
      self._fp.close()
    super().close()


def open_input(fname):
  """A binary reader over `fname`, decompressed when it starts with the gzip magic."""
  fp = open(fname, 'rb')
  try:
    head = fp.read(2)   # a buffered read: blocks until two bytes or EOF, also on a pipe
  except BaseException:
    fp.close()
    raise
  stream = io.BufferedReader(_Prefixed(head, fp), 1 << 20)
  return gzip.GzipFile(fileobj=stream, mode='rb') if head == b'\x1f\x8b' else stream
