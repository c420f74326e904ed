"""FASTA access for read generation (replaces pysam.FastaFile.fetch, reference readgenerate.py:181,186)."""


def read_fasta(fname, names=None):
  """{contig name (first word of the header): bytes}.  If `names` is given, other contigs are skipped.  Parsed by the
  host C++ reader (mh_fasta.cpp)."""
  from mitty_amd import _native
  return _native.read_fasta(fname, names)


def read_fasta_py(fname, names=None):
  """The same in Python (kept for the host-reader test)."""
  from mitty_amd.lib.openfile import open_input
  seqs, name, chunks, keep = {}, None, [], True
  with open_input(fname) as fp:   # one open: FIFOs and process substitution lose no bytes
    for line in fp:
      if line.startswith(b'>'):
        if name is not None and keep:
          seqs[name] = b''.join(chunks)
        name = line[1:].split()[0].decode()
        chunks = []
        keep = names is None or name in names
      elif keep:
        chunks.append(line.rstrip(b'\r\n'))
  if name is not None and keep:
    seqs[name] = b''.join(chunks)
  return seqs


def fetch(seqs, reference, start, end):
  """pysam FastaFile.fetch semantics: clamp [start, end) to the contig."""
  s = seqs[reference]
  return s[max(0, start):max(0, min(end, len(s)))]
