"""Minimal stand-in for the pysam API surface the reference's generate/corrupt paths touch.

Used ONLY by tests/golden/make_golden.py in the build container to run the reference (pure Python) and capture
golden vectors.  It is not product code and never travels as part of the GPU path.

Semantics restated from htslib as the reference relies on them:
* VariantFile.fetch(contig, start, stop): records on `contig` with pos-1 < stop and pos-1+len(REF) > start, in
  file order.
* record.samples[0]['GT'] is a tuple of ints (None for '.'); record.samples[0].alleles maps each GT entry to its
  allele string ((REF,)+ALTS indexed by the GT value).
"""
import gzip


def _open_text(fname):
  with open(fname, 'rb') as fp:
    magic = fp.read(2)
  if magic == b'\x1f\x8b':
    return gzip.open(fname, 'rt')
  return open(fname, 'r')


class FastaFile:
  def __init__(self, fname):
    self.seqs = {}
    name, chunks = None, []
    with _open_text(fname) as fp:
      for line in fp:
        line = line.rstrip('\n').rstrip('\r')
        if line.startswith('>'):
          if name is not None:
            self.seqs[name] = ''.join(chunks)
          name, chunks = line[1:].split()[0], []
        else:
          chunks.append(line)
    if name is not None:
      self.seqs[name] = ''.join(chunks)

  def fetch(self, reference=None, start=None, end=None):
    s = self.seqs[reference]
    return s[(start or 0):(len(s) if end is None else end)]


class _Sample:
  def __init__(self, gt, alleles):
    self._gt, self.alleles = gt, alleles

  def __getitem__(self, k):
    if k != 'GT':
      raise KeyError(k)
    return self._gt


class _Samples(list):
  def values(self):
    return list(self)


class _Record:
  __slots__ = ('contig', 'pos', 'ref', 'alts', 'rlen', 'samples')


class VariantFile:
  def __init__(self, fname, mode='r', header=None):
    self.records, self.sample_names, self._col = [], [], None
    with _open_text(fname) as fp:
      for line in fp:
        if line.startswith('##'):
          continue
        f = line.rstrip('\n').split('\t')
        if line.startswith('#CHROM'):
          self.sample_names = f[9:]
          continue
        self.records.append(f)

  def subset_samples(self, samples):
    self._col = 9 + self.sample_names.index(samples[0])

  def _make(self, f):
    r = _Record()
    r.contig, r.pos, r.ref = f[0], int(f[1]), f[3]
    r.alts = tuple(f[4].split(',')) if f[4] != '.' else None
    r.rlen = len(r.ref)
    col = self._col if self._col is not None else 9
    fmt = f[8].split(':')
    gt_txt = f[col].split(':')[fmt.index('GT')]
    gt = tuple(None if g == '.' else int(g) for g in gt_txt.replace('/', '|').split('|'))
    al = (r.ref,) + (r.alts or ())
    alleles = tuple(None if g is None else al[g] for g in gt)
    r.samples = _Samples([_Sample(gt, alleles)])
    return r

  def fetch(self, contig=None, start=None, stop=None):
    for f in self.records:
      if f[0] != contig:
        continue
      beg = int(f[1]) - 1
      end = beg + len(f[3])
      if beg < stop and end > start:
        yield self._make(f)


class _FastxRecord:
  __slots__ = ('name', 'sequence', 'quality', 'comment')


class FastxFile:
  def __init__(self, fname):
    self.fname = fname

  def __iter__(self):
    with _open_text(self.fname) as fp:
      while True:
        h = fp.readline()
        if not h:
          return
        s = fp.readline().rstrip('\n')
        fp.readline()
        q = fp.readline().rstrip('\n')
        r = _FastxRecord()
        parts = h[1:].rstrip('\n').split(None, 1)
        r.name = parts[0]
        r.comment = parts[1] if len(parts) > 1 else None
        r.sequence, r.quality = s, q
        yield r
