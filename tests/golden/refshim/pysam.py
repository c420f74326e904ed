"""Minimal stand-in for the pysam API surface the reference's generate/corrupt paths touch.

Used ONLY by tests/golden/make_golden.py in the build container to run the reference (pure Python) and capture
golden vectors.  It is not product code and never travels as part of the GPU path.

Semantics restated from htslib as the reference relies on them:
* VariantFile.fetch(contig, start, stop): records on `contig` with pos-1 < stop and pos-1+len(REF) > start, in
  file order.
* record.samples[0]['GT'] is a tuple of ints (None for '.'); record.samples[0].alleles maps each GT entry to its
  allele string ((REF,)+ALTS indexed by the GT value).
* rlen = END - POS + 1 when INFO carries END=, else len(REF) (htslib).
* VariantFile(fname, 'w', header=...): a writer that records each written record as its first 9 columns plus the
  subset sample's column (what the retained-record fixture of filter-variants compares; htslib's own re-serialisation
  of header and fields is not reproduced).
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
  __slots__ = ('contig', 'pos', 'ref', 'alts', 'rlen', 'samples', 'raw')


class _Header:
  def __init__(self, lines, samples):
    self.lines, self.samples = lines, samples


class VariantFile:
  def __init__(self, fname, mode='r', header=None):
    self.records, self.sample_names, self._col, self._meta = [], [], None, []
    if mode.startswith('w'):
      self._out = open(fname, 'w')
      for line in header.lines:
        self._out.write(line + '\n')
      self._out.write('\t'.join(['#CHROM', 'POS', 'ID', 'REF', 'ALT', 'QUAL', 'FILTER', 'INFO', 'FORMAT'] +
                                 header.samples) + '\n')
      return
    self._out = None
    with _open_text(fname) as fp:
      for line in fp:
        if line.startswith('##'):
          self._meta.append(line.rstrip('\n'))
          continue
        f = line.rstrip('\n').split('\t')
        if line.startswith('#CHROM'):
          self.sample_names = f[9:]
          continue
        self.records.append(f)

  @property
  def header(self):
    return _Header(self._meta, [self.sample_names[self._col - 9]] if self._col is not None else self.sample_names)

  def write(self, rec):
    self._out.write('\t'.join(rec.raw) + '\n')
    self._out.flush()

  def subset_samples(self, samples):
    self._col = 9 + self.sample_names.index(samples[0])

  def _make(self, f):
    r = _Record()
    r.contig, r.pos, r.ref = f[0], int(f[1]), f[3]
    r.alts = tuple(f[4].split(',')) if f[4] != '.' else None
    r.rlen = len(r.ref)
    for kv in f[7].split(';'):
      if kv.startswith('END='):
        r.rlen = int(kv[4:]) - r.pos + 1
    col = self._col if self._col is not None else 9
    r.raw = f[:9] + [f[col]]
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
      r = self._make(f)
      beg = r.pos - 1
      if beg < stop and beg + r.rlen > start:
        yield r


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
