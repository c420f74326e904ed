"""Python driver for the CPU parity oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  It restates the
reference's orchestration (mitty/simulation/readgenerate.py:76-218, threads=1, worker 0) and VCF loading
(mitty/lib/vcfio.py:45-126 with htslib region-overlap semantics) in plain Python, and
calls the scalar C restatement in mitty_oracle.c for the per-unit work.
"""
import ctypes
import gzip
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'build', 'libmitty_oracle.so')

_lib = None

I64P = ctypes.POINTER(ctypes.c_int64)


def build():
  subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
  global _lib
  if _lib is None:
    if not os.path.exists(LIB_PATH):
      build()
    L = ctypes.CDLL(LIB_PATH)
    L.mo_mt_words.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int64]
    L.mo_read_model_params.argtypes = [ctypes.c_int64, ctypes.c_double, ctypes.POINTER(ctypes.c_double), I64P]
    L.mo_work_units.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.mo_work_units.restype = ctypes.c_int64
    L.mo_create_node_list.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 5 + \
                                     [ctypes.c_int64] + [ctypes.c_void_p] * 7
    L.mo_create_node_list.restype = ctypes.c_int64
    L.mo_template_capacity.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_double]
    L.mo_template_capacity.restype = ctypes.c_int64
    L.mo_generate_templates.argtypes = [ctypes.c_double, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.mo_generate_templates.restype = ctypes.c_int64
    L.mo_generate_unit.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 5 + \
                                  [ctypes.c_char_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int64, ctypes.c_void_p,
                                   ctypes.c_int64, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64,
                                   ctypes.POINTER(ctypes.c_void_p), I64P, ctypes.POINTER(ctypes.c_void_p), I64P]
    L.mo_generate_unit.restype = ctypes.c_int64
    L.mo_corrupt_fastq.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), I64P,
                                   ctypes.POINTER(ctypes.c_void_p), I64P]
    L.mo_corrupt_fastq.restype = ctypes.c_int64
    L.mo_free.argtypes = [ctypes.c_void_p]
    _lib = L
  return _lib


def _p(a):
  return a.ctypes.data_as(ctypes.c_void_p)


def _take(ptr, n):
  """n bytes at ptr (ctypes.string_at takes a C int size: it fails past 2 GiB)."""
  return bytes((ctypes.c_char * n).from_address(ptr.value)) if n else b''


# ---- RNG / small primitives ------------------------------------------------------------------------------------
def mt_words(seed, n):
  out = np.empty(n, dtype=np.uint32)
  lib().mo_mt_words(seed, _p(out), n)
  return out


def read_model_params(mean_rlen, coverage):
  p, passes = ctypes.c_double(), ctypes.c_int64()
  lib().mo_read_model_params(int(mean_rlen), float(coverage), ctypes.byref(p), ctypes.byref(passes))
  return p.value, passes.value


def work_units(seed, ploidy, passes):
  ploidy = np.asarray(ploidy, dtype=np.int32)
  n = int(ploidy.sum()) * passes
  r, c, s = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint32)
  lib().mo_work_units(seed, _p(ploidy), len(ploidy), passes, _p(r), _p(c), _p(s))
  return [(int(a), int(b), int(x)) for a, b, x in zip(r, c, s)]


def generate_templates(p, rlen, cum_tlen, p_min, p_max, seed):
  cum_tlen = np.ascontiguousarray(cum_tlen, dtype=np.float64)
  cap = lib().mo_template_capacity(p_min, p_max, p) + 1
  fo, p0, p1 = np.empty(cap, np.int8), np.empty(cap, np.int64), np.empty(cap, np.int64)
  m = lib().mo_generate_templates(p, rlen, _p(cum_tlen), len(cum_tlen), p_min, p_max, seed, _p(fo), _p(p0), _p(p1))
  if m < 0:
    raise ValueError('Seed value {} is out of range'.format(seed))
  return fo[:m], p0[:m], p1[:m]


# ---- inputs ----------------------------------------------------------------------------------------------------
def _open(fname):
  with open(fname, 'rb') as fp:
    gz = fp.read(2) == b'\x1f\x8b'
  return gzip.open(fname, 'rb') if gz else open(fname, 'rb')


def read_fasta(fname):
  seqs, name, chunks = {}, None, []
  with _open(fname) as fp:
    for line in fp:
      line = line.rstrip(b'\r\n')
      if line.startswith(b'>'):
        if name is not None:
          seqs[name] = b''.join(chunks)
        name, chunks = line[1:].split()[0].decode(), []
      else:
        chunks.append(line)
  if name is not None:
    seqs[name] = b''.join(chunks)
  return seqs


def read_bed(fname):
  with open(fname) as fp:
    return [(x[0], int(x[1]), int(x[2])) for x in (ln.split() for ln in fp.readlines())]


class Variant:
  __slots__ = ('pos', 'ref', 'alt', 'cigarop', 'oplen')

  def __init__(self, pos, ref, alt, cigarop, oplen):
    self.pos, self.ref, self.alt, self.cigarop, self.oplen = pos, ref, alt, cigarop, oplen

  def tuple(self):
    return self.pos, self.ref, self.alt, self.cigarop, self.oplen


def load_variant_file(fname, sample, bed_fname):
  """vcfio.load_variant_file + split_copies + parse (vcfio.py:51-126)."""
  recs, col = [], None
  with _open(fname) as fp:
    for line in fp:
      line = line.decode()
      if line.startswith('##'):
        continue
      f = line.rstrip('\n').split('\t')
      if line.startswith('#CHROM'):
        col = f.index(sample)
        continue
      recs.append((f[0], int(f[1]), f[3], f[4].split(','), f[col].split(':')[f[8].split(':').index('GT')]))
  out = []
  for region in read_bed(bed_fname):
    chrom, s0, e = region
    vl = [r for r in recs if r[0] == chrom and r[1] - 1 < e and r[1] - 1 + len(r[2]) > s0]
    ploidy = 2 if not vl else len(vl[0][4].replace('/', '|').split('|'))
    copies = []
    for cpy in range(ploidy):
      lst = []
      for _, pos, ref, alts, gt in vl:
        g = gt.replace('/', '|').split('|')[cpy]
        g = None if g == '.' else int(g)
        if g == 0:
          continue
        alt = ([ref] + alts)[g]
        lr, la = len(ref), len(alt)
        if lr == 1:
          op, ol = ('X', 0) if la == 1 else ('I', la - lr)
        elif la == 1:
          op, ol = 'D', lr - la
        else:
          raise ValueError('Complex variants present in VCF. Please filter or refactor these.')
        lst.append(Variant(pos, ref, alt, op, ol))
      copies.append(lst)
    out.append({'region': region, 'v': copies})
  return out


def _variant_soa(vl):
  pos = np.array([v.pos for v in vl], dtype=np.int64)
  op = ''.join(v.cigarop for v in vl).encode() or b'\0'
  oplen = np.array([v.oplen for v in vl], dtype=np.int64)
  alts = [v.alt.encode() for v in vl]
  alen = np.array([len(a) for a in alts], dtype=np.int64)
  aoff = np.zeros(len(vl), dtype=np.int64)
  if len(vl):
    aoff[1:] = np.cumsum(alen)[:-1]
  pool = b''.join(alts) or b'\0'
  return pos, np.frombuffer(op, dtype=np.uint8).copy(), oplen, aoff, alen, pool


def create_node_list(ref_seq, ref_start_pos, vl):
  pos, op, oplen, aoff, alen, pool = _variant_soa(vl)
  cap = 2 * len(vl) + 1
  ps, pr, ol, off, sl = (np.empty(cap, np.int64) for _ in range(5))
  nop, src = np.empty(cap, np.uint8), np.empty(cap, np.uint8)
  n = lib().mo_create_node_list(ref_seq, len(ref_seq), ref_start_pos, _p(pos), _p(op), _p(oplen), _p(aoff), _p(alen),
                                len(vl), _p(ps), _p(pr), _p(nop), _p(ol), _p(src), _p(off), _p(sl))
  nodes = []
  for k in range(n):
    base = pool if src[k] else ref_seq
    seq = base[off[k]:off[k] + sl[k]].decode()
    o = chr(nop[k])
    v = {'=': None, 'X': 0, 'I': int(ol[k]), 'D': -int(ol[k])}[o]
    nodes.append((int(ps[k]), int(pr[k]), o, int(ol[k]), seq, v))
  return nodes


def generate_unit(ref_seq, region_start0, vl, p, rlen, cum_tlen, rng_seed, serial_stub, chrom, cpy):
  pos, op, oplen, aoff, alen, pool = _variant_soa(vl)
  cum_tlen = np.ascontiguousarray(cum_tlen, dtype=np.float64)
  o1, o2 = ctypes.c_void_p(), ctypes.c_void_p()
  l1, l2 = ctypes.c_int64(), ctypes.c_int64()
  n = lib().mo_generate_unit(ref_seq, len(ref_seq), region_start0, _p(pos), _p(op), _p(oplen), _p(aoff), _p(alen),
                             pool, len(vl), p, rlen, _p(cum_tlen), len(cum_tlen), rng_seed, serial_stub.encode(),
                             chrom.encode(), cpy, ctypes.byref(o1), ctypes.byref(l1), ctypes.byref(o2),
                             ctypes.byref(l2))
  b1 = _take(o1, l1.value)
  b2 = _take(o2, l2.value)
  lib().mo_free(o1)
  lib().mo_free(o2)
  return n, b1, b2


def generate_unit_soa(ref_seq, region_start0, soa, p, rlen, cum_tlen, rng_seed, serial_stub, chrom, cpy,
                      keep_output=True, digest=False):
  """generate_unit for variants already in structure-of-arrays form (pos, op, oplen, alt_off, alt_len, alt_pool).
  keep_output=False frees the FASTQ bytes without copying them into Python (timing runs: no GIL-held copy);
  digest=True returns (n, len1, sha256 hex 1, len2, sha256 hex 2), hashed in place (no copy)."""
  import hashlib
  pos = np.ascontiguousarray(soa['pos'], dtype=np.int64)
  op = np.ascontiguousarray(soa['op'], dtype=np.uint8)
  oplen = np.ascontiguousarray(soa['oplen'], dtype=np.int64)
  aoff = np.ascontiguousarray(soa['alt_off'], dtype=np.int64)
  alen = np.ascontiguousarray(soa['alt_len'], dtype=np.int64)
  pool = soa['alt_pool'] or b'\0'
  if len(op) == 0:
    op = np.zeros(1, np.uint8)
  cum_tlen = np.ascontiguousarray(cum_tlen, dtype=np.float64)
  o1, o2 = ctypes.c_void_p(), ctypes.c_void_p()
  l1, l2 = ctypes.c_int64(), ctypes.c_int64()
  n = lib().mo_generate_unit(ref_seq, len(ref_seq), region_start0, _p(pos), _p(op), _p(oplen), _p(aoff), _p(alen),
                             pool, len(pos), p, rlen, _p(cum_tlen), len(cum_tlen), rng_seed, serial_stub.encode(),
                             chrom.encode(), cpy, ctypes.byref(o1), ctypes.byref(l1), ctypes.byref(o2),
                             ctypes.byref(l2))
  try:
    if digest:
      hs = []
      for o, ln in ((o1, l1.value), (o2, l2.value)):
        h = hashlib.sha256()
        if ln:
          h.update(memoryview((ctypes.c_char * ln).from_address(o.value)).cast('B'))
        hs.append(h.hexdigest())
      return n, l1.value, hs[0], l2.value, hs[1]
    b1 = _take(o1, l1.value) if keep_output else b''
    b2 = _take(o2, l2.value) if keep_output else b''
  finally:
    lib().mo_free(o1)
    lib().mo_free(o2)
  return n, b1, b2


def generate_reads_fastq(fasta, vcf, sample, bed, model, coverage, seed, max_units=None):
  """readgenerate.process_multi_threaded(..., threads=1): returns (r1_bytes, r2_bytes, n_templates)."""
  seqs = read_fasta(fasta) if isinstance(fasta, str) else fasta
  vdf = load_variant_file(vcf, sample, bed) if isinstance(vcf, str) else vcf
  p, passes = read_model_params(model['mean_rlen'], coverage)
  units = work_units(seed, [len(r['v']) for r in vdf], passes)
  out1, out2, total = [], [], 0
  for ps, (ri, cpy, s) in enumerate(units[:max_units] if max_units else units):
    chrom, s0, e = vdf[ri]['region']
    ref_seq = seqs[chrom][s0:e]
    n, b1, b2 = generate_unit(ref_seq, s0, vdf[ri]['v'][cpy], p, int(model['mean_rlen']), model['cum_tlen'], s,
                              '{}:{}:{}'.format(sample, 0, ps), chrom, cpy)
    out1.append(b1)
    out2.append(b2)
    total += n
  return b''.join(out1), b''.join(out2), total


PHRED_P = 10 ** (-np.arange(100) / 10)   # illumina.py:162 (computed exactly as the reference does)


def corrupt_fastq(model, names, seq1, seq2, seed=7):
  """readcorrupt.multi_process(processes=1): single MT stream over the file (readcorrupt.py:31-37, :84)."""
  n = len(names)
  keep = [ctypes.c_char_p(x.encode()) for x in names]
  k1 = [ctypes.c_char_p(x.encode()) for x in seq1]
  k2 = [ctypes.c_char_p(x.encode()) for x in seq2]
  a_names = (ctypes.c_char_p * n)(*keep)
  a1 = (ctypes.c_char_p * n)(*k1)
  a2 = (ctypes.c_char_p * n)(*k2)
  l1 = np.array([len(x) for x in seq1], np.int64)
  l2 = np.array([len(x) for x in seq2], np.int64)
  cum = np.ascontiguousarray(model['cum_bq_mat'], dtype=np.float64)
  ph = np.ascontiguousarray(PHRED_P)
  o1, o2 = ctypes.c_void_p(), ctypes.c_void_p()
  ol1, ol2 = ctypes.c_int64(), ctypes.c_int64()
  r = lib().mo_corrupt_fastq(seed, n, ctypes.cast(a_names, ctypes.c_void_p), ctypes.cast(a1, ctypes.c_void_p),
                             ctypes.cast(a2, ctypes.c_void_p), _p(l1), _p(l2), _p(cum), cum.shape[1], cum.shape[2],
                             _p(ph), ctypes.byref(o1), ctypes.byref(ol1), ctypes.byref(o2), ctypes.byref(ol2))
  if r < 0:
    raise ValueError('read longer than the BQ model')
  b1, b2 = _take(o1, ol1.value), _take(o2, ol2.value)
  lib().mo_free(o1)
  lib().mo_free(o2)
  return b1, b2


def _unit_digest(args):
  """One work unit in a worker process: (templates, len1, sha256 of file 1's bytes, len2, sha256 of file 2's).
  ref_seq may be (path, offset, length): the unit's reference bytes read from a file the caller wrote."""
  ref_seq, s0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy = args
  if isinstance(ref_seq, tuple):
    path, off, ln = ref_seq
    with open(path, 'rb') as fp:
      fp.seek(off)
      ref_seq = fp.read(ln)
  return generate_unit_soa(ref_seq, s0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy, digest=True)


def unit_digests(seqs, vdf, sample, model, coverage, seed, workers=8):
  """readgenerate.process_multi_threaded(..., threads=1) unit by unit: per unit in the reference's order (ps), the
  byte length and sha256 of its piece of each FASTQ file (the files are the pieces concatenated in ps order).  Units
  run in `workers` spawned processes.  Returns [(ps, region_idx, cpy, templates, len1, sha1, len2, sha2)]."""
  p, passes = read_model_params(model['mean_rlen'], coverage)
  units = work_units(seed, [len(r['v']) for r in vdf], passes)
  jobs = []
  for ps, (ri, cpy, s) in enumerate(units):
    chrom, s0, e = vdf[ri]['region']
    pos, op, oplen, aoff, alen, pool = _variant_soa(vdf[ri]['v'][cpy])
    soa = {'pos': pos, 'op': op, 'oplen': oplen, 'alt_off': aoff, 'alt_len': alen, 'alt_pool': pool}
    jobs.append((seqs[chrom][s0:e], s0, soa, p, int(model['mean_rlen']), model['cum_tlen'], s,
                 '{}:{}:{}'.format(sample, 0, ps), chrom, cpy))
  res = digest_jobs(jobs, workers)
  return [(ps, units[ps][0], units[ps][1]) + tuple(res[ps]) for ps in range(len(jobs))]


def _ref_len(ref):
  return ref[2] if isinstance(ref, tuple) else len(ref)


def digest_jobs(jobs, workers=8):
  """_unit_digest over jobs (ref_seq, s0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy) in `workers` spawned
  processes, longest region first; results in job order.  The pool is closed and joined (not terminated)."""
  import multiprocessing as mp
  order = sorted(range(len(jobs)), key=lambda k: -_ref_len(jobs[k][0]))   # longest first
  pool = mp.get_context('spawn').Pool(max(1, min(workers, len(jobs))))
  try:
    got = pool.map(_unit_digest, [jobs[k] for k in order], chunksize=1)
  except BaseException:
    pool.terminate()
    raise
  pool.close()
  pool.join()
  res = [None] * len(jobs)
  for k, r in zip(order, got):
    res[k] = r
  return res
