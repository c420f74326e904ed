"""Deterministic synthetic inputs shaped like the reference's benchmark configs.

* Reference: GRCh37 contig names/lengths, i.i.d. uppercase ACGT, 10 kbp 'N' telomere caps plus one centromere
  'N' block per contig (~7.5 % N overall on the large contigs).
* Variants (one sample, phased diploid): ~1.3 per kbp; 80 % SNV, 10 % INS, 10 % DEL; indel length 1+geometric(0.3)
  capped at 50; 0.1 % long insertions (200-600 bp, exercise '>p:nI'); GT 0|1 / 1|0 / 1|1 = 0.4 / 0.4 / 0.2; a
  seeded 0.1 % of deliberate overlaps (exercise the accept chain).
Everything is produced directly as the structure-of-arrays form the engine consumes; `write_fasta` / `write_vcf`
emit files for the CLI.
"""
import gzip

import numpy as np

GRCH37 = [('1', 249250621), ('2', 243199373), ('3', 198022430), ('4', 191154276), ('5', 180915260),
          ('6', 171115067), ('7', 159138663), ('8', 146364022), ('9', 141213431), ('10', 135534747),
          ('11', 135006516), ('12', 133851895), ('13', 115169878), ('14', 107349540), ('15', 102531392),
          ('16', 90354753), ('17', 81195210), ('18', 78077248), ('19', 59128983), ('20', 63025520),
          ('21', 48129895), ('22', 51304566), ('X', 155270560), ('Y', 59373566), ('MT', 16569)]

_ACGT = np.frombuffer(b'ACGT', dtype=np.uint8)


def spawn_map(fn, jobs, workers, chunksize=1):
  """pool.map over fresh (spawned) interpreters, the pool closed and joined afterwards.  (`with Pool()` terminates
  its workers with SIGTERM on exit, which a profiler's signal handler in each idle worker reports as an abort.)"""
  import multiprocessing as mp
  pool = mp.get_context('spawn').Pool(max(1, workers))
  try:
    out = pool.map(fn, jobs, chunksize=chunksize)
  except BaseException:
    pool.terminate()
    raise
  pool.close()
  pool.join()
  return out


def contig(length, seed, n_gaps=True):
  rs = np.random.RandomState(seed)
  s = _ACGT[rs.randint(0, 4, size=length, dtype=np.uint8)]
  if n_gaps and length > 100000:
    cap = 10000
    s[:cap] = ord('N')
    s[-cap:] = ord('N')
    c0 = int(length * 0.45)
    s[c0:c0 + int(length * 0.055)] = ord('N')
  return s.tobytes()


def variants(seq, seed, rate=1.3e-3, start0=0, end=None):
  """Records for one contig: dict of arrays pos (1-based), ref_len, alt (list of bytes), gt (n, 2) int8."""
  end = len(seq) if end is None else end
  rs = np.random.RandomState(seed)
  arr = np.frombuffer(seq, dtype=np.uint8)
  span = end - start0
  n = rs.binomial(span, rate)
  pos0 = np.unique(rs.randint(start0 + 1, end - 60, size=n))
  pos0 = pos0[arr[pos0] != ord('N')]
  # keep variants apart so only the deliberate overlaps interact
  keep = np.ones(len(pos0), bool)
  keep[1:] = np.diff(pos0) > 60
  pos0 = pos0[keep]
  n = len(pos0)
  kind = rs.choice(3, size=n, p=[0.8, 0.1, 0.1])      # 0 SNV, 1 INS, 2 DEL
  ilen = np.minimum(1 + rs.geometric(0.3, size=n), 50)
  long_ins = rs.rand(n) < 0.001
  kind[long_ins] = 1
  ilen[long_ins] = rs.randint(200, 601, size=long_ins.sum())
  overlap = rs.rand(n) < 0.001                        # move next to its predecessor's span
  for i in np.nonzero(overlap)[0]:
    if i > 0:
      pos0[i] = pos0[i - 1] + rs.randint(0, 3)
  order = np.argsort(pos0, kind='stable')
  pos0, kind, ilen = pos0[order], kind[order], ilen[order]
  gt_pick = rs.choice(3, size=n, p=[0.4, 0.4, 0.2])
  gt = np.array([[0, 1], [1, 0], [1, 1]], dtype=np.int8)[gt_pick]
  ref_len = np.where(kind == 2, ilen + 1, 1).astype(np.int64)
  ref_len = np.minimum(ref_len, len(seq) - pos0)
  rand_bases = _ACGT[rs.randint(0, 4, size=int(ilen.sum()) + n)]
  lut = np.zeros(256, dtype=np.int64)
  lut[_ACGT] = np.arange(4)
  snv = _ACGT[(lut[arr[pos0]] + 1 + np.arange(n) % 3) % 4]
  alts, off = [], 0
  for i in range(n):
    b = seq[pos0[i]:pos0[i] + 1]
    if kind[i] == 0:
      a = bytes([snv[i]])
    elif kind[i] == 1:
      a = b + rand_bases[off:off + ilen[i]].tobytes()
      off += ilen[i]
    else:
      a = b
    alts.append(a)
  return {'pos': pos0.astype(np.int64) + 1, 'ref_len': ref_len, 'alt': alts, 'gt': gt}


def copies_soa(recs, start0=0, end=None):
  """vcfio-equivalent split into per-copy SoA for a region [start0, end) (htslib overlap semantics)."""
  pos, rl = recs['pos'], recs['ref_len']
  end = np.iinfo(np.int64).max if end is None else end
  sel = np.nonzero((pos - 1 < end) & (pos - 1 + rl > start0))[0]
  out = []
  for cpy in range(2):
    idx = sel[recs['gt'][sel, cpy] != 0]
    alts = [recs['alt'][i] for i in idx]
    al = np.array([len(a) for a in alts], dtype=np.int64)
    r = rl[idx]
    op = np.where(r == 1, np.where(al == 1, ord('X'), ord('I')), ord('D')).astype(np.uint8)
    oplen = np.where(op == ord('X'), 0, np.where(op == ord('I'), al - 1, r - 1)).astype(np.int64)
    ao = np.zeros(len(idx), dtype=np.int64)
    if len(idx):
      ao[1:] = np.cumsum(al)[:-1]
    out.append({'pos': pos[idx].copy(), 'op': op, 'oplen': oplen, 'alt_off': ao, 'alt_len': al,
                'alt_pool': b''.join(alts)})
  return out


def genome_contigs(scale=1.0, min_len=20000):
  """GRCh37's contigs, lengths scaled by `scale` (rehearsals on small genomes; 1 = the real lengths)."""
  if scale == 1.0:
    return list(GRCH37)
  return [(n, max(min_len, int(L * scale))) for n, L in GRCH37]


def _region_job(args):
  length, cseed, vseed = args
  seq = contig(length, cseed)
  recs = variants(seq, vseed)
  return seq, recs, copies_soa(recs)


def genome_regions(contigs, indices, workers=8):
  """Synthetic inputs of the whole-genome workload for the regions `indices` of `contigs`: region ri gets contig seed
  1000 + ri and variant seed 2000 + ri.  Returns {ri: (seq, records, per-copy SoA)}.  Built in `workers` spawned
  processes (fresh interpreters: safe whether or not the caller has touched the GPU)."""
  jobs = [(contigs[ri][1], 1000 + ri, 2000 + ri) for ri in indices]
  if workers <= 1 or len(jobs) <= 1:
    res = [_region_job(j) for j in jobs]
  else:
    order = sorted(range(len(jobs)), key=lambda k: -jobs[k][0])   # longest first
    got = spawn_map(_region_job, [jobs[k] for k in order], min(workers, len(jobs)))
    res = [None] * len(jobs)
    for k, r in zip(order, got):
      res[k] = r
  return dict(zip(indices, res))


def write_fasta(path, contigs, width=60):
  with open(path, 'wb') as fp:
    for name, s in contigs:
      fp.write(b'>' + name.encode() + b'\n')
      for i in range(0, len(s), width):
        fp.write(s[i:i + width] + b'\n')


def write_vcf(path, contigs, recs_by_contig, sample='SYN'):
  op = gzip.open if path.endswith('.gz') else open
  with op(path, 'wb') as fp:
    fp.write(b'##fileformat=VCFv4.1\n')
    for name, s in contigs:
      fp.write('##contig=<ID={},length={}>\n'.format(name, len(s)).encode())
    fp.write(b'##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n')
    fp.write('#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t{}\n'.format(sample).encode())
    seqd = dict(contigs)
    for name, _ in contigs:
      recs = recs_by_contig.get(name)
      if recs is None:
        continue
      s = seqd[name]
      for i in range(len(recs['pos'])):
        p = int(recs['pos'][i])
        ref = s[p - 1:p - 1 + int(recs['ref_len'][i])]
        gt = '{}|{}'.format(*recs['gt'][i])
        fp.write(b'%s\t%d\t.\t%s\t%s\t50\tPASS\t.\tGT\t%s\n' % (name.encode(), p, ref, recs['alt'][i], gt.encode()))
