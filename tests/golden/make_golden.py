#!/usr/bin/env python3
"""Capture golden vectors from the reference (alenzhao/Mitty, pure Python) — build container only.

Run:  python tests/golden/make_golden.py        (needs /root/reference; writes tests/golden/*)

The reference is imported from /root/reference with the test-side pysam/nose stand-ins in
tests/golden/refshim (the reference's own 16 tests pass under them).  Read models are NOT unpickled: they are
decoded with mitty_amd.readmodel.parse_model_pickle and handed to the reference functions as dicts.

Outputs (data only — inputs and expected outputs):
  data/syn.fa, data/syn.vcf, data/syn.bed   synthetic edge-case genome (our own inputs)
  data/tiny*.{fasta,vcf,bed}                 the reference's own test fixtures (mitty/test/data)
  rng.json            raw MT19937 / legacy-distribution vectors (numpy RandomState, the reference's RNG)
  units.json          work-unit order from readgenerate.get_data_for_workers
  templates.npz       illumina.generate_reads arrays (3 seeds x 2 models, 200 kbp span)
  nodes.json          rpc.create_node_list for every (region, copy) of syn + tiny
  reads.json          rpc.generate_read for sampled (p, l) incl. edge cases
  e2e_<model>.r{1,2}.fq.gz  readgenerate.process_multi_threaded(threads=1) FASTQ pairs
  corrupt_<model>.r{1,2}.fq.gz + corrupt_in_*  readcorrupt.multi_process(processes=1, seed=7)
  qnames.json         parse_qname results
  god.json            god_aligner.write_perfect_reads record attributes (stub AlignedSegment)
"""
import gzip
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
DATA = os.path.join(HERE, 'data')

sys.path.insert(0, REPO)
from mitty_amd.readmodel import parse_model_pickle  # noqa: E402

MODELS = ['hiseq-X-v2.5-Garvan', '1kg-pcr-free']


def load_model(name):
  with open(os.path.join(REF, 'mitty/data/readmodels', name + '.pkl'), 'rb') as fp:
    return parse_model_pickle(fp.read())


# ----------------------------------------------------------------------------------------------------------------
# Synthetic edge-case genome (our own data)
# ----------------------------------------------------------------------------------------------------------------
def make_syn_inputs():
  rng = np.random.RandomState(20240607)
  ab = np.frombuffer(b'ACGT', dtype=np.uint8)

  def rand_seq(n):
    return bytearray(ab[rng.randint(0, 4, n)].tobytes())

  c1 = rand_seq(50000)
  c1[20000:20030] = b'N' * 30                     # N run -> templates dropped
  for q in (5000, 5003):                           # 2 isolated N's: kept (count <= 2)
    c1[q] = ord('N')
  for q in (7000, 7010, 7020):                     # 3 N's within 21 bp: dropped
    c1[q] = ord('N')
  c1[30000:30200] = c1[30000:30200].lower()        # lowercase passes through, not complemented
  for q, b in ((31000, 'R'), (31050, 'Y'), (31100, 'K')):
    c1[q] = ord(b)                                 # IUPAC passes through
  c2 = rand_seq(20000)
  c3 = rand_seq(8000)
  contigs = [('1', bytes(c1)), ('2', bytes(c2)), ('3', bytes(c3))]

  with open(os.path.join(DATA, 'syn.fa'), 'w') as fp:
    for name, s in contigs:
      fp.write('>{} synthetic\n'.format(name))
      for i in range(0, len(s), 60):
        fp.write(s[i:i + 60].decode() + '\n')

  seqd = dict(contigs)
  recs = []   # (chrom, pos1, ref, alts, gt_S1, gt_S0)

  def refb(ch, pos1, n=1):
    return seqd[ch][pos1 - 1:pos1 - 1 + n].decode().upper().replace('N', 'A')

  def other(b):
    return 'ACGT'[('ACGT'.index(b) + 1 + rng.randint(0, 3)) % 4] if b in 'ACGT' else 'A'

  def randalt(n):
    return ''.join('ACGT'[k] for k in rng.randint(0, 4, n))

  gts = ['0|1', '1|0', '1|1']
  # contig 1: dense mixed variants, plus hand-placed edge cases
  special = {
    998: ('del', 10, '0|1'),       # deletion starting before BED start 1000 (overlaps region; skipped)
    1001: ('snp', 0, '1|1'),       # SNP on the first base of the region (no leading '=')
    1500: ('ins', 3, '1|1'),
    12000: ('ins', 400, '0|1'),    # long insertion > rlen: '>p:nI' reads
    12800: ('ins', 260, '1|0'),
    15000: ('del', 5, '1|1'),      # DEL then overlapping SNP (skipped)
    15002: ('snp', 0, '1|1'),
    15010: ('snp', 0, '1|1'),      # SNP and INS at the same position: INS skipped
    15011: ('ins', 2, '1|1'),
    16000: ('multi', 0, '1|2'),    # multi-allelic SNP, different allele per copy
    17000: ('del', 40, '1/0'),     # unphased GT treated as phased order
    39995: ('del', 12, '1|1'),     # deletion crossing BED end 40000 (p_max beyond data)
  }
  pos = 1002
  rows = []
  while pos < 41000:
    if pos in special or any(pos <= s < pos + 60 for s in special):
      nxt = min(s for s in special if s >= pos)
      kind, ln, gt = special[nxt]
      rows.append((nxt, kind, ln, gt))
      pos = nxt + max(ln, 1) + 2
      continue
    kind = rng.choice(['snp'] * 8 + ['ins', 'del'])
    ln = 1 + min(rng.geometric(0.3), 10)
    rows.append((pos, kind, ln, gts[rng.randint(0, 3)]))
    pos += max(ln, 1) + 20 + rng.randint(0, 180)
  rows.sort(key=lambda r: r[0])
  for p1, kind, ln, gt in rows:
    r = refb('1', p1)
    if kind == 'snp':
      recs.append(('1', p1, r, [other(r)], gt, '0|0'))
    elif kind == 'multi':
      recs.append(('1', p1, r, [other(r), other(other(r))], gt, '0|1'))
    elif kind == 'ins':
      recs.append(('1', p1, r, [r + randalt(ln)], gt, '0|0'))
    else:
      recs.append(('1', p1, refb('1', p1, ln + 1), [r], gt, '1|1'))
  # contig 2: sparse variants, but none in [15000, 16000] (empty BED region -> diploid default)
  pos = 300
  while pos < 19800:
    if 14800 <= pos <= 16200:
      pos = 16300
    kind = rng.choice(['snp'] * 6 + ['ins', 'del'])
    ln = 1 + min(rng.geometric(0.4), 8)
    r = refb('2', pos)
    gt = gts[rng.randint(0, 3)]
    if kind == 'snp':
      recs.append(('2', pos, r, [other(r)], gt, '0|1'))
    elif kind == 'ins':
      recs.append(('2', pos, r, [r + randalt(ln)], gt, '0|1'))
    else:
      recs.append(('2', pos, refb('2', pos, ln + 1), [r], gt, '0|1'))
    pos += 100 + rng.randint(0, 400)
  # contig 3: haploid GTs
  pos = 150
  while pos < 7800:
    r = refb('3', pos)
    gt = '1' if rng.rand() < 0.7 else '0'
    kind = rng.choice(['snp'] * 6 + ['ins', 'del'])
    if kind == 'snp':
      recs.append(('3', pos, r, [other(r)], gt, '1'))
    elif kind == 'ins':
      recs.append(('3', pos, r, [r + randalt(3)], gt, '1'))
    else:
      recs.append(('3', pos, refb('3', pos, 4), [r], gt, '1'))
    pos += 80 + rng.randint(0, 300)

  with open(os.path.join(DATA, 'syn.vcf'), 'w') as fp:
    fp.write('##fileformat=VCFv4.1\n')
    for name, s in contigs:
      fp.write('##contig=<ID={},length={}>\n'.format(name, len(s)))
    fp.write('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n')
    fp.write('#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS0\tS1\n')
    for ch, p1, r, alts, gt1, gt0 in recs:
      fp.write('{}\t{}\t.\t{}\t{}\t50\tPASS\t.\tGT\t{}\t{}\n'.format(ch, p1, r, ','.join(alts), gt0, gt1))
  with open(os.path.join(DATA, 'syn.vcf'), 'rb') as fi, gzip.open(os.path.join(DATA, 'syn.vcf.gz'), 'wb') as fo:
    fo.write(fi.read())
  with open(os.path.join(DATA, 'syn.bed'), 'w') as fp:
    fp.write('1\t1000\t40000\n2\t0\t20000\n2\t15000\t16000\n3\t100\t7900\n')


def copy_ref_test_data():
  src = os.path.join(REF, 'mitty/test/data')
  for f in ['tiny.fasta', 'tiny.vcf', 'flawed-tiny.vcf', 'tiny.whole.bed', 'tiny.8-14.bed']:
    shutil.copy(os.path.join(src, f), os.path.join(DATA, f))


# ----------------------------------------------------------------------------------------------------------------
def main():
  os.makedirs(DATA, exist_ok=True)
  make_syn_inputs()
  copy_ref_test_data()

  sys.dont_write_bytecode = True
  sys.path[:0] = [os.path.join(HERE, 'refshim'), REF]
  import mitty.simulation.rpc as rpc
  import mitty.simulation.illumina as illumina
  import mitty.simulation.readgenerate as rg
  import mitty.simulation.readcorrupt as rc
  import mitty.lib.vcfio as vio
  import mitty.benchmarking.god_aligner as god

  models = {m: load_model(m) for m in MODELS}

  # ---- rng.json: raw MT19937 + legacy distribution vectors --------------------------------------------------
  rng_out = {}
  for seed in [0, 1, 7, 12345, 327741615, 4294967295]:
    rs = np.random.RandomState(seed)
    st = rs.get_state()
    d = {'words': np.random.RandomState(seed).randint(0, 2**32, size=1300, dtype=np.uint64).tolist()}
    d['doubles'] = [float(x).hex() for x in np.random.RandomState(seed).rand(500)]
    d['randint_seedmax'] = np.random.RandomState(seed).randint((1 << 32) - 1, size=64).tolist()
    d['randint_0_3'] = np.random.RandomState(seed).randint(0, 3, size=500).tolist()
    d['randint_i1'] = np.random.RandomState(seed).randint(2, size=501, dtype='i1').tolist()
    d['geometric_0.025'] = np.random.RandomState(seed).geometric(0.025, 2000).tolist()
    d['geometric_0.015'] = np.random.RandomState(seed).geometric(0.015, 2000).tolist()
    d['geometric_0.0125'] = np.random.RandomState(seed).geometric(0.0125, 2000).tolist()
    x = np.arange(1000, dtype=np.int64)
    np.random.RandomState(seed).shuffle(x)
    d['shuffle_1000'] = x.tolist()
    x = np.arange(70000, dtype=np.int64)
    np.random.RandomState(seed).shuffle(x)
    d['shuffle_70000_head'] = x[:200].tolist()
    d['shuffle_70000_sum_ix'] = int((x * np.arange(70000)).sum())
    d['state0_key_head'] = st[1][:8].tolist()
    rng_out[str(seed)] = d
  # read_model_params
  rng_out['read_model_params'] = {
    m: {str(cov): {k: (float(v).hex() if k == 'p' else v) for k, v in illumina.read_model_params(models[m], cov).items()
                   if k in ('p', 'passes', 'rlen')}
        for cov in [5.0, 10.0, 30.0, 60.0, 0.5, 200.0]} for m in MODELS}
  with open(os.path.join(HERE, 'rng.json'), 'w') as fp:
    json.dump(rng_out, fp)

  # ---- units.json ---------------------------------------------------------------------------------------------
  units = {}
  for seed in [7, 1, 99]:
    for passes in [1, 2, 4]:
      fake_vcf = [{'region': ('1', 0, 10), 'v': [[], []]}, {'region': ('2', 0, 10), 'v': [[]]},
                  {'region': ('3', 0, 10), 'v': [[], [], []]}, {'region': ('4', 0, 10), 'v': [[], []]}]
      units['{}:{}'.format(seed, passes)] = {
        'ploidy': [2, 1, 3, 2],
        'units': [[u['region_idx'], u['region_cpy'], int(u['rng_seed'])]
                  for u in rg.get_data_for_workers({'passes': passes}, fake_vcf, seed)]}
  with open(os.path.join(HERE, 'units.json'), 'w') as fp:
    json.dump(units, fp)

  # ---- templates.npz ------------------------------------------------------------------------------------------
  arrs = {}
  for m in MODELS:
    rm = illumina.read_model_params(models[m], 30.0)
    for seed in [7, 12345, 4000000000]:
      for (p_min, p_max) in [(1000, 201000), (5, 400)]:
        r = illumina.generate_reads(rm, p_min, p_max, seed)
        key = '{}|{}|{}|{}'.format(m, seed, p_min, p_max)
        arrs[key + '|fo0'] = r[0]['file_order']
        arrs[key + '|pos0'] = r[0]['pos']
        arrs[key + '|pos1'] = r[1]['pos']
  np.savez_compressed(os.path.join(HERE, 'templates.npz'), **arrs)

  # ---- nodes.json + reads.json --------------------------------------------------------------------------------
  fasta = sys.modules['pysam'].FastaFile(os.path.join(DATA, 'syn.fa'))
  node_out, read_out = {}, {}
  cases = [('syn', os.path.join(DATA, 'syn.vcf'), 'S1', os.path.join(DATA, 'syn.bed'), fasta),
           ('tiny', os.path.join(DATA, 'tiny.vcf'), 'g0_s0', os.path.join(DATA, 'tiny.whole.bed'),
            sys.modules['pysam'].FastaFile(os.path.join(DATA, 'tiny.fasta')))]
  prng = np.random.RandomState(5)
  for tag, vcf, sample, bed, fa in cases:
    vdf = vio.load_variant_file(vcf, sample, bed)
    for ri, reg in enumerate(vdf):
      region = reg['region']
      ref_seq = fa.fetch(reference=region[0], start=region[1], end=region[2])
      for cpy, vl in enumerate(reg['v']):
        nodes = rpc.create_node_list(ref_seq, region[1] + 1, vl)
        key = '{}|{}|{}'.format(tag, ri, cpy)
        node_out[key] = {'region': list(region), 'variants': [list(v.tuple()) for v in vl],
                         'nodes': [list(n.tuple()) for n in nodes]}
        p_min, p_max = nodes[0].ps, nodes[-1].ps + nodes[-1].oplen
        ps_l, l_l = [], []
        for l in (150, 250, 10, 1):
          lo = p_min
          hi = max(p_min + 1, p_max - l)
          if hi - lo < 400:
            pl = list(range(lo, hi))
          else:
            pl = sorted(set(prng.randint(lo, hi, 300).tolist()))
            for n in nodes:              # starts around every non-'=' node
              if n.cigarop != '=':
                for dp in (-l, -l + 1, -1, 0, 1, 2):
                  if lo <= n.ps + dp < hi:
                    pl.append(n.ps + dp)
          ps_l += pl
          l_l += [l] * len(pl)
        if not ps_l:
          continue
        pl = np.array(ps_l, dtype=np.int64)
        ll = np.array(l_l, dtype=np.uint32)
        n0, n1 = rpc.get_begin_end_nodes(pl, ll, nodes)
        out = []
        for p, l, a, b in zip(pl.tolist(), l_l, n0.tolist(), n1.tolist()):
          pos, cigar, v_list, seq = rpc.generate_read(p, l, a, b, nodes)
          out.append([p, l, a, b, int(pos), cigar, [int(v) for v in v_list], seq])
        read_out[key] = out
  with open(os.path.join(HERE, 'nodes.json'), 'w') as fp:
    json.dump(node_out, fp)
  with gzip.open(os.path.join(HERE, 'reads.json.gz'), 'wt') as fp:
    json.dump(read_out, fp)

  # ---- e2e FASTQ (threads=1 => byte-identical ordering) ------------------------------------------------------
  tmp = tempfile.mkdtemp()
  e2e_cfg = {'hiseq-X-v2.5-Garvan': (10.0, 7), '1kg-pcr-free': (6.0, 11)}
  for m in MODELS:
    cov, seed = e2e_cfg[m]
    f1, f2 = os.path.join(tmp, m + '.r1.fq'), os.path.join(tmp, m + '.r2.fq')
    rg.process_multi_threaded(os.path.join(DATA, 'syn.fa'), os.path.join(DATA, 'syn.vcf'), 'S1',
                              os.path.join(DATA, 'syn.bed'), illumina, models[m], cov, f1, f2, threads=1, seed=seed)
    for src, dst in ((f1, 'r1'), (f2, 'r2')):
      with open(src, 'rb') as fi, gzip.open(os.path.join(HERE, 'e2e_{}.{}.fq.gz'.format(m, dst)), 'wb', 6) as fo:
        fo.write(fi.read())
  with open(os.path.join(HERE, 'e2e_config.json'), 'w') as fp:
    json.dump({m: {'coverage': e2e_cfg[m][0], 'seed': e2e_cfg[m][1], 'sample': 'S1', 'fasta': 'data/syn.fa',
                   'vcf': 'data/syn.vcf', 'bed': 'data/syn.bed', 'threads': 1} for m in MODELS}, fp, indent=1)

  # ---- corruption (processes=1 => a single MT stream over the file) -----------------------------------------
  for m in MODELS:
    cin = []
    for r in ('r1', 'r2'):
      with gzip.open(os.path.join(HERE, 'e2e_{}.{}.fq.gz'.format(m, r)), 'rt') as fp:
        lines = fp.read().split('\n')
      n_rec = 300 * 4
      path = os.path.join(tmp, 'cin_{}_{}.fq'.format(m, r))
      with open(path, 'w') as fo:
        fo.write('\n'.join(lines[:n_rec]) + '\n')
      cin.append(path)
      with gzip.open(os.path.join(HERE, 'corrupt_in_{}.{}.fq.gz'.format(m, r)), 'wt') as fo:
        fo.write('\n'.join(lines[:n_rec]) + '\n')
    o1, o2 = os.path.join(tmp, 'cout1.fq'), os.path.join(tmp, 'cout2.fq')
    rc.multi_process(illumina, models[m], cin[0], o1, cin[1], o2, processes=1, seed=7)
    for src, dst in ((o1, 'r1'), (o2, 'r2')):
      with open(src, 'rb') as fi, gzip.open(os.path.join(HERE, 'corrupt_{}.{}.fq.gz'.format(m, dst)), 'wb') as fo:
        fo.write(fi.read())

  # ---- parse_qname + god-aligner records --------------------------------------------------------------------
  q_out, god_out = [], []

  class Seg:
    pass

  class FP:
    def __init__(self):
      self.recs = []

    def write(self, r):
      self.recs.append(r)

  sys.modules['pysam'].AlignedSegment = Seg
  ref_dict = {'1': 0, '2': 1, '3': 2}
  for m in MODELS:
    with gzip.open(os.path.join(HERE, 'e2e_{}.r1.fq.gz'.format(m)), 'rt') as fp:
      l1 = fp.read().split('\n')
    with gzip.open(os.path.join(HERE, 'e2e_{}.r2.fq.gz'.format(m)), 'rt') as fp:
      l2 = fp.read().split('\n')
    n = len(l1) // 4
    pick = sorted(set(list(range(0, n, max(1, n // 150))) +
                      [i for i in range(n) if '|>' in l1[4 * i]][:40]))
    for i in pick:
      qn = l1[4 * i][1:]
      q_out.append([qn, [list(r) for r in rg.parse_qname(qn)]])
      fp_ = FP()
      god.write_perfect_reads(qn, ref_dict, [(l1[4 * i + 1], l1[4 * i + 3]), (l2[4 * i + 1], l2[4 * i + 3])], fp_)
      god_out.append([qn, [{k: getattr(r, k) for k in ('qname', 'reference_id', 'pos', 'cigarstring', 'mapq',
                                                          'is_reverse', 'seq', 'qual', 'is_paired', 'is_proper_pair',
                                                          'is_read1', 'is_read2', 'pnext', 'rnext')}
                           for r in fp_.recs]])
  with open(os.path.join(HERE, 'qnames.json'), 'w') as fp:
    json.dump(q_out, fp)
  with open(os.path.join(HERE, 'god.json'), 'w') as fp:
    json.dump(god_out, fp)
  with open(os.path.join(HERE, 'god_header.json'), 'w') as fp:
    ann = os.path.join(tmp, 'x.ann')
    with open(ann, 'w') as fo:
      fo.write('1 1 11\n0 1 (null)\n0 50000 0\n0 2 (null)\n0 20000 0\n0 3 (null)\n0 8000 0\n')
    json.dump(god.parse_ann(ann), fp)
  shutil.rmtree(tmp)
  print('golden vectors written to', HERE)


if __name__ == '__main__':
  main()
