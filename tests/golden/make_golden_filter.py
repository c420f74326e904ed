#!/usr/bin/env python3
"""Capture the filter-variants fixture from the reference (vcfio.prepare_variant_file, vcfio.py:129-168; CLI
cli.py:20-35) — build container only.

Run:  python tests/golden/make_golden_filter.py     (needs /root/reference; writes tests/golden/data/filt.*,
                                                      tests/golden/filter_variants.json)

Input: our own two-sample VCF with SNVs, indels, complex records (REF > 1 with a longer ALT in the sample's
genotype; multi-allelic with the complex allele in or out of the genotype; REF-equal alleles), haploid and missing
genotypes on single-base records, INFO END spans, and BED regions that overlap (a record in two regions is written
twice by the reference).  Output: the records the reference writes, in order, as [CHROM, POS, ID, REF, ALT, sample
column] — the retained-record set.  Header text and field re-serialisation by htslib are not captured (no htslib
in the image): the shim writer records fields as given.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
DATA = os.path.join(HERE, 'data')


def make_inputs():
  rs = np.random.RandomState(4242)
  seq = {c: ''.join('ACGT'[i] for i in rs.randint(0, 4, 3000)) for c in ('1', '2')}
  recs = []
  gts = ['0|1', '1|0', '1|1', '0|0', '1|2', '2|1', '0|2', '0/1', '1', '.|1', '.']
  for c in ('1', '2'):
    pos = 5
    while pos < 2900:
      kind = rs.randint(0, 7)
      ref = seq[c][pos - 1]
      if kind == 0:                                     # SNV
        alts = [('ACGT'.replace(ref, ''))[rs.randint(0, 3)]]
      elif kind == 1:                                   # insertion
        alts = [ref + ''.join('ACGT'[i] for i in rs.randint(0, 4, rs.randint(1, 5)))]
      elif kind == 2:                                   # deletion
        ref = seq[c][pos - 1:pos - 1 + rs.randint(2, 6)]
        alts = [ref[0]]
      elif kind == 3:                                   # complex: REF > 1 and a longer, different ALT
        ref = seq[c][pos - 1:pos + 2]
        alts = [ref[0] + 'TT', ref[0]]
      elif kind == 4:                                   # multi-allelic deletion + complex second allele
        ref = seq[c][pos - 1:pos + 1]
        alts = [ref[0], ref + 'G']
      elif kind == 5:                                   # MNP (REF 2, ALT 2)
        ref = seq[c][pos - 1:pos + 1]
        alts = ['GG' if ref != 'GG' else 'CC']
      else:                                             # REF > 1 with an ALT equal to REF (not complex)
        ref = seq[c][pos - 1:pos + 1]
        alts = [ref[0], ref]
      gt = gts[rs.randint(0, len(gts))]
      if len(ref) > 1 and '.' in gt:                    # the reference raises on a missing allele there
        gt = '0|1'
      if any(int(g) > len(alts) for g in gt.replace('/', '|').split('|') if g != '.'):
        gt = '0|1'
      other = gts[rs.randint(0, 8)]
      info = '.' if rs.rand() < 0.8 else 'DP=7;END={}'.format(pos + len(ref) - 1 + rs.randint(0, 40))
      recs.append((c, pos, ref, ','.join(alts), info, other, gt))
      pos += len(ref) + rs.randint(2, 40)
  with open(os.path.join(DATA, 'filt.vcf'), 'w') as fp:
    fp.write('##fileformat=VCFv4.1\n##contig=<ID=1,length=3000>\n##contig=<ID=2,length=3000>\n')
    fp.write('##INFO=<ID=DP,Number=1,Type=Integer,Description="Depth">\n')
    fp.write('##INFO=<ID=END,Number=1,Type=Integer,Description="End">\n')
    fp.write('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n')
    fp.write('#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tOTHER\tS1\n')
    for k, (c, pos, ref, alt, info, other, gt) in enumerate(recs):
      fp.write('{}\t{}\tv{}\t{}\t{}\t50\tPASS\t{}\tGT\t{}\t{}\n'.format(c, pos, k, ref, alt, info, other, gt))
  with open(os.path.join(DATA, 'filt.bed'), 'w') as fp:
    fp.write('1\t0\t1200\n1\t1000\t2000\n2\t100\t2950\n')


def main():
  make_inputs()
  sys.dont_write_bytecode = True
  sys.path[:0] = [os.path.join(HERE, 'refshim'), REF]
  import mitty.lib.vcfio as vio
  with tempfile.TemporaryDirectory() as td:
    out = os.path.join(td, 'out.vcf')
    vio.prepare_variant_file(os.path.join(DATA, 'filt.vcf'), 'S1', os.path.join(DATA, 'filt.bed'), out)
    lines = [ln.rstrip('\n').split('\t') for ln in open(out) if not ln.startswith('#')]
  kept = [[f[0], int(f[1]), f[2], f[3], f[4], f[9]] for f in lines]
  with open(os.path.join(HERE, 'filter_variants.json'), 'w') as fp:
    json.dump({'sample': 'S1', 'records': kept}, fp)
  print('{} records written by the reference'.format(len(kept)))


if __name__ == '__main__':
  main()
