"""god-aligner: a perfectly aligned BAM from simulated FASTQ (reference mitty/benchmarking/god_aligner.py:19-183,
CLI cli.py:183-204), MI355X build.

The reference feeds templates through worker processes that build pysam records (write_perfect_reads,
god_aligner.py:153-183), then runs `samtools cat`, `sort -m 2G` and `index` via pysam (:117-131).  Here the FASTQ
bytes go to the GPU in large chunks; parsing, record encoding and the coordinate sort run on the device
(mitty_amd/csrc/mh_bam.hip); the host only deflates BGZF blocks on a thread pool and writes the BAI
(mh_bgzf.cpp).  Records equal write_perfect_reads' (pinned by tests/golden/god.json); the order is samtools
sort's coordinate order (tid, pos+1, strand), input order on ties.

Header: construct_header (:19-28) rendered the way pysam renders a header dict (records HD, SQ, RG, PG; fields in
pysam's order; values through str(), so the base64 RG ID keeps its b'...' form and an absent sample name reads
'None'), with SO:coordinate added to @HD as samtools sort does.  samtools' own @PG line is not added (its text
depends on the samtools version bundled with pysam).
"""
import base64
import logging
import os
import sys
import time

from mitty_amd import _native
from mitty_amd.lib.fastq_stream import stream_templates

logger = logging.getLogger(__name__)

__version__ = '2.7.3.dev0'

# pysam's output order of the fields within header records
_FIELD_ORDER = {'HD': ('VN', 'SO', 'GO'),
                'SQ': ('SN', 'LN', 'AS', 'M5', 'UR', 'SP', 'AH'),
                'RG': ('ID', 'CN', 'SM', 'LB', 'PU', 'PI', 'DT', 'DS', 'PL', 'FO', 'KS', 'PG', 'PM'),
                'PG': ('PN', 'ID', 'VN', 'PP', 'DS', 'CL')}


def construct_header(fasta_ann, rg_id, sample='S'):
  """god_aligner.construct_header (:19-28)."""
  return {
    'HD': {'VN': '1.0'},
    'PG': [{'CL': ' '.join(sys.argv),
            'ID': 'mitty-god-aligner',
            'PN': 'god-aligner',
            'VN': __version__}],
    'RG': [{'ID': rg_id, 'SM': sample}],
    'SQ': parse_ann(fasta_ann)
  }


def parse_ann(fn):
  """Given a fasta.ann file name parse it (god_aligner.py:31-40)."""
  logger.debug('Parsing {} for sequence header information'.format(fn))
  ln = open(fn, 'r').readlines()[1:]
  return [{'SN': ln[n].split()[1], 'LN': int(ln[n + 1].split()[1])} for n in range(0, len(ln), 2)]


def _header_line(fields, record):
  line = ['@' + record]
  for key in _FIELD_ORDER[record]:
    if key in fields:
      line.append('{}:{}'.format(key, str(fields[key])))
  for key in fields:
    if not key.isupper():
      line.append('{}:{}'.format(key, str(fields[key])))
  return '\t'.join(line)


def header_text(hdr, sorted_by='coordinate'):
  """SAM header text of a header dict as pysam writes it, plus samtools sort's SO tag."""
  lines = []
  for record in ('HD', 'SQ', 'RG', 'PG'):
    if record not in hdr:
      continue
    data = hdr[record]
    if record == 'HD' and sorted_by:
      data = dict(data)
      data['SO'] = sorted_by
    for fields in ([data] if isinstance(data, dict) else data):
      lines.append(_header_line(fields, record))
  for co in hdr.get('CO', []):
    lines.append('@CO\t' + co)
  return '\n'.join(lines) + '\n'


def process_multi_threaded(fasta, bam_fname, fastq1, fastq2=None, threads=1, max_templates=None,
                           sample_name='Seven', device=0, level=6, chunk_bytes=1 << 30, gpu_bgzf=False,
                           hbm_capacity=0):
  """god_aligner.process_multi_threaded (:44-131): `bam_fname` (coordinate-sorted BAM) + `bam_fname.bai`.

  As in the reference, max_templates stops after template index max_templates, i.e. max_templates + 1 templates.
  `threads` sizes the BGZF deflate pool; gpu_bgzf: the record blocks deflated on the device instead
  (mh_bam_write_gpu: the same BAM stream, only the compressed bytes leave the GPU).  hbm_capacity: record bytes held
  in HBM before they spill to host memory (0: no limit) — the reference sorts with `samtools sort -m 2G`, an external
  merge sort in bounded memory (god_aligner.py:100-116); here only the records' bytes leave HBM, their keys stay and
  are sorted on the device, and the sorted stream is assembled on the host (mh_bam_set_capacity).
  """
  rg_id = base64.b64encode(' '.join(sys.argv).encode('ascii'))
  hdr = construct_header(fasta + '.ann', rg_id=rg_id, sample=sample_name)
  t0 = time.time()
  ctx = _native.Context(device)
  try:
    ctx.bam_set_refs([s['SN'] for s in hdr['SQ']], [s['LN'] for s in hdr['SQ']])
    ctx.bam_set_capacity(hbm_capacity)
    limit = None if max_templates is None else max_templates + 1
    n_t = stream_templates(fastq1, fastq2, lambda b1, b2, want, done: ctx.bam_add_fastq(b1, b2, want),
                           chunk_bytes, limit)
    if gpu_bgzf:
      n_rec, n_bytes, _ = ctx.bam_write_gpu(bam_fname, header_text(hdr), bai_path=bam_fname + '.bai')
    else:
      n_rec, n_bytes = ctx.bam_write(bam_fname, header_text(hdr), level=level, threads=max(threads, 1),
                                     bai_path=bam_fname + '.bai')
    spilled = ctx.bam_spilled()
  finally:
    ctx.close()
  logger.debug('Processed {} templates ({} records) in {:0.2f}s'.format(n_t, n_rec, time.time() - t0))
  return {'templates': n_t, 'records': n_rec, 'bam_bytes_uncompressed': n_bytes, 'seconds': time.time() - t0,
          'spilled_bytes': spilled[0], 'spill_blocks': spilled[1]}
