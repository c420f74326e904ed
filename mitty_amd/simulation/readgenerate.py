"""generate-reads orchestration, qname codec (reference mitty/simulation/readgenerate.py).

`process_multi_threaded` keeps the reference's signature (readgenerate.py:76-78).  The per-unit work runs on the
GPU (mitty_amd.engine); the host only parses inputs, walks the reference's work-unit order and streams the device
FASTQ arenas to the output files in that order.  Output is byte-identical to the reference run with --threads 1
(worker id 0, ps = index of the unit in the shuffled list): the reference's own multi-process output differs from
that only in the serial's worker/ps fields and in record order (SURVEY.md Finding 2).  `threads` is accepted for
CLI compatibility; `gpus` > 1 is handled by mitty_amd.distributed.
"""
import logging
import re
import time
from collections import namedtuple

from mitty_amd import _native
from mitty_amd.engine import Engine
from mitty_amd.lib import fasta as mfasta
from mitty_amd.lib import vcfio
from mitty_amd.lib.fastq_stream import FastqSink, PairWriter

logger = logging.getLogger(__name__)

SEED_MAX = (1 << 32) - 1
DNA_complement = str.maketrans('ATCGN', 'TAGCN')

__qname_format__ = '@read_serial|chrom|copy|strand|pos|rlen|cigar|vs1,vs2,...|strand|pos|rlen|cigar|vs1,vs2,...'
__qname_format_details__ = """
@read_serial|chrom|copy|strand|pos|rlen|cigar|vs1,vs2,...|strand|pos|rlen|cigar|vs1,vs2,...
    |          |     |    |     |    |    |        |         |                      |
 unique        |     |    |     | read    |        |         ---- repeated for ------
 code for      |     |    |     | len     |        |          other read in template
 template      |     |    |     |         |        |
               |     |    |     |     cigar    comma separated
      chrom read     |    |     |              list of sizes of
  was taken from     |    |     |              variants this read
       One based     |    |     |              covers
                     |    |     |
                     |    |     |
    copy of chrom read    |     |
 was taken from (0, 1)    |     |
                          |     |
         forward strand (0)     |
      or reverse strand (1)     |
                                |
                      pos of read
                        One based

The chrom and pos are one based to make comparing qname info in genome browser easier

For reads from inside a long insertion the CIGAR has the following format:

  '>p:nI'

where:

 '>' is the unique key that indicates a read inside a long insertion
 'p' is how many bases into the insertion branch the read starts
 'n' is simply the length of the read
"""


def get_data_for_workers(model, vcf, seed):
  """Work units in the reference's order (readgenerate.py:129-159).  `vcf` entries need 'ploidy' or 'v'."""
  ploidy = [v['ploidy'] if 'ploidy' in v else len(v['v']) for v in vcf]
  for r, c, s in _native.work_units(seed, ploidy, model['passes']):
    yield {'region_idx': r, 'region_cpy': c, 'rng_seed': s}


def process_multi_threaded(fasta_fname, vcf_fname, sample_name, bed_fname, read_module, model, coverage,
                           fastq1_fname, fastq2_fname, threads=2, seed=7, device=0, rng='mitty', corrupt_seed=None,
                           flush_bytes=1 << 30, max_batch_units=32, max_batch_draws=200_000_000, compress=None,
                           gz_level=6, gz_threads=8, gz_device=True, stage_times=False):
  """Generate reads for every (region, copy, pass) unit and write FASTQ (reference readgenerate.py:76-126).

  compress: None = BGZF for file names ending in '.gz' (FastqSink), True / False forces it; gz_device: deflated on
  the GPU (mh_output_bgzf) straight from the arenas, else on gz_threads host threads at gz_level.  Returns a stats
  dict (templates sampled, kept, bytes, seconds; setup_s = inputs parsed (parse_s) and loaded, run_s = the unit loop
  = gpu_s + flush_s, flush_s = fetch_s (waiting for the GPU and its D2H, deflate included) + write_s (waiting for
  the file writes to free a staging slot) + bookkeeping, close_s = files closed and the engine released).
  stage_times: also the device's per-stage times (stages_ms: e.g. bgzf_deflate, bgzf_d2h, output_d2h, emit).
  """
  t0 = time.time()
  read_model = read_module.read_model_params(model, coverage)
  vdf = vcfio.load_variants_soa(vcf_fname, sample_name, bed_fname)
  seqs = mfasta.read_fasta(fasta_fname, names={r['region'][0] for r in vdf})
  units = list(get_data_for_workers(read_model, vdf, seed))
  logger.debug('{} passes will be made'.format(len(units)))
  t_parse = time.time()
  eng = Engine(device)
  if stage_times:
    eng.ctx.enable_timing(True)
  if corrupt_seed is not None:
    import numpy as np
    eng.ctx.set_corruption(True, model['cum_bq_mat'], 10 ** (-np.arange(100) / 10), corrupt_seed)
  for ri, reg in enumerate(vdf):
    chrom, s0, e = reg['region']
    eng.load_region(ri, reg['region'], mfasta.fetch(seqs, chrom, s0, e))
  stats = {'units': len(units), 'templates': 0, 'kept': 0, 'bytes1': 0, 'bytes2': 0, 'setup_s': time.time() - t0,
           'parse_s': t_parse - t0, 'fetch_s': 0.0, 'write_s': 0.0, 'flush_s': 0.0}
  write2 = fastq2_fname is not None
  fp1 = FastqSink(fastq1_fname, gz_level, gz_threads, compress)   # '.gz' names get BGZF output
  fp2 = FastqSink(fastq2_fname, gz_level, gz_threads, compress) if write2 else None

  # page-locked D2H staging: two slots (double buffering) of one buffer per file; each file is written on its own
  # thread (PairWriter), so a FIFO reader that takes the two files in lockstep (examples/reads/run.sh:13-16) is never
  # starved of one while we block on the other, and the next chunk's D2H overlaps the writes of this one
  sinks = [fp1, fp2 if write2 else None]
  pw = PairWriter(sinks)
  pins = [[_native.PinnedBuffer(), _native.PinnedBuffer()] for _ in range(2)]
  nslot = [0]
  CHUNK = 64 << 20   # (page-locking costs ~0.1 s per GB: four 64 MiB slots, not four 256 MiB ones)
  GZ_CHUNK = 4096 * 0xff00   # whole BGZF blocks: the members equal one compression of the whole arena

  def flush(ps, n, kept, b1, b2):
    tfl = time.time()
    try:
      _flush(ps, n, kept, b1, b2)
    finally:
      stats['flush_s'] += time.time() - tfl

  def _flush(ps, n, kept, b1, b2):
    stats['templates'] += n
    stats['kept'] += kept
    stats['bytes1'] += b1
    stats['bytes2'] += b2
    u1, u2 = eng.ctx.output_size()
    if u1 + u2 >= flush_bytes or ps == len(units) - 1:
      if gz_device and all(s is None or s.gz for s in sinks):
        # BGZF members deflated on the GPU from the arenas (chunks of whole 0xff00-byte blocks), then D2H of the
        # compressed bytes only: a chunk's copies run behind its deflates on a second stream, beside the next
        # chunk's deflates, and the chunk goes to the writers once they are in
        pending = None
        for off in range(0, max(u1, u2), GZ_CHUNK):
          slot = nslot[0] % 2
          nslot[0] += 1
          tw = time.time()
          pw.wait(slot)   # the writes of this slot's previous chunk
          tf = time.time()
          n1, n2 = max(0, min(GZ_CHUNK, u1 - off)), max(0, min(GZ_CHUNK, u2 - off))
          ticket, z = eng.ctx.output_bgzf_pair(pins[slot], off, n1, n2)
          if pending is not None:
            eng.ctx.output_bgzf_wait(pending[0])
            pw.submit(*pending[1:])
          pending = (ticket, slot, [z[0] if n1 else None, z[1] if n2 else None], [n1, n2])
          stats['write_s'] += tf - tw
          stats['fetch_s'] += time.time() - tf
        if pending is not None:
          tf = time.time()
          eng.ctx.output_bgzf_wait(pending[0])
          pw.submit(*pending[1:])
          stats['fetch_s'] += time.time() - tf
      else:
        # two chunks' copies in flight: chunk k's D2H is queued before chunk k - 1 goes to the writers
        pending = None
        for off in range(0, max(u1, u2), CHUNK):
          slot = nslot[0] % 2
          nslot[0] += 1
          tw = time.time()
          pw.wait(slot)   # the writes of this slot's previous chunk
          tf = time.time()
          n1, n2 = max(0, min(CHUNK, u1 - off)), max(0, min(CHUNK, u2 - off))
          ticket, (d1, d2) = eng.ctx.fetch_range_async(pins[slot], off, n1, off, n2)
          if pending is not None:
            eng.ctx.fetch_wait(pending[0])
            pw.submit(*pending[1:])
          pending = (ticket, slot, [d1 if n1 else None, d2 if n2 else None])
          stats['write_s'] += tf - tw
          stats['fetch_s'] += time.time() - tf
        if pending is not None:
          tf = time.time()
          eng.ctx.fetch_wait(pending[0])
          pw.submit(*pending[1:])
          stats['fetch_s'] += time.time() - tf
      eng.ctx.reset_output()

  t_run = time.time()
  try:
    # batches of units sampled together (their MT19937 streams run concurrently); order of emission unchanged
    batch, batch_draws = [], 0
    for ps, wd in enumerate(units):
      ri, cpy = wd['region_idx'], wd['region_cpy']
      reg = vdf[ri]['region']
      batch.append((ps, ri, cpy, wd['rng_seed']))
      batch_draws += int((reg[2] - reg[1]) * read_model['p'] * 1.2)
      if len(batch) >= max_batch_units or batch_draws >= max_batch_draws or ps == len(units) - 1:
        t1 = time.time()
        eng.run_units(batch, lambda r, c: vdf[r]['copies'][c], read_model['p'], read_model['rlen'],
                      read_model['cum_tlen'], sample_name, 0, write2, rng, on_unit=flush)
        logger.debug('Units {}..{}: {:0.3f}s'.format(batch[0][0], batch[-1][0], time.time() - t1))
        batch, batch_draws = [], 0
  finally:
    # run_s: the unit loop (GPU job + flushes); gpu_s = run_s - flush_s: splice, sampling and emission as the host
    # sees them
    stats['run_s'] = time.time() - t_run
    stats['gpu_s'] = stats['run_s'] - stats['flush_s']
    if stage_times:
      agg = {}
      for name, ms in eng.ctx.stage_times():
        agg[name] = agg.get(name, 0.0) + ms
      stats['stages_ms'] = {k: round(v, 2) for k, v in sorted(agg.items(), key=lambda kv: -kv[1])}
    t_close = time.time()
    try:
      tw = time.time()
      pw.close()
      stats['write_s'] += time.time() - tw
    finally:
      fp1.close()
      if fp2:
        fp2.close()
      eng.close()
      for slot in pins:
        for b in slot:
          b.free()
  stats['written1'], stats['written2'] = fp1.written, fp2.written if fp2 else 0
  stats['close_s'] = time.time() - t_close
  stats['seconds'] = time.time() - t0
  return stats


def fastq_lines(n, chrom, cpy, reads):
  """readgenerate.fastq_lines (readgenerate.py:222-230) — host-side formatter for single templates."""
  qname = '@{}|{}|{}'.format(n, chrom, cpy)
  for r in reads:
    qname += '|{}|{}|{}|{}|{}'.format(r[0], r[1], r[2], r[3], ','.join(str(int(v)) for v in r[4]))
  return [qname + '\n' + r[5] + '\n+\n' + '~' * int(r[2]) + '\n' for r in reads]


ri = namedtuple('ReadInfo', ['sample', 'rid', 'chrom', 'cpy', 'strand', 'pos', 'rlen', 'cigar', 'special_cigar',
                             'v_list'])


def parse_qname(qname):
  """readgenerate.parse_qname (readgenerate.py:259-291): the qname's reads, in file order, as ReadInfo.

  A read from inside a long insertion carries the CIGAR '>p:nI'; it is reported as cigar 'nI' with the original in
  special_cigar.  Fields of a trailing incomplete read are ignored, as the reference's zip() ignores them."""
  fields = qname.split('|')
  rid, chrom, cpy = fields[0], fields[1], int(fields[2])
  sample = rid[:rid.index(':')]   # ValueError without a ':' (the reference's tuple unpacking raises too)
  reads = []
  for k in range(3, 3 + 5 * ((len(fields) - 3) // 5), 5):
    strand, pos, rlen, cigar, vs = fields[k:k + 5]
    special = cigar if cigar[:1] == '>' else None
    reads.append(ri(sample, rid, chrom, cpy, int(strand), int(pos), int(rlen),
                    cigar.rpartition(':')[2] if special else cigar, special, [int(x) for x in vs.split(',') if x]))
  return reads


cigar_parser = re.compile(r'(\d+)(\D)')
