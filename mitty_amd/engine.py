"""Device-resident generate-reads pipeline for one GPU (the orchestration of reference readgenerate.py:76-218).

One Engine = one HIP context.  Per BED region the fetched reference bytes are uploaded once; per (region, copy)
the haplotype is spliced on the device once and kept resident for all of that copy's passes; per work unit
(region, copy, pass) the templates are sampled and the FASTQ records emitted into device arenas.
"""
import logging

from mitty_amd import _native

logger = logging.getLogger(__name__)

RNG_MODES = {'mitty': _native.MH_RNG_MITTY, 'philox': _native.MH_RNG_PHILOX}


class Engine:
  SLOTS_PER_REGION = 64

  def __init__(self, device=0):
    self.ctx = _native.Context(device)
    self.device = device
    self._regions = {}   # ri -> region tuple (contig uploaded)
    self._haps = {}      # (ri, cpy) -> (slot, n_nodes, p_min, p_max)

  def close(self):
    self.ctx.close()

  def load_region(self, ri, region, ref_seq):
    self.ctx.upload_contig(ri, ref_seq)
    self._regions[ri] = region

  def haplotype(self, ri, cpy, soa):
    key = (ri, cpy)
    if key not in self._haps:
      region = self._regions[ri]
      slot = ri * self.SLOTS_PER_REGION + cpy
      n_nodes, p_min, p_max = self.ctx.build_haplotype(slot, ri, region[1] + 1, soa)
      self._haps[key] = (slot, n_nodes, p_min, p_max)
    return self._haps[key]

  def drop_haplotypes(self):
    for slot, *_ in self._haps.values():
      self.ctx.release_haplotype(slot)
    self._haps.clear()

  def run_unit(self, ps, ri, cpy, rng_seed, soa, p, rlen, cum_tlen, sample_name, worker_id=0, write_fastq2=True,
               rng='mitty'):
    """One work unit: sample templates, emit FASTQ.  Returns (n_templates, kept, bytes1, bytes2)."""
    chrom = self._regions[ri][0]
    slot, _, _, _ = self.haplotype(ri, cpy, soa)
    n = self.ctx.sample_templates(slot, p, rlen, cum_tlen, rng_seed, RNG_MODES[rng])
    kept, b1, b2 = self.ctx.emit_reads(slot, '{}:{}:{}'.format(sample_name, worker_id, ps), chrom, cpy,
                                       write_fastq2, unit_key=rng_seed)
    return n, kept, b1, b2
