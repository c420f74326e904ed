"""Device-resident generate-reads pipeline for one GPU (the orchestration of reference readgenerate.py:76-218).

One Engine = one HIP context.  Per BED region the fetched reference bytes are uploaded once; per (region, copy)
the haplotype is spliced on the device once and kept resident for all of that copy's passes; work units
(region, copy, pass) are sampled in batches — all their MT19937 streams generated at once in jump-ahead
segments — and then emitted one by one, in the reference's unit order, into the device FASTQ arenas.
"""
import logging

from mitty_amd import _native

logger = logging.getLogger(__name__)

RNG_MODES = {'mitty': _native.MH_RNG_MITTY, 'philox': _native.MH_RNG_PHILOX}


class Engine:
  SLOTS_PER_REGION = 64
  TPL_BATCH = 1 << 20   # template-set ids: [0, TPL_BATCH) and [TPL_BATCH, 2 * TPL_BATCH), alternating per batch

  EMIT_SETS = 4   # the two-pass path: units prepared ahead of their writers (of the library's 16 emission buffer sets)

  def __init__(self, device=0, emit_mode=0):
    """emit_mode (mh_set_emit_mode): 0 every unit queued with no host readback (mh_emit_reads_async: measure pass,
    tile scan and writer chained on the device); 3 the same through the single-pass writer (k_emit_fused); 2 the
    two-pass path with the host reading each unit's totals before its writer (round 5's flow; A/B and tests); 1 the
    LDS-image writer."""
    self.ctx = _native.Context(device)
    self.device = device
    self.emit_mode = emit_mode
    if emit_mode:
      self.ctx.set_emit_mode(emit_mode)
    self._regions = {}   # ri -> region tuple (contig uploaded)
    self._haps = {}      # (ri, cpy) -> (slot, n_nodes, p_min, p_max)
    self._pre = {}       # (ri, cpy) -> (slot, ...) prefetched for the next step (adopted by drop_haplotypes)
    self._gen = {}       # (ri, cpy) -> the generation (0 / 1) of its last slot: a new build takes the other one
    self._vsets = {}     # (ri, cpy) -> resident variant set id (upload_variants)
    self._tpl_base = 0
    self._lazy_n = []    # template counts of the units queued by run_units and not yet collected
    self._two_pass_done = []

  def close(self):
    self.ctx.close()

  def load_region(self, ri, region, ref_seq):
    self.ctx.upload_contig(ri, ref_seq)
    self._regions[ri] = region

  def upload_variants(self, ri, cpy, soa):
    """Keep (ri, cpy)'s variants in HBM: later haplotype builds of that copy splice from the device copy."""
    vset = ri * self.SLOTS_PER_REGION + cpy
    self.ctx.upload_variants(vset, soa)
    self._vsets[(ri, cpy)] = vset

  def _slot(self, key):
    """A slot for a new build of key: the generation its last slot did not use (that one may still be live)."""
    g = 1 - self._gen.get(key, 1)
    self._gen[key] = g
    return key[0] * self.SLOTS_PER_REGION + 2 * g + key[1]

  def haplotype(self, ri, cpy, soa):
    key = (ri, cpy)
    if key not in self._haps:
      region = self._regions[ri]
      slot = self._slot(key)
      if key in self._vsets:
        n_nodes, p_min, p_max = self.ctx.build_haplotype_vset(slot, ri, region[1] + 1, self._vsets[key])
      else:
        n_nodes, p_min, p_max = self.ctx.build_haplotype(slot, ri, region[1] + 1, soa)
      self._haps[key] = (slot, n_nodes, p_min, p_max)
    return self._haps[key]

  def haplotypes(self, keys):
    """Build the haplotypes of several (ri, cpy) keys whose variants are resident (upload_variants), two copies at a
    time side by side (mh_build_haplotypes_vset); keys already built are kept."""
    todo = [k for k in dict.fromkeys(keys) if k not in self._haps and k in self._vsets]
    if todo:
      slots = [self._slot(k) for k in todo]
      res = self.ctx.build_haplotypes_vset(slots, [ri for ri, _ in todo],
                                           [self._regions[ri][1] + 1 for ri, _ in todo],
                                           [self._vsets[k] for k in todo])
      for k, slot, r in zip(todo, slots, res):
        self._haps[k] = (slot,) + tuple(r)

  def prefetch(self, units, next_step=False, p=None, rng='mitty'):
    """Build the haplotypes of the next batch's units [(ps, ri, cpy, seed)] while the current one is sampled and
    written, and (given p, rng 'mitty') their MT19937 word streams (mh_prefetch_haplotypes_vset: returns at once, the
    splices and the word generation off the batch boundary's critical path).  Keys already built are kept, unless
    next_step: then every key gets a fresh build (into its other slot generation), kept apart until drop_haplotypes
    adopts them for the next step."""
    keys = [(ri, cpy) for _, ri, cpy, _ in units]
    todo = [k for k in dict.fromkeys(keys) if k in self._vsets and k not in self._pre and
            (next_step or k not in self._haps)]
    slots = [self._slot(k) for k in todo]
    for k, slot in zip(todo, slots):   # (n_nodes, p_min, p_max: not known until the splice has run; get_nodes)
      (self._pre if next_step else self._haps)[k] = (slot, None, None, None)
    home = self._pre if next_step else self._haps
    words = p is not None and rng == 'mitty' and all(k in home for k in keys)
    if not todo and not words:
      return
    self.ctx.prefetch_haplotypes_vset(slots, [ri for ri, _ in todo], [self._regions[ri][1] + 1 for ri, _ in todo],
                                      [self._vsets[k] for k in todo],
                                      [home[k][0] for k in keys] if words else (),
                                      [u[3] for u in units] if words else (), p if words else 1.0)

  def drop_variants(self):
    for vset in self._vsets.values():
      self.ctx.release_variants(vset)
    self._vsets.clear()

  def drop_haplotypes(self):
    """Release the haplotypes; those prefetched for the next step (prefetch(..., next_step=True)) become current."""
    for slot, *_ in self._haps.values():
      self.ctx.release_haplotype(slot)
    self._haps, self._pre = self._pre, {}

  def run_units(self, units, soa_of, p, rlen, cum_tlen, sample_name, worker_id=0, write_fastq2=True, rng='mitty',
                on_unit=None, lazy=False, prefetch=None, prefetch_next_step=False, prefetch_after=1):
    """Sample a batch of work units together, then emit them in order.

    units: [(ps, ri, cpy, rng_seed)]; soa_of(ri, cpy) -> variant SoA.  on_unit(ps, n, kept, b1, b2) runs after each
    unit's emission (e.g. to stream the arena to files).  Returns [(n, kept, b1, b2)] per unit; lazy=True returns None
    and leaves the units' results to collect(), so the caller queues the next batch while these writers run.
    prefetch: the next batch's units [(ps, ri, cpy, seed)] (same p and rng), whose haplotypes and word streams are
    built (Engine.prefetch) once unit `prefetch_after` is queued (-1: before unit 0) instead of at the next batch's
    start; unit 1 measured best (the wait for the batch's head is over, and the prefetch has the rest of the batch to
    finish before the next head needs it).
    """
    self.haplotypes([(ri, cpy) for _, ri, cpy, _ in units])
    slots = [self.haplotype(ri, cpy, soa_of(ri, cpy))[0] for _, ri, cpy, _ in units]
    # template ids alternate between two ranges per batch, so this batch's sampling never waits for the previous
    # batch's FASTQ writers (still queued on their own stream) to finish reading theirs
    base = self._tpl_base
    self._tpl_base = self.TPL_BATCH - base
    # the units' last sampling stages run on without a host wait; each unit's template set is resolved when its
    # emission first uses it (unit 0's writer does not wait for the whole batch's tail)
    self.ctx.sample_units_async([base + k for k in range(len(units))], slots, [u[3] for u in units], p, rlen,
                                cum_tlen, RNG_MODES[rng])
    # every unit's writer queued as soon as its templates are resolved (mh_emit_reads_async: the single-pass writer,
    # no measure pass and no readback between units); the writers drain while the caller moves on
    if self.emit_mode in (1, 2):
      return self._emit_two_pass(units, slots, base, sample_name, worker_id, write_fastq2, on_unit, lazy)
    out = []
    at = min(prefetch_after, len(units) - 1) if prefetch else -1
    if prefetch and prefetch_after < 0:   # (before unit 0: beside this batch's sampling head)
      self.prefetch(prefetch, prefetch_next_step, p, rng)
    for k, (ps, ri, cpy, seed) in enumerate(units):
      self.ctx.use_templates(base + k)
      self.ctx.emit_async(slots[k], '{}:{}:{}'.format(sample_name, worker_id, ps), self._regions[ri][0], cpy,
                          write_fastq2, unit_key=seed)
      self._lazy_n.append(self.ctx.template_count(base + k))
      if k == at:
        self.prefetch(prefetch, prefetch_next_step, p, rng)
      if on_unit is not None:
        done = self.collect()
        out += done
        on_unit(ps, *done[-1])
    if on_unit is not None:
      return out
    return None if lazy else self.collect()

  def _emit_two_pass(self, units, slots, base, sample_name, worker_id, write_fastq2, on_unit, lazy):
    # measure passes of up to EMIT_SETS units first (main stream), then their writers queued back to back (writer
    # stream).  Unit 0 goes alone: preparing a unit waits for its sampling tail, so at a batch boundary the idle
    # writer stream would otherwise wait for the tails and measure passes of the whole first chunk
    out = []
    order = list(enumerate(units))
    k0 = 1 if len(units) > 1 else 0
    chunks = ([order[:1]] if k0 else []) + [order[c0:c0 + self.EMIT_SETS]
                                            for c0 in range(k0, len(units), self.EMIT_SETS)]
    for chunk in chunks:
      for k, (ps, ri, cpy, seed) in chunk:
        self.ctx.use_templates(base + k)
        self.ctx.emit_prepare(slots[k], '{}:{}:{}'.format(sample_name, worker_id, ps), self._regions[ri][0], cpy,
                              write_fastq2, unit_key=seed, wait=False)
      for k, (ps, ri, cpy, seed) in chunk:
        self.ctx.use_templates(base + k)
        kept, b1, b2 = self.ctx.emit_reads(slots[k], '{}:{}:{}'.format(sample_name, worker_id, ps),
                                           self._regions[ri][0], cpy, write_fastq2, unit_key=seed)
        n = self.ctx.template_count(base + k)
        out.append((n, kept, b1, b2))
        if on_unit is not None:
          on_unit(ps, n, kept, b1, b2)
    if lazy:
      self._two_pass_done += out
      return None
    return out

  def collect(self):
    """[(n, kept, b1, b2)] of every unit queued by run_units since the last collect (waits for their writers)."""
    if self.emit_mode in (1, 2):
      out, self._two_pass_done = self._two_pass_done, []
      return out
    res = self.ctx.emit_collect()
    if len(res) != len(self._lazy_n):
      raise RuntimeError('emit_collect returned {} units for {} queued'.format(len(res), len(self._lazy_n)))
    out = [(n,) + tuple(r) for n, r in zip(self._lazy_n, res)]
    self._lazy_n = []
    return out

  def run_unit(self, ps, ri, cpy, rng_seed, soa, p, rlen, cum_tlen, sample_name, worker_id=0, write_fastq2=True,
               rng='mitty'):
    """One work unit: sample templates, emit FASTQ.  Returns (n_templates, kept, bytes1, bytes2)."""
    return self.run_units([(ps, ri, cpy, rng_seed)], lambda a, b: soa, p, rlen, cum_tlen, sample_name, worker_id,
                          write_fastq2, rng)[0]

