"""Multi-GPU generate-reads: one process per GPU, torch.distributed over RCCL.

Work units (region, copy, pass) are independent given their rng_seed (reference readgenerate.py:149-154,
illumina.py:56-58), so the path shards without any data-path collective:

* every rank builds the reference's unit list (A6) itself, so seeds and `ps` do not depend on the GPU count;
* with at least 2 units per GPU the units are dealt out whole by LPT on region length;
* with fewer (chr1 = 4 units on 8 GPUs) every rank emits only its slice [m*r/W, m*(r+1)/W) of every unit's
  templates.  Each unit is sampled once, on rank u mod W, and its template arrays (17 B per template) are broadcast
  to the other ranks (RCCL over xGMI on device buffers; gloo on host arrays for the CPU tests); the cnt of a slice's
  first kept template comes from one all-reduce of the per-slice N-filter survivor counts (the only coupling between
  templates, an exclusive prefix);
* the output streams: every piece is measured first (mh_emit_measure: the measure pass alone, its templates kept
  resident under their own set id) and one all-reduce of the sizes places every piece in the files; then each piece
  is emitted, fetched and pwritten at its offset, and the arenas are recycled after it (readgenerate.py:233-253
  writes as it goes).  A '.gz' file's pieces are deflated on the device as they are emitted and held compressed
  (~4.5x smaller) until an all-reduce of the compressed sizes places them.  The files are byte-identical to the
  single-GPU run (= reference --threads 1) at any GPU count.

The collectives carry a few int64 per piece; no sequence data crosses xGMI for the FASTQ files.  Outputs must be
regular files (ranks write at offsets); FIFOs / process substitution need the single-GPU path.

With a BAM output (configs[4]: the god-aligner's perfect BAM of the generated reads), the coordinate order is cut
into one range per rank (range_splitters: the BED regions' bases in @SQ order, split evenly — templates start
uniformly over the regions, illumina.py:66-76), and no rank merges the others' records:

* as each piece is emitted, its rank turns it into BAM records on its GPU (mh_bam_add_output on the arenas) and
  partitions them by range (mh_bam_partition: packed per destination, each record with its global input index as a
  tie); one all-to-all per round of pieces (RCCL on device buffers under 'nccl', gloo on host arrays) moves every
  record to its range's rank, whose store (a second HIP context) imports it (mh_bam_import_tie);
* each rank sorts its range on its GPU (equal keys by tie: the one-rank store's input order) and deflates it into
  BGZF blocks cut where the one-rank file cuts them (every 0xff00 bytes of the whole sorted stream: a rank skips the
  bytes that complete the previous rank's last block and appends the head of the next ranks' ranges —
  mh_bam_write_part), into a part file of its own; an all-gather of the parts' sizes places them, and every rank
  copies its part into the BAM at its offset (rank 0's part starts with the header, the last ends with the EOF);
* the BAI: every rank's raw plan of its range (mh_bam_bai_runs: runs of one bin, first record per 16 kbp window) in
  virtual offsets of the final file, gathered to rank 0 and joined (runs cut at a range boundary are one run again)
  into the one-rank index.

The bounded store (mh_bam_set_capacity, `bam_capacity`) applies to every rank's range: records past it spill to host
memory (or, with `bam_spill_dir`, to unlinked temporary files, as `samtools sort -m` does), so a rank's memory
follows its range, not the job — the reference's workers' fragments, cat, `samtools sort -m 2G -@N` and
pysam.index (god_aligner.py:63-68,100-116).  The BAM and BAI equal the one-GPU god-aligner's over the same FASTQ,
byte for byte.

A process holds one HIP runtime: torch must load before libmitty_hip.so (mitty_amd._native does that itself when
WORLD_SIZE > 1), otherwise torch brings its own runtime and whichever of the two initialises second sees no GPU.
"""
import logging
import os
import time

import numpy as np

from mitty_amd.lib import fasta as mfasta
from mitty_amd.lib import vcfio

logger = logging.getLogger(__name__)


def lpt_assign(weights, world):
  """Longest-processing-time: items by decreasing weight (ties: lower index first) to the least-loaded rank
  (ties: lower rank).  Returns owner rank per item."""
  load = [0] * world
  owner = [0] * len(weights)
  for i in sorted(range(len(weights)), key=lambda i: (-weights[i], i)):
    r = min(range(world), key=lambda r: (load[r], r))
    owner[i] = r
    load[r] += weights[i]
  return owner


def plan_pieces(unit_weights, world, layout=None):
  """Pieces = (unit index, slice, n_slices, owner rank) in output order (unit, slice).
  layout: None = whole units by LPT when there are >= 2 units per rank, else slices; 'lpt' / 'slice' force one."""
  n = len(unit_weights)
  if layout == 'lpt' or (layout is None and (world <= 1 or n >= 2 * world)):
    owner = lpt_assign(unit_weights, max(world, 1))
    return [(u, 0, 1, owner[u]) for u in range(n)]
  return [(u, s, world, s) for u in range(n) for s in range(world)]


def slice_range(m, s, n_slices):
  return m * s // n_slices, m * (s + 1) // n_slices


def exclusive_bases(pieces, kept):
  """cnt base of each piece = templates kept by the earlier slices of the same unit."""
  base, acc, cur = [], 0, None
  for (u, s, _, _), k in zip(pieces, kept):
    if u != cur:
      cur, acc = u, 0
    base.append(acc)
    acc += k
  return base


def file_offsets(sizes):
  out, acc = [], 0
  for x in sizes:
    out.append(acc)
    acc += x
  return out, acc


def allreduce_i64(vals, group=None):
  """Sum an int64 vector over ranks (RCCL on GPU tensors under 'nccl', gloo on CPU tensors)."""
  import torch
  import torch.distributed as dist
  if not dist.is_available() or not dist.is_initialized():
    return [int(v) for v in vals]
  dev = 'cuda' if dist.get_backend(group) == 'nccl' else 'cpu'
  t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=dev)
  dist.all_reduce(t, group=group)
  return [int(v) for v in t.cpu().tolist()]


class DeviceBackend:
  """The per-rank device side: one Engine (HIP context) on this rank's GPU."""

  def __init__(self, device):
    from mitty_amd import _native
    from mitty_amd.engine import Engine
    self.eng = Engine(device)
    self._slots = {}   # template set id -> haplotype slot
    self._pin = _native.PinnedBuffer()

  def set_corruption(self, model, seed):
    import numpy as np
    self.eng.ctx.set_corruption(True, model['cum_bq_mat'], 10 ** (-np.arange(100) / 10), seed)

  def load_region(self, ri, region, seq):
    self.eng.load_region(ri, region, seq)

  def sample(self, units, soa_of, p, rlen, cum_tlen, rng, which=None, ids=None):
    """units: [(ps, ri, cpy, seed)]; the units k in `which` (all by default) are sampled into template set ids[k]
    (k by default).  Every unit's haplotype is built (its slices are emitted here).  Returns template counts (None
    where not sampled)."""
    from mitty_amd.engine import RNG_MODES
    ids = list(range(len(units))) if ids is None else list(ids)
    for k, (_, ri, cpy, _) in enumerate(units):
      self._slots[ids[k]] = self.eng.haplotype(ri, cpy, soa_of(ri, cpy))[0]
    which = list(range(len(units))) if which is None else list(which)
    out = [None] * len(units)
    if which:
      ns = self.eng.ctx.sample_units([ids[k] for k in which], [self._slots[ids[k]] for k in which],
                                     [units[k][3] for k in which], p, rlen, cum_tlen, RNG_MODES[rng])
      for k, n in zip(which, ns):
        out[k] = int(n)
    return out

  # the broadcast buffer of a template set of n templates: pos0 at 0, pos1 at 8n, fo0 at 16n (17 B per template)
  def pack_device(self, k, n, ptr):
    """Template set k into the device buffer at ptr (>= 17 n bytes); returns n."""
    return self.eng.ctx.templates_export(k, ptr + 16 * n, ptr, ptr + 8 * n, n)

  def unpack_device(self, k, n, rlen, ptr):
    self.eng.ctx.templates_import(k, n, rlen, ptr + 16 * n, ptr, ptr + 8 * n, on_device=True)

  def pack_host(self, k, n, a):
    """Template set k into the uint8 host array a (>= 17 n bytes)."""
    fo0, p0, p1 = self.eng.ctx.templates_export(k)
    assert len(fo0) == n
    a[:8 * n] = p0.view(np.uint8)
    a[8 * n:16 * n] = p1.view(np.uint8)
    a[16 * n:17 * n] = fo0.view(np.uint8)

  def unpack_host(self, k, n, rlen, a):
    self.eng.ctx.templates_import(k, n, rlen, a[16 * n:17 * n].view(np.int8), a[:8 * n].view(np.int64),
                                  a[8 * n:16 * n].view(np.int64))

  def share(self, k, n, src, rlen, group=None, into=None):
    """Template set k (n templates) from rank src to every rank: an RCCL broadcast of the device arrays under
    'nccl' (pos0 | pos1 | fo0 packed in one buffer, device-to-device copies on either side), host arrays under gloo.
    The receivers unpack into set k; `into` names another set the source also unpacks its broadcast buffer into
    (the whole round trip on one rank: the one-GPU test of the RCCL path)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    dst = k if rank != src else into
    if dist.get_backend(group) == 'nccl':
      buf = torch.empty(max(17 * n, 16), dtype=torch.uint8, device='cuda')
      if rank == src:
        self.pack_device(k, n, buf.data_ptr())   # (synchronous: the copies are done before the broadcast reads)
      dist.broadcast(buf, src, group=group)
      torch.cuda.current_stream().synchronize()
      if dst is not None:
        self.unpack_device(dst, n, rlen, buf.data_ptr())
      return
    buf = torch.empty(max(17 * n, 16), dtype=torch.uint8)
    if rank == src:
      self.pack_host(k, n, buf.numpy())
    dist.broadcast(buf, src, group=group)
    if dst is not None:
      self.unpack_host(dst, n, rlen, buf.numpy())

  def count_kept(self, k, t0, t1):
    self.eng.ctx.use_templates(k)
    return self.eng.ctx.count_kept(self._slots[k], t0, t1)

  def measure(self, k, stub, chrom, cpy, write2, unit_key, t_range, cnt_base):
    """-> (kept, bytes file 1, bytes file 2) that emit() with the same arguments writes (mh_emit_measure)."""
    ctx = self.eng.ctx
    ctx.use_templates(k)
    return ctx.emit_measure(self._slots[k], stub, chrom, cpy, write2, unit_key, t_range, cnt_base)

  def emit(self, k, stub, chrom, cpy, write2, unit_key, t_range, cnt_base):
    """-> (kept, (arena offset, length) for file 1, same for file 2)"""
    ctx = self.eng.ctx
    ctx.use_templates(k)
    u1, u2 = ctx.output_size()
    kept, b1, b2 = ctx.emit_reads(self._slots[k], stub, chrom, cpy, write2, unit_key, t_range, cnt_base)
    return kept, (u1, b1), (u2, b2)

  def fetch(self, r1, r2):
    return self.eng.ctx.fetch_output(r1[0], r1[1], r2[0], r2[1])

  def fetch_gz(self, f, r):
    """Arena range r = (offset, length) of file f as BGZF members deflated on the device (mh_output_bgzf_range)."""
    return self.eng.ctx.bgzf_range(f, r[0], r[1], self._pin)

  def reset_output(self):
    self.eng.ctx.reset_output()

  # ---- the BAM leg (configs[4]): each piece's records partitioned by coordinate range (this context's store
  # stages one piece at a time); this rank's range in a store of its own (a second context on the same GPU) ----
  def bam_begin(self, refs, capacity=0, spill_dir=None):
    from mitty_amd import _native
    names, lens = [r[0] for r in refs], [r[1] for r in refs]
    self.eng.ctx.bam_set_refs(names, lens)
    self.eng.ctx.bam_set_capacity(0)
    if getattr(self, 'rctx', None) is None:
      self.rctx = _native.Context(self.eng.device)
    self.rctx.bam_set_refs(names, lens)
    self.rctx.bam_set_capacity(capacity)
    if spill_dir is not None:
      self.rctx.bam_set_spill_dir(spill_dir)

  def bam_partition(self, splitters, tie_base):
    """The arenas' records (this piece) by range -> (segment offsets, records, record bytes) per destination."""
    ctx = self.eng.ctx
    ctx.bam_reset()
    ctx.bam_add_output()
    return ctx.bam_partition(splitters, tie_base)

  def bam_partition_into(self, t):
    """The packed segments into torch tensor t (host or device)."""
    self.eng.ctx.bam_partition_fetch(t.data_ptr(), t.numel())

  def bam_import_segment(self, t, off, n, nb):
    self.rctx.bam_import_tie(n, nb, t.data_ptr() + off)

  def bam_range(self):
    """(records, bytes) of this rank's range."""
    return self.rctx.bam_records()

  def bam_head(self, n):
    return self.rctx.bam_sorted_head(n)

  def bam_write_part(self, path, header_text, skip, tail, eof):
    return self.rctx.bam_write_part(path, header_text, skip, tail, eof)

  def bam_bai_runs(self, n_refs):
    return self.rctx.bam_bai_runs(n_refs)

  def close(self):
    if getattr(self, 'rctx', None) is not None:
      self.rctx.close()
      self.rctx = None
    self.eng.close()


def generate_reads_distributed(fasta_fname, vcf_fname, sample_name, bed_fname, read_module, model, coverage,
                               fastq1_fname, fastq2_fname, seed=7, rng='mitty', corrupt_seed=None, backend=None,
                               group=None, max_batch_draws=200_000_000, layout=None, bam_fname=None,
                               bam_header_text=None, bam_refs=None, bam_capacity=0, bam_spill_dir=None):
  """process_multi_threaded (readgenerate.py:76-126) over the ranks of the default process group.

  `backend` defaults to DeviceBackend(LOCAL_RANK); tests pass a host stand-in to exercise the orchestration with
  the gloo backend on CPU.  Returns this rank's stats plus the job totals.
  bam_fname: also the god-aligner's BAM (+ .bai) of the reads, header bam_header_text, @SQ bam_refs [(name, length)]
  (god_aligner.construct_header from the FASTA's .ann); bam_capacity: each rank's range store's record bytes in HBM
  before a spill; bam_spill_dir: spill to unlinked temporary files there instead of host memory.
  """
  import torch.distributed as dist
  from mitty_amd.simulation.readgenerate import get_data_for_workers
  t0 = time.time()
  rank = dist.get_rank(group) if dist.is_initialized() else 0
  world = dist.get_world_size(group) if dist.is_initialized() else 1
  read_model = read_module.read_model_params(model, coverage)
  vdf = vcfio.load_variants_soa(vcf_fname, sample_name, bed_fname)
  units = [(ps, w['region_idx'], w['region_cpy'], w['rng_seed'])
           for ps, w in enumerate(get_data_for_workers(read_model, vdf, seed))]
  weights = [vdf[ri]['region'][2] - vdf[ri]['region'][1] for _, ri, _, _ in units]
  pieces = plan_pieces(weights, world, layout)
  mine = [i for i, pc in enumerate(pieces) if pc[3] == rank]
  my_units = sorted({pieces[i][0] for i in mine})
  write2 = fastq2_fname is not None

  if backend is None:
    backend = DeviceBackend(int(os.environ.get('LOCAL_RANK', '0')))
  if corrupt_seed is not None:
    backend.set_corruption(model, corrupt_seed)
  regions = sorted({units[u][1] for u in my_units})
  if regions:
    seqs = mfasta.read_fasta(fasta_fname, names={vdf[ri]['region'][0] for ri in regions})
    for ri in regions:
      chrom, s0, e = vdf[ri]['region']
      backend.load_region(ri, vdf[ri]['region'], mfasta.fetch(seqs, chrom, s0, e))

  # batches of this rank's units; in the sliced layout every rank holds every unit, so the batches (and the
  # per-batch all-reduce of slice survivor counts) line up across ranks
  sliced = any(pc[2] > 1 for pc in pieces)
  batches, cur, draws = [], [], 0
  for u in my_units:
    ri = units[u][1]
    cur.append(u)
    draws += int(weights[u] * read_model['p'] * 1.2)
    if draws >= max_batch_draws or u == my_units[-1]:
      batches.append(cur)
      cur, draws = [], 0

  # ---- phase A: every piece sampled (its templates resident under its own set id) and measured ----------------
  stats = {'units': len(units), 'pieces': len(mine), 'templates': 0, 'kept': 0}
  soa_of = lambda r, c: vdf[r]['copies'][c]
  fnames = [fastq1_fname] + ([fastq2_fname] if write2 else [])
  gz = [fn.endswith('.gz') for fn in fnames] + [False]
  plan = {}   # piece index -> (template set id, stub, chrom, cpy, unit seed, t_range, cnt base)
  sizes = {}  # piece index -> (kept, bytes1, bytes2)
  for batch in batches:
    ids = list(batch)   # the unit index is the template set id: every set stays resident until phase B
    if sliced and world > 1:
      # each unit sampled once, on rank u mod W; its template count all-reduced, its arrays broadcast
      owner = [u % world for u in batch]
      got = backend.sample([units[u] for u in batch], soa_of, read_model['p'], read_model['rlen'],
                           read_model['cum_tlen'], rng, which=[k for k, o in enumerate(owner) if o == rank], ids=ids)
      ns = allreduce_i64([got[k] if o == rank else 0 for k, o in enumerate(owner)], group)
      for k, o in enumerate(owner):
        backend.share(ids[k], ns[k], o, read_model['rlen'], group)
      stats['sampled'] = stats.get('sampled', 0) + sum(1 for o in owner if o == rank)
    else:
      ns = backend.sample([units[u] for u in batch], soa_of, read_model['p'], read_model['rlen'],
                          read_model['cum_tlen'], rng, ids=ids)
    k_of = {u: k for k, u in enumerate(batch)}
    bases = {}
    if sliced:
      local = [0] * len(pieces)
      for i in mine:
        u, s, S, _ = pieces[i]
        if u in k_of:
          local[i] = backend.count_kept(u, *slice_range(ns[k_of[u]], s, S))
      kept_all = allreduce_i64(local, group)
      bases = dict(enumerate(exclusive_bases(pieces, kept_all)))
    for i in mine:
      u, s, S, _ = pieces[i]
      if u not in k_of:
        continue
      ps, ri, cpy, useed = units[u]
      rng_range = slice_range(ns[k_of[u]], s, S) if S > 1 else None
      plan[i] = (u, '{}:{}:{}'.format(sample_name, 0, ps), vdf[ri]['region'][0], cpy, useed, rng_range, bases.get(i, 0))
      if not all(gz[:len(fnames)]):   # plain files are placed from these sizes before anything is written
        sizes[i] = backend.measure(u, plan[i][1], plan[i][2], cpy, write2, useed, rng_range, bases.get(i, 0))
      stats['templates'] += (rng_range[1] - rng_range[0]) if S > 1 else ns[k_of[u]]

  # plain files: every piece's offset from one all-reduce of the measured sizes; rank 0 sizes the files.  Every rank
  # joins (a flag all ranks share, not `sizes`: a rank that owns no pieces contributes zeros)
  off = [None, None]
  if not all(gz[:len(fnames)]):
    sz = [0] * (2 * len(pieces))
    for i, (_, b1, b2) in sizes.items():
      sz[2 * i], sz[2 * i + 1] = b1, b2
    sz = allreduce_i64(sz, group)
    for f in range(len(fnames)):
      if not gz[f]:
        off[f], total = file_offsets(sz[f:2 * len(pieces):2])
        if rank == 0:
          with open(fnames[f], 'wb') as fp:
            fp.truncate(total)
    if world > 1:
      dist.barrier(group)

  # ---- phase B: each piece emitted, then written at its offset (plain) or deflated on the device and held (gz);
  # the arenas are recycled after every piece.  With a BAM, the pieces go in rounds (the k-th piece of every rank),
  # each round closed by one all-to-all of the pieces' records to their coordinate ranges' ranks ------------------
  fds = [os.open(fn, os.O_WRONLY) if not gz[f] else None for f, fn in enumerate(fnames)]
  held = {}   # piece index -> compressed bytes per gz file
  raw = [0, 0]
  order = sorted(plan)
  rounds = len(order)
  splitters = None
  if bam_fname is not None:
    rounds = max(sum(1 for pc in pieces if pc[3] == r) for r in range(world)) if pieces else 0
    splitters = range_splitters([vdf[ri]['region'] for ri in range(len(vdf))], bam_refs, world)
    backend.bam_begin(bam_refs, bam_capacity, bam_spill_dir)
    stats['bam_rounds'] = rounds
  try:
    for r in range(rounds):
      i = order[r] if r < len(order) else None
      if i is None:   # (a rank with fewer pieces: an empty contribution to the round's exchange)
        _bam_exchange(backend, None, world, group, stats)
        continue
      k, stub, chrom, cpy, useed, rng_range, base = plan[i]
      backend.reset_output()
      kept, r1, r2 = backend.emit(k, stub, chrom, cpy, write2, useed, rng_range, base)
      stats['kept'] += kept
      raw[0] += r1[1]
      raw[1] += r2[1] if write2 else 0
      if i in sizes and (kept, r1[1], r2[1] if write2 else 0) != tuple(sizes[i]):
        raise RuntimeError('piece {}: emitted {} differs from its measured sizes {}'.format(
            i, (kept, r1[1], r2[1]), sizes[i]))
      rs = (r1, r2)
      plain = [f for f in range(len(fnames)) if not gz[f]]
      if plain:
        data = backend.fetch(r1 if 0 in plain else (0, 0), r2 if 1 in plain else (0, 0))
        for f in plain:
          _pwrite_all(fds[f], data[f], off[f][i])
      held[i] = [backend.fetch_gz(f, rs[f]) if gz[f] else None for f in range(len(fnames))]
      if bam_fname is not None:   # the piece's records to their ranges (tie: piece index, record index)
        _bam_exchange(backend, backend.bam_partition(splitters, i << 32), world, group, stats)
  finally:
    for fd in fds:
      if fd is not None:
        os.close(fd)

  # gz files: offsets from the compressed sizes, then the held members written (rank 0 adds the EOF marker)
  if any(gz[:len(fnames)]):
    zs = [0] * (2 * len(pieces))
    for i, h in held.items():
      for f in range(len(fnames)):
        if gz[f]:
          zs[2 * i + f] = len(h[f])
    zs = allreduce_i64(zs, group)
    for f in range(len(fnames)):
      if not gz[f]:
        continue
      zoff, ztotal = file_offsets(zs[f:2 * len(pieces):2])
      if rank == 0:
        from mitty_amd import _native
        with open(fnames[f], 'wb') as fp:
          fp.truncate(ztotal)
          fp.seek(ztotal)
          fp.write(_native.bgzf_eof())
      if world > 1:
        dist.barrier(group)
      fd = os.open(fnames[f], os.O_WRONLY)
      try:
        for i, h in held.items():
          _pwrite_all(fd, h[f], zoff[i])
      finally:
        os.close(fd)
  held.clear()
  if bam_fname is not None:
    stats['bam_records'] = _bam_write_ranges(backend, rank, world, group, bam_fname, bam_header_text, bam_refs)
  tot = allreduce_i64([stats['templates'], stats['kept']] + raw, group)
  if world > 1:
    dist.barrier(group)
  stats.update({'job_templates': tot[0], 'job_kept': tot[1], 'bytes1': tot[2], 'bytes2': tot[3] if write2 else 0,
                'seconds': time.time() - t0, 'rank': rank, 'world': world})
  return stats


BGZF_BLOCK = 0xff00   # uncompressed bytes per BGZF block (htslib's BGZF_BLOCK_SIZE; mh_bgzf.h)


def sort_key(tid, pos0):
  """The god-aligner store's coordinate key of a record at (tid, 0-based pos) on the forward strand
  (samtools sort's order: tid, pos + 1, is_reverse)."""
  return (int(tid) << 33) | ((int(pos0) + 1) << 1)


def range_splitters(regions, refs, world):
  """world - 1 ascending sort keys that cut the coordinate order into `world` ranges of about equal bases of the BED
  regions (templates start uniformly over the regions: illumina.py:66-76, geometric gaps); range d holds the keys
  k with splitters[d - 1] <= k < splitters[d].  regions: [(chrom, start0, end)]; refs: the @SQ [(name, length)]."""
  tid = {name: t for t, (name, _) in enumerate(refs)}
  segs = sorted((tid[c], s0, e) for c, s0, e in regions if c in tid and e > s0)
  total = sum(e - s0 for _, s0, e in segs)
  out = []
  for d in range(1, world):
    want, acc = total * d // world, 0
    key = sort_key(len(refs), 0)   # (past every record: an empty range)
    for t, s0, e in segs:
      if acc + (e - s0) > want:
        key = sort_key(t, s0 + (want - acc))
        break
      acc += e - s0
    out.append(max(key, out[-1]) if out else key)
  return out


def _bam_exchange(backend, part, world, group, stats):
  """One round: every rank's packed segments (backend.bam_partition: offsets, records and record bytes per
  destination; None = nothing this round) to their destinations (all-to-all, RCCL on device buffers under 'nccl',
  gloo on host tensors), imported into the receiving ranks' range stores."""
  import torch
  from mitty_amd import _native
  if part is None:   # an empty segment per destination (its layout: the one record offset, 0)
    off, seg_n, seg_b = 8 * np.arange(world + 1, dtype=np.int64), np.zeros(world, np.int64), np.zeros(world, np.int64)
  else:
    off, seg_n, seg_b = part
  import torch.distributed as dist
  if not (dist.is_available() and dist.is_initialized()):   # one process, no group: straight into the range store
    t = torch.empty(max(int(off[-1]), 8), dtype=torch.uint8)
    if part is not None:
      backend.bam_partition_into(t)
      backend.bam_import_segment(t, 0, int(seg_n[0]), int(seg_b[0]))
    stats['bam_sent'] = stats.get('bam_sent', 0) + int(seg_n.sum())
    return
  dev = 'cuda' if dist.get_backend(group) == 'nccl' else 'cpu'
  # sizes first: (records, record bytes) per destination, all-to-all
  sz = torch.tensor(np.stack([seg_n, seg_b], 1).reshape(-1), dtype=torch.int64, device=dev)
  rs = torch.empty(2 * world, dtype=torch.int64, device=dev)
  dist.all_to_all_single(rs, sz, group=group)
  rs = rs.cpu().numpy().reshape(world, 2)
  tot_in = [int(_native.bam_part_layout(int(n), int(nb))[4]) for n, nb in rs]
  tot_out = [int(off[d + 1] - off[d]) for d in range(world)]
  send = (torch.empty if part is not None else torch.zeros)(max(int(off[-1]), 8), dtype=torch.uint8, device=dev)
  if part is not None and int(off[-1]) > 0:
    backend.bam_partition_into(send)
  recv = torch.empty(max(sum(tot_in), 8), dtype=torch.uint8, device=dev)
  dist.all_to_all_single(recv[:sum(tot_in)], send[:int(off[-1])], tot_in, tot_out, group=group)
  if dev == 'cuda':
    torch.cuda.current_stream().synchronize()
  o = 0
  for s in range(world):
    n, nb = int(rs[s][0]), int(rs[s][1])
    if n:
      backend.bam_import_segment(recv, o, n, nb)
    o += tot_in[s]
  stats['bam_sent'] = stats.get('bam_sent', 0) + int(seg_n.sum())
  stats['bam_received'] = stats.get('bam_received', 0) + int(rs[:, 0].sum())


def _allgather_i64(vals, world, group):
  """Every rank's int64 vector (same length), as a [world, len] array (an all-reduce of a zero-padded slot each)."""
  import torch.distributed as dist
  vals = [int(v) for v in vals]
  if world == 1:
    return np.array([vals], np.int64)
  rank = dist.get_rank(group)
  buf = [0] * (world * len(vals))
  buf[rank * len(vals):(rank + 1) * len(vals)] = vals
  return np.array(allreduce_i64(buf, group), np.int64).reshape(world, len(vals))


def _allgather_bytes(data, cap, world, group):
  """Every rank's bytes (at most cap), as a list."""
  import torch
  import torch.distributed as dist
  if world == 1:
    return [bytes(data)]
  dev = 'cuda' if dist.get_backend(group) == 'nccl' else 'cpu'
  t = torch.zeros(cap + 8, dtype=torch.uint8)
  t[:8] = torch.from_numpy(np.array([len(data)], np.int64).view(np.uint8))
  if len(data):
    t[8:8 + len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy())
  t = t.to(dev)
  out = [torch.empty_like(t) for _ in range(world)]
  dist.all_gather(out, t, group=group)
  res = []
  for x in out:
    x = x.cpu().numpy()
    n = int(x[:8].view(np.int64)[0])
    res.append(x[8:8 + n].tobytes())
  return res


def _bam_write_ranges(backend, rank, world, group, bam_fname, header_text, refs):
  """Each rank's range sorted and deflated where the one-rank file cuts its blocks, the parts placed by an
  all-gather of their sizes and copied into the BAM; the BAI joined on rank 0 from every rank's raw plan.  Returns
  the BAM's record count."""
  n_rec, nbytes = backend.bam_range()
  tab = _allgather_i64([n_rec, nbytes], world, group)
  U = np.concatenate([[0], np.cumsum(tab[:, 1])])   # each range's first byte in the whole sorted stream
  total = int(U[-1])
  B = BGZF_BLOCK
  skip = [min(int(tab[r, 1]), (-int(U[r])) % B) for r in range(world)]
  heads = _allgather_bytes(backend.bam_head(min(B, nbytes)), B, world, group)
  # the tail: the next ranges' first bytes up to the end of this rank's last block (or of the stream)
  tail = b''
  own = nbytes - skip[rank]
  if own > 0:
    nb_local = (own + B - 1) // B
    end = min(total, int(U[rank]) + skip[rank] + nb_local * B)
    need, r = end - int(U[rank + 1]), rank + 1
    while need > 0 and r < world:
      take = heads[r][:need]
      tail += take
      need -= len(take)
      r += 1
    assert need <= 0, 'BAM ranges: the next ranges\' heads do not complete the last block'
  part = '{}.part{}'.format(bam_fname, rank)
  nblk, data_pos, fbytes, boff = backend.bam_write_part(part, header_text if rank == 0 else None, skip[rank], tail,
                                                        rank == world - 1)
  z = int(boff[-1]) if len(boff) else 0
  lastz = int(boff[-1] - boff[-2]) if nblk > 0 else 0
  pt = _allgather_i64([fbytes, data_pos, nblk, z, lastz], world, group)
  part_off = np.concatenate([[0], np.cumsum(pt[:, 0])])
  if world > 1:
    import torch.distributed as dist
    if rank == 0:
      with open(bam_fname, 'wb') as fp:
        fp.truncate(int(part_off[-1]))
    dist.barrier(group)
  elif rank == 0:
    open(bam_fname, 'wb').close()
  fd_in, fd_out = os.open(part, os.O_RDONLY), os.open(bam_fname, os.O_WRONLY)
  try:
    o, n = int(part_off[rank]), int(fbytes)
    src = 0
    while src < n:
      m = os.copy_file_range(fd_in, fd_out, n - src, src, o + src)
      if m <= 0:
        raise OSError('copy_file_range: no progress copying {} into {}'.format(part, bam_fname))
      src += m
  finally:
    os.close(fd_in)
    os.close(fd_out)
    os.remove(part)
  # the BAI: this range's raw plan in the final file's virtual offsets
  b0 = [(int(U[r]) + skip[r]) // B for r in range(world)]

  def coff(b):   # the file offset of (whole-stream) block b
    lb = b - b0[rank]
    if 0 <= lb < nblk:
      return int(part_off[rank] + data_pos + boff[lb])
    for r in range(world):
      if pt[r, 2] > 0 and b == b0[r]:
        return int(part_off[r] + pt[r, 1])
      if pt[r, 2] > 0 and b == b0[r] + pt[r, 2] - 1:
        return int(part_off[r] + pt[r, 1] + pt[r, 3] - pt[r, 4])
    if b * B >= total:   # the end of the stream: the EOF block's offset
      return int(part_off[world - 1] + pt[world - 1, 1] + pt[world - 1, 3])
    raise RuntimeError('BAI: block {} is not a block this range can reference'.format(b))

  def voff(u):
    b = u // B
    return (coff(b) << 16) | (u - b * B)

  runs, win, rnwin = backend.bam_bai_runs(len(refs))
  base = int(U[rank])
  plan = {'runs': [(int(t) >> 32, int(t) & 0xffffffff, int(a) + base, int(e) + base, voff(int(a) + base),
                    voff(int(e) + base), int(c)) for t, a, e, c in runs],
          'win': {}, 'nwin': [int(x) for x in rnwin]}
  wo = np.concatenate([[0], np.cumsum([(ln >> 14) + 1 for _, ln in refs])])
  for t in range(len(refs)):
    ws = win[wo[t]:wo[t] + int(rnwin[t])]
    plan['win'][t] = [(w, voff(int(x) + base)) for w, x in enumerate(ws) if x >= 0]
  plans = _gather_to0(plan, rank, world, group)
  if rank == 0:
    with open(bam_fname + '.bai', 'wb') as fp:
      fp.write(bai_join(plans, len(refs)))
  if world > 1:
    import torch.distributed as dist
    dist.barrier(group)
  return int(tab[:, 0].sum())


def _gather_to0(obj, rank, world, group):
  if world == 1:
    return [obj]
  import torch.distributed as dist
  out = [None] * world if rank == 0 else None
  dist.gather_object(obj, out, dst=0, group=group)
  return out


def bai_join(plans, n_refs):
  """The BAI (SAM spec §5.2, as mh_bgzf.cpp bai_emit writes it) from the ranks' plans in range order.  A plan:
  'runs' [(tid, bin, first data offset, end offset, first voffset, end voffset, records)] in record order, 'win'
  {tid: [(window, voffset of its first record)]}, 'nwin' [window count per tid].  Runs of one bin that meet at a
  range boundary are one run (as the one-rank plan finds them); each reference's runs are then ordered by bin
  (stable); a window's first record is the first range's that has one."""
  import struct
  out = bytearray(b'BAI\x01')
  out += struct.pack('<i', n_refs)
  for t in range(n_refs):
    runs = []   # [bin, ub, ue, vb, ve, n]
    for p in plans:
      for (tid, b, ub, ue, vb, ve, c) in p['runs']:
        if tid != t:
          continue
        if runs and runs[-1][0] == b and runs[-1][2] == ub:
          runs[-1][2], runs[-1][4], runs[-1][5] = ue, ve, runs[-1][5] + c
        else:
          runs.append([b, ub, ue, vb, ve, c])
    if not runs:
      out += struct.pack('<ii', 0, 0)
      continue
    n = sum(r[5] for r in runs)
    vi, vj = runs[0][3], runs[-1][4]
    ordered = sorted(runs, key=lambda r: r[0])   # (stable)
    bins = []
    for r in ordered:
      if bins and bins[-1][0] == r[0]:
        bins[-1][1].append((r[3], r[4]))
      else:
        bins.append((r[0], [(r[3], r[4])]))
    out += struct.pack('<i', len(bins) + 1)
    for b, chunks in bins:
      out += struct.pack('<Ii', b, len(chunks))
      for vb, ve in chunks:
        out += struct.pack('<QQ', vb, ve)
    out += struct.pack('<IiQQQQ', 37450, 2, vi, vj, n, 0)
    nw = max(p['nwin'][t] for p in plans)
    lin = [-1] * nw
    for p in plans:
      for w, v in p['win'].get(t, []):
        if lin[w] < 0:
          lin[w] = v
    nxt = vj
    for w in range(nw - 1, -1, -1):
      if lin[w] >= 0:
        nxt = lin[w]
      lin[w] = nxt
    out += struct.pack('<i', nw)
    out += struct.pack('<{}Q'.format(nw), *lin)
  out += struct.pack('<Q', 0)
  return bytes(out)


def _pwrite_all(fd, data, off):
  mv = memoryview(data)
  while len(mv):
    n = os.pwrite(fd, mv, off)
    mv, off = mv[n:], off + n
