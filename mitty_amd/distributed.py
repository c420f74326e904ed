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

With a BAM output (configs[4]: the god-aligner's perfect BAM of the generated reads), every rank also turns each of
its pieces into BAM records on its own GPU as the piece is emitted (parse, encode, keys: mh_bam_add_output on the
arenas), and rank 0's store takes the pieces in piece order (RCCL point-to-point on device buffers; gloo on host
arrays), sorts the keys once and writes the BAM and BAI — the reference's pysam.cat of the workers' fragments before
one sort (god_aligner.py:63-68,100-108).  The BAM equals the one-GPU god-aligner's over the same FASTQ, byte for byte.

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

  # ---- the BAM leg: per piece the records of the arenas, packed (_native.bam_piece_layout); rank 0's store ----
  def bam_piece(self, refs):
    ctx = self.eng.ctx
    ctx.bam_set_refs([r[0] for r in refs], [r[1] for r in refs])
    ctx.bam_add_output()
    n, nb = ctx.bam_records()
    return n, nb, ctx.bam_export(0, n, nb)

  def bam_begin(self, refs, capacity=0):
    ctx = self.eng.ctx
    ctx.bam_set_refs([r[0] for r in refs], [r[1] for r in refs])
    ctx.bam_set_capacity(capacity)

  def bam_import(self, n, nb, ptr):
    self.eng.ctx.bam_import(n, nb, ptr)

  def bam_write(self, path, header_text, bai=True):
    return self.eng.ctx.bam_write_gpu(path, header_text, bai_path=path + '.bai' if bai else None)

  def close(self):
    self.eng.close()


def generate_reads_distributed(fasta_fname, vcf_fname, sample_name, bed_fname, read_module, model, coverage,
                               fastq1_fname, fastq2_fname, seed=7, rng='mitty', corrupt_seed=None, backend=None,
                               group=None, max_batch_draws=200_000_000, layout=None, bam_fname=None,
                               bam_header_text=None, bam_refs=None, bam_capacity=0):
  """process_multi_threaded (readgenerate.py:76-126) over the ranks of the default process group.

  `backend` defaults to DeviceBackend(LOCAL_RANK); tests pass a host stand-in to exercise the orchestration with
  the gloo backend on CPU.  Returns this rank's stats plus the job totals.
  bam_fname: also the god-aligner's BAM (+ .bai) of the reads, header bam_header_text, @SQ bam_refs [(name, length)]
  (god_aligner.construct_header from the FASTA's .ann); bam_capacity: rank 0's record bytes in HBM before a spill.
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
  # the arenas are recycled after every piece -------------------------------------------------------------------
  fds = [os.open(fn, os.O_WRONLY) if not gz[f] else None for f, fn in enumerate(fnames)]
  held = {}   # piece index -> compressed bytes per gz file
  bam_held = {}   # piece index -> (records, record bytes, packed piece)
  raw = [0, 0]
  try:
    for i in sorted(plan):
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
      if bam_fname is not None:
        bam_held[i] = backend.bam_piece(bam_refs)
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
    stats['bam_records'] = _bam_merge(backend, pieces, bam_held, rank, world, group, bam_fname, bam_header_text,
                                      bam_refs, bam_capacity)
  tot = allreduce_i64([stats['templates'], stats['kept']] + raw, group)
  if world > 1:
    dist.barrier(group)
  stats.update({'job_templates': tot[0], 'job_kept': tot[1], 'bytes1': tot[2], 'bytes2': tot[3] if write2 else 0,
                'seconds': time.time() - t0, 'rank': rank, 'world': world})
  return stats


def _bam_merge(backend, pieces, bam_held, rank, world, group, bam_fname, header_text, refs, capacity):
  """Rank 0's store takes every piece's records in piece order (its own from memory, the others' over the process
  group: point-to-point, RCCL on device buffers under 'nccl'), then sorts and writes the BAM + BAI once.  The ranks
  hold their packed pieces until then.  Returns the BAM's record count on rank 0 (0 elsewhere)."""
  import torch
  from mitty_amd import _native
  sz = [0] * (2 * len(pieces))
  for i, (n, nb, _) in bam_held.items():
    sz[2 * i], sz[2 * i + 1] = n, nb
  sz = allreduce_i64(sz, group)
  dev = None
  if world > 1:
    import torch.distributed as dist
    dev = 'cuda' if dist.get_backend(group) == 'nccl' else 'cpu'
  if rank == 0:
    backend.bam_begin(refs, capacity)
  total = 0
  for i in range(len(pieces)):
    n, nb = sz[2 * i], sz[2 * i + 1]
    if n == 0:
      continue
    owner = pieces[i][3]
    size = _native.bam_piece_layout(n, nb)[3]
    if owner == rank:
      buf = bam_held.pop(i)[2]
      if rank == 0:
        backend.bam_import(n, nb, buf.ctypes.data)
      else:
        t = torch.from_numpy(buf[:size])
        dist.send(t.to(dev) if dev == 'cuda' else t, 0, group=group)
    elif rank == 0:
      t = torch.empty(size, dtype=torch.uint8, device=dev)
      dist.recv(t, owner, group=group)
      if dev == 'cuda':
        torch.cuda.current_stream().synchronize()
      backend.bam_import(n, nb, t.data_ptr())
    total += n
  if rank == 0:
    backend.bam_write(bam_fname, header_text)
  if world > 1:
    dist.barrier(group)
  return total if rank == 0 else 0


def _pwrite_all(fd, data, off):
  mv = memoryview(data)
  while len(mv):
    n = os.pwrite(fd, mv, off)
    mv, off = mv[n:], off + n
