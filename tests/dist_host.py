"""Host stand-in for DeviceBackend (test infrastructure): per-unit FASTQ from the CPU oracle, so the multi-rank
orchestration of mitty_amd.distributed (plan, slice counts, cnt bases, file offsets, pwrite) runs with gloo on CPU.
Every oracle record is a kept template, and the stand-in renumbers cnt from the base it is given, so a wrong
cnt_base or offset shows up as a byte difference against the single-process output."""
from oracle import oracle as O


class OracleBackend:
  def __init__(self):
    self.regions = {}
    self.arena = [bytearray(), bytearray()]

  def set_corruption(self, model, seed):
    raise NotImplementedError

  def load_region(self, ri, region, seq):
    self.regions[ri] = (region, seq)

  def sample(self, units, soa_of, p, rlen, cum_tlen, rng, which=None, ids=None):
    ids = list(range(len(units))) if ids is None else list(ids)
    if not hasattr(self, 'recs'):
      self.recs = {}
    self.sampled = []
    out = []
    for k, (ps, ri, cpy, seed) in enumerate(units):
      if which is not None and k not in which:
        self.recs.pop(ids[k], None)
        out.append(None)
        continue
      (chrom, s0, _), seq = self.regions[ri]
      _, b1, b2 = O.generate_unit_soa(seq, s0, soa_of(ri, cpy), p, rlen, cum_tlen, seed, 'X:0:0', chrom, cpy)
      self.recs[ids[k]] = (_records(b1), _records(b2))
      self.sampled.append(k)
      out.append(len(self.recs[ids[k]][0]))
    return out

  def share(self, k, n, src, rlen, group=None, into=None):
    """The unit's records (the stand-in's 'templates') from rank src, as DeviceBackend.share sends arrays."""
    import torch.distributed as dist
    obj = [self.recs.get(k) if dist.get_rank(group) == src else None]
    dist.broadcast_object_list(obj, src, group=group)
    assert obj[0] is not None and len(obj[0][0]) == n
    self.recs[k] = obj[0]

  def count_kept(self, k, t0, t1):
    return t1 - t0

  def _data(self, k, stub, write2, t_range, cnt_base):
    r1, r2 = self.recs[k]
    t0, t1 = t_range if t_range is not None else (0, len(r1))
    out = []
    for f, recs in enumerate((r1, r2)):
      if f == 1 and not write2:
        out.append(b'')
        continue
      out.append(b''.join(b'@' + stub.encode() + b':' + str(cnt_base + j + 1).encode() + b'|' + recs[t0 + j]
                         for j in range(t1 - t0)))
    return t1 - t0, out

  def measure(self, k, stub, chrom, cpy, write2, unit_key, t_range, cnt_base):
    kept, (d1, d2) = self._data(k, stub, write2, t_range, cnt_base)
    return kept, len(d1), len(d2)

  def emit(self, k, stub, chrom, cpy, write2, unit_key, t_range, cnt_base):
    kept, datas = self._data(k, stub, write2, t_range, cnt_base)
    out = []
    for f, data in enumerate(datas):
      out.append((len(self.arena[f]), len(data)))
      self.arena[f] += data
    return kept, out[0], out[1]

  def fetch(self, r1, r2):
    return bytes(self.arena[0][r1[0]:r1[0] + r1[1]]), bytes(self.arena[1][r2[0]:r2[0] + r2[1]])

  def fetch_gz(self, f, r):
    from mitty_amd import _native
    return _native.bgzf_compress(bytes(self.arena[f][r[0]:r[0] + r[1]])) if r[1] else b''

  def reset_output(self):
    self.arena = [bytearray(), bytearray()]

  def close(self):
    pass


  # ---- the BAM leg (DeviceBackend.bam_*): records from oracle/god.py, packed as mh_bam_export packs them ----------
  def bam_piece(self, refs):
    import numpy as np
    from oracle import god
    from mitty_amd import _native
    ref_dict = {name: k for k, (name, _) in enumerate(refs)}
    recs = god.god_records(bytes(self.arena[0]), bytes(self.arena[1]) if self.arena[1] else None, ref_dict)
    enc = [god.encode(r) for r in recs]
    n, nb = len(enc), sum(len(e) for e in enc)
    o_roff, o_key, o_info, total = _native.bam_piece_layout(n, nb)
    buf = np.zeros(max(total, 8), np.uint8)
    buf[:nb] = np.frombuffer(b''.join(enc), np.uint8)
    buf[o_roff:o_key].view(np.int64)[:] = np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64)
    buf[o_key:o_info].view(np.uint64)[:] = [r['reference_id'] << 33 | (r['pos'] + 1) << 1 | int(r['is_reverse'])
                                            for r in recs]
    buf[o_info:total].view(np.int32)[:] = np.array(
        [[r['reference_id'], r['pos'], god.end_pos(r), god.reg2bin(r['pos'], god.end_pos(r))] for r in recs],
        np.int32).reshape(-1) if n else []
    return n, nb, buf

  def bam_begin(self, refs, capacity=0):
    self.bam = []   # (key, import order, record bytes)

  def bam_import(self, n, nb, ptr):
    import ctypes
    import numpy as np
    from mitty_amd import _native
    o_roff, o_key, _, total = _native.bam_piece_layout(n, nb)
    buf = np.frombuffer(ctypes.string_at(ptr, total), np.uint8)
    roff = buf[o_roff:o_key].view(np.int64)
    keys = buf[o_key:o_key + 8 * n].view(np.uint64)
    for k in range(n):
      self.bam.append((int(keys[k]), len(self.bam), bytes(buf[roff[k] - roff[0]:roff[k + 1] - roff[0]])))

  def bam_write(self, path, header_text, bai=True):
    """The sorted record stream, uncompressed (the stand-in checks the order, not the BGZF framing)."""
    with open(path, 'wb') as fp:
      for _, _, rec in sorted(self.bam, key=lambda x: (x[0], x[1])):
        fp.write(rec)


def _records(b):
  """FASTQ bytes -> records with the '@{stub}:{cnt}|' head stripped."""
  lines = b.split(b'\n')
  return [lines[i].split(b'|', 1)[1] + b'\n' + b'\n'.join(lines[i + 1:i + 4]) + b'\n'
          for i in range(0, len(lines) - 1, 4)]

