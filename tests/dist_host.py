"""Host stand-in for DeviceBackend (test infrastructure): per-unit FASTQ from the CPU oracle, so the multi-rank
orchestration of mitty_amd.distributed (plan, slice counts, cnt bases, file offsets, pwrite) runs with gloo on CPU.
Every oracle record is a kept template, and the stand-in renumbers cnt from the base it is given, so a wrong
cnt_base or offset shows up as a byte difference against the single-process output."""
import numpy as np

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


  # ---- the BAM leg (DeviceBackend.bam_*): records from oracle/god.py, partitioned and packed as mh_bam_partition
  # packs them; the range store sorted by (key, tie); parts as host BGZF (zlib) cut every 0xff00 bytes ----------
  def bam_begin(self, refs, capacity=0, spill_dir=None):
    self.refs = refs
    self.bam = []   # the range store: (key, tie, record bytes, BAI info)

  def bam_partition(self, splitters, tie_base):
    import bisect
    import numpy as np
    from oracle import god
    from mitty_amd import _native
    ref_dict = {name: k for k, (name, _) in enumerate(self.refs)}
    recs = god.god_records(bytes(self.arena[0]), bytes(self.arena[1]) if self.arena[1] else None, ref_dict)
    segs = [[] for _ in range(len(splitters) + 1)]
    for i, r in enumerate(recs):
      key = r['reference_id'] << 33 | (r['pos'] + 1) << 1 | int(r['is_reverse'])
      info = (r['reference_id'], r['pos'], god.end_pos(r), god.reg2bin(r['pos'], god.end_pos(r)))
      segs[bisect.bisect_right(splitters, key)].append((key, tie_base + i, god.encode(r), info))
    out, off = [], [0]
    for seg in segs:
      n, nb = len(seg), sum(len(e) for _, _, e, _ in seg)
      o_roff, o_key, o_info, o_tie, total = _native.bam_part_layout(n, nb)
      buf = np.zeros(total, np.uint8)
      buf[:nb] = np.frombuffer(b''.join(e for _, _, e, _ in seg), np.uint8)
      buf[o_roff:o_key].view(np.int64)[:] = np.concatenate([[0], np.cumsum([len(e) for _, _, e, _ in seg])])
      buf[o_key:o_info].view(np.uint64)[:] = [k for k, _, _, _ in seg]
      buf[o_info:o_tie].view(np.int32)[:] = np.array([x for *_, x in seg], np.int32).reshape(-1) if n else []
      buf[o_tie:total].view(np.uint64)[:] = [t for _, t, _, _ in seg]
      out.append(buf.tobytes())
      off.append(off[-1] + total)
    self._send = b''.join(out)
    return (np.array(off, np.int64), np.array([len(x) for x in segs], np.int64),
            np.array([sum(len(e) for _, _, e, _ in x) for x in segs], np.int64))

  def bam_partition_into(self, t):
    t.numpy()[:len(self._send)] = np.frombuffer(self._send, np.uint8)

  def bam_import_segment(self, t, off, n, nb):
    from mitty_amd import _native
    o_roff, o_key, o_info, o_tie, total = _native.bam_part_layout(n, nb)
    buf = t.numpy()[off:off + total]
    roff = buf[o_roff:o_key].view(np.int64)
    keys, ties = buf[o_key:o_info].view(np.uint64), buf[o_tie:total].view(np.uint64)
    info = buf[o_info:o_tie].view(np.int32).reshape(-1, 4)
    for k in range(n):
      self.bam.append((int(keys[k]), int(ties[k]), bytes(buf[roff[k]:roff[k + 1]]), tuple(int(x) for x in info[k])))

  def _sorted(self):
    return sorted(self.bam, key=lambda x: (x[0], x[1]))

  def bam_range(self):
    return len(self.bam), sum(len(x[2]) for x in self.bam)

  def bam_head(self, n):
    return b''.join(x[2] for x in self._sorted())[:n]

  def bam_write_part(self, path, header_text, skip, tail, eof):
    from oracle import god
    from mitty_amd import _native
    data = b''.join(x[2] for x in self._sorted())[skip:] + tail
    hz = b''
    if header_text is not None:
      hz = _native.bgzf_compress(god.header_bytes(header_text, [{'SN': n, 'LN': ln} for n, ln in self.refs]))
    blocks = [_native.bgzf_compress(data[o:o + 0xff00]) for o in range(0, len(data), 0xff00)]
    boff = np.concatenate([[0], np.cumsum([len(z) for z in blocks])]).astype(np.int64)
    with open(path, 'wb') as fp:
      fp.write(hz + b''.join(blocks) + (_native.bgzf_eof() if eof else b''))
    return len(blocks), len(hz), len(hz) + int(boff[-1]) + (28 if eof else 0), boff

  def bam_bai_runs(self, n_refs):
    """mh_bam_bai_runs' arrays from the sorted records (runs of one bin in record order; first record per window)."""
    recs = self._sorted()
    soff = np.concatenate([[0], np.cumsum([len(x[2]) for x in recs])]).astype(np.int64)
    runs = []
    for k, x in enumerate(recs):
      tid, _, _, b = x[3]
      if runs and runs[-1][0] == (tid << 32 | b) and runs[-1][2] == soff[k]:
        runs[-1][2] = soff[k + 1]
        runs[-1][3] += 1
      else:
        runs.append([tid << 32 | b, soff[k], soff[k + 1], 1])
    wo = np.concatenate([[0], np.cumsum([(ln >> 14) + 1 for _, ln in self.refs])])
    win = np.full(int(wo[-1]), -1, np.int64)
    nwin = np.zeros(n_refs, np.int64)
    for k, x in enumerate(recs):
      tid, beg, end, _ = x[3]
      for w in range(beg >> 14, ((end - 1) >> 14) + 1):
        if win[wo[tid] + w] < 0:
          win[wo[tid] + w] = soff[k]
      nwin[tid] = max(nwin[tid], ((end - 1) >> 14) + 1)
    return np.array(runs, np.int64).reshape(-1, 4), win, nwin


def _records(b):
  """FASTQ bytes -> records with the '@{stub}:{cnt}|' head stripped."""
  lines = b.split(b'\n')
  return [lines[i].split(b'|', 1)[1] + b'\n' + b'\n'.join(lines[i + 1:i + 4]) + b'\n'
          for i in range(0, len(lines) - 1, 4)]

