"""Read-generation algorithms (reference mitty/simulation/rpc.py), backed by the device splice.

`create_node_list` splices on the GPU (mh_build_haplotype) and returns a NodeList — a list of Node exactly as the
reference builds it — that remembers its device slot, so `get_begin_end_nodes` and `generate_read` run on the
device (mh_read_batch) against the same haplotype.  The reference's per-variant helpers `create_nodes` / `snp` /
`insertion` / `deletion` (rpc.py:66-116) are exposed over mh_expand_variant: the node rules the device splice applies
to each accepted variant (one function, compiled for the kernel and the host), given the caller's cursors.
"""
import itertools

import numpy as np

from mitty_amd.lib import vcfio


class Node(object):
  __slots__ = ('ps', 'pr', 'cigarop', 'oplen', 'seq', 'v')

  def __init__(self, ps, pr, cigarop, oplen, seq):
    self.ps = ps
    self.pr = pr
    self.cigarop = cigarop
    self.oplen = oplen
    self.seq = seq
    self.v = {'=': None, 'X': 0, 'I': oplen, 'D': -oplen}[cigarop]

  def tuple(self):
    return self.ps, self.pr, self.cigarop, self.oplen, self.seq, self.v

  def __repr__(self):
    return self.tuple().__repr__()

  def __eq__(self, other):
    if isinstance(other, self.__class__):
      return self.tuple() == other.tuple()
    return self.tuple() == other

  def __ne__(self, other):
    return not self.__eq__(other)


class NodeList(list):
  """Nodes plus the device haplotype slot they came from."""
  _slots = itertools.count(1 << 20)

  def __init__(self, nodes, ctx, slot, contig_id):
    super().__init__(nodes)
    self.ctx, self.slot, self.contig_id = ctx, slot, contig_id

  def __del__(self):
    try:
      self.ctx.release_haplotype(self.slot)
    except Exception:
      pass


def _ctx():
  from mitty_amd.simulation.illumina import device_context
  return device_context()


def create_node_list(ref_seq, ref_start_pos, vl):
  """rpc.create_node_list (rpc.py:38-63) on the device."""
  ctx = _ctx()
  slot = next(NodeList._slots)
  raw = ref_seq.encode() if isinstance(ref_seq, str) else bytes(ref_seq)
  ctx.upload_contig(slot, raw)
  soa = vcfio.soa_from_variants(vl)
  n, p_min, _ = ctx.build_haplotype(slot, slot, ref_start_pos, soa)
  ps, pr, op, ol, hap = ctx.get_nodes(slot, n)
  hap = hap.decode('latin-1')
  nodes = []
  for k in range(n):
    o = chr(op[k])
    seq = '' if o == 'D' else hap[ps[k] - p_min: ps[k] - p_min + ol[k]]
    nodes.append(Node(int(ps[k]), int(pr[k]), o, int(ol[k]), seq))
  return NodeList(nodes, ctx, slot, slot)


def _expand(op, ref_seq, samp_pos, ref_pos, v, ref_start_pos):
  from mitty_amd import _native
  raw, samp_next, ref_next = _native.expand_variant(samp_pos, ref_pos, ref_start_pos, v.pos, op, v.oplen)
  nodes = []
  for ps, pr, o, ol, src in raw:
    seq = ref_seq[src:src + ol] if o == '=' else ('' if o == 'D' else v.alt[src:])
    nodes.append(Node(ps, pr, o, ol, seq))
  return nodes, samp_next, ref_next


def snp(ref_seq, samp_pos, ref_pos, v, ref_start_pos):
  """rpc.snp (rpc.py:75-87): ([optional '=' node, 'X' node], samp_pos, ref_pos) after the variant."""
  return _expand('X', ref_seq, samp_pos, ref_pos, v, ref_start_pos)


def insertion(ref_seq, samp_pos, ref_pos, v, ref_start_pos):
  """rpc.insertion (rpc.py:90-101)."""
  return _expand('I', ref_seq, samp_pos, ref_pos, v, ref_start_pos)


def deletion(ref_seq, samp_pos, ref_pos, v, ref_start_pos):
  """rpc.deletion (rpc.py:104-116)."""
  return _expand('D', ref_seq, samp_pos, ref_pos, v, ref_start_pos)


def create_nodes(ref_seq, samp_pos, ref_pos, v, ref_start_pos):
  """rpc.create_nodes (rpc.py:66-72): the helper v.cigarop selects ('X', 'I', anything else 'D')."""
  return _expand(v.cigarop if v.cigarop in ('X', 'I') else 'D', ref_seq, samp_pos, ref_pos, v, ref_start_pos)


def _device_nodes(nodes):
  if not isinstance(nodes, NodeList):
    raise TypeError('node list must come from mitty_amd.simulation.rpc.create_node_list (device-resident)')
  return nodes


def get_begin_end_nodes(pl, ll, nodes):
  """rpc.get_begin_end_nodes (rpc.py:119-130): [n0 array, n1 array]."""
  nodes = _device_nodes(nodes)
  pl = np.asarray(pl, dtype=np.int64)
  ll = np.broadcast_to(np.asarray(ll, dtype=np.int64), pl.shape)
  _, n0, n1, _, _ = nodes.ctx.read_batch(nodes.slot, pl, ll)
  return [n0, n1]


def generate_reads_batch(pl, ll, nodes):
  """Vectorised rpc.generate_read: [(pos, cigar, v_list, seq), ...] for reads (p, l)."""
  nodes = _device_nodes(nodes)
  pl = np.asarray(pl, dtype=np.int64)
  ll = np.broadcast_to(np.asarray(ll, dtype=np.int64), pl.shape)
  pos, n0, n1, (ct, vt, st), (co, vo, so) = nodes.ctx.read_batch(nodes.slot, pl, ll)
  out = []
  for i in range(len(pl)):
    v = vt[vo[i]:vo[i + 1]]
    out.append((int(pos[i]), ct[co[i]:co[i + 1]], [int(x) for x in v.split(',')] if v else [], st[so[i]:so[i + 1]]))
  return out, n0, n1


def generate_read(p, l, n0, n1, nodes):
  """rpc.generate_read (rpc.py:133-160) -> (pos, cigar, v_list, seq)."""
  res, a, b = generate_reads_batch([p], [l], nodes)
  if int(a[0]) != int(n0) or int(b[0]) != int(n1):
    raise ValueError('n0/n1 ({}, {}) are not the start/end nodes of read ({}, {}): expected ({}, {})'.format(
      n0, n1, p, l, int(a[0]), int(b[0])))
  return res[0]
