"""CPU oracle for the god-aligner BAM (TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker, never by the
product path).

Restates, in plain Python:
* write_perfect_reads (reference mitty/benchmarking/god_aligner.py:153-183) -> per-read attribute dicts, the form
  tests/golden/god.json captured from the reference (pinned by test_oracle_golden.py);
* the BAM record encoding of those attributes (SAM/BAM specification §4.2; bin = reg2bin(pos, bam_endpos) as
  htslib computes it), and samtools sort's coordinate order (tid, pos+1, is_reverse; stable);
* a BGZF block reader (virtual offsets of each record) and a BAI restatement over those offsets.
The BAM bytes and the BAI are pinned by the specification only (no htslib / samtools in the image): parity
unpinned beyond the record attributes.
"""
import struct
import zlib

DNA_complement = str.maketrans('ATCGN', 'TAGCN')
_NT16 = {c: i for i, c in enumerate('=ACMGRSVTWYHKDBN')}
_CIGAR = {c: i for i, c in enumerate('MIDNSHP=X')}


def parse_qname(qname):
  """readgenerate.parse_qname (readgenerate.py:259-291), as tuples (strand, pos, cigar, chrom)."""
  d = qname.split('|')
  out = []
  for strand, pos, rlen, cigar, v_list in zip(d[3::5], d[4::5], d[5::5], d[6::5], d[7::5]):
    if cigar[0] == '>':
      cigar = cigar.split(':')[-1]
    out.append((int(strand), int(pos), cigar, d[1]))
  return out


def perfect_reads(qname, ref_dict, read_data):
  """write_perfect_reads: attribute dicts of the records for one template."""
  reads = [dict() for _ in read_data]
  for (strand, pos, cigar, chrom), rd, r in zip(parse_qname(qname), read_data, reads):
    r['qname'] = qname
    r['reference_id'] = ref_dict[chrom]
    r['pos'] = pos - 1
    r['cigarstring'] = cigar
    r['mapq'] = 60
    if strand:
      r['is_reverse'] = 1
      r['seq'] = rd[0].translate(DNA_complement)[::-1]
      r['qual'] = rd[1][::-1]
    else:
      r['is_reverse'] = 0
      r['seq'] = rd[0]
      r['qual'] = rd[1]
  if len(reads) == 2:
    for n, r in enumerate(reads):
      r['is_paired'] = True
      r['is_proper_pair'] = True
      r['is_read1'] = n == 0
      r['is_read2'] = n == 1
      r['pnext'] = reads[1 - n]['pos']
      r['rnext'] = reads[1 - n]['reference_id']
  return reads


def _cigar_ops(cigar):
  ops, num = [], ''
  for c in cigar:
    if c.isdigit():
      num += c
    else:
      ops.append((int(num), _CIGAR[c]))
      num = ''
  return ops


def reg2bin(beg, end):
  end -= 1
  for shift, off in ((14, 4681), (17, 585), (20, 73), (23, 9), (26, 1)):
    if beg >> shift == end >> shift:
      return off + (beg >> shift)
  return 0


def end_pos(r):
  span = sum(n for n, op in _cigar_ops(r['cigarstring']) if op in (0, 2, 3, 7, 8))
  return r['pos'] + (span if span > 0 else 1)


def flag(r):
  f = 0x10 if r['is_reverse'] else 0
  if r.get('is_paired'):
    f |= 0x1 | 0x2 | (0x40 if r['is_read1'] else 0x80)
  return f


def encode(r):
  """BAM record bytes (block_size included) for an attribute dict."""
  ops = _cigar_ops(r['cigarstring'])
  seq, qual = r['seq'], r['qual']
  qn = r['qname'].encode() + b'\0'
  packed = bytearray()
  for i in range(0, len(seq), 2):
    hi = _NT16.get(seq[i].upper(), 15)
    lo = _NT16.get(seq[i + 1].upper(), 15) if i + 1 < len(seq) else 0
    packed.append(hi << 4 | lo)
  body = struct.pack('<iiBBHHHIiii', r['reference_id'], r['pos'], len(qn), r['mapq'], reg2bin(r['pos'], end_pos(r)),
                     len(ops), flag(r), len(seq), r.get('rnext', -1), r.get('pnext', -1), 0)
  body += qn + b''.join(struct.pack('<I', n << 4 | op) for n, op in ops) + bytes(packed)
  body += bytes(ord(c) - 33 for c in qual)
  return struct.pack('<i', len(body)) + body


def sort_key(r):
  return (r['reference_id'], r['pos'] + 1, 1 if r['is_reverse'] else 0)


def god_records(fq1_bytes, fq2_bytes, ref_dict, max_templates=None):
  """Attribute dicts of every record of a FASTQ (pair), in input order."""
  l1 = fq1_bytes.decode().split('\n')
  l2 = fq2_bytes.decode().split('\n') if fq2_bytes is not None else None
  n = len(l1) // 4
  out = []
  for i in range(n):
    if max_templates is not None and i >= max_templates:
      break
    qn = l1[4 * i][1:].split()[0]
    rd = [(l1[4 * i + 1], l1[4 * i + 3])]
    if l2 is not None:
      rd.append((l2[4 * i + 1], l2[4 * i + 3]))
    out += perfect_reads(qn, ref_dict, rd)
  return out


def sorted_stream(recs):
  order = sorted(range(len(recs)), key=lambda i: (sort_key(recs[i]), i))
  return [recs[i] for i in order]


def header_bytes(text, sq):
  b = b'BAM\1' + struct.pack('<i', len(text)) + text.encode() + struct.pack('<i', len(sq))
  for s in sq:
    nm = s['SN'].encode() + b'\0'
    b += struct.pack('<i', len(nm)) + nm + struct.pack('<i', s['LN'])
  return b


# ---- BGZF / BAI ---------------------------------------------------------------------------------------------------
def bgzf_blocks(data):
  """[(file offset, uncompressed bytes)] of a BGZF file; checks every block's framing and CRC."""
  out, pos = [], 0
  while pos < len(data):
    assert data[pos:pos + 4] == b'\x1f\x8b\x08\x04', 'bad BGZF magic at {}'.format(pos)
    xlen = struct.unpack_from('<H', data, pos + 10)[0]
    assert data[pos + 12:pos + 14] == b'BC' and xlen == 6
    bsize = struct.unpack_from('<H', data, pos + 16)[0] + 1
    cdata = data[pos + 18:pos + bsize - 8]
    crc, isize = struct.unpack_from('<II', data, pos + bsize - 8)
    raw = zlib.decompress(cdata, -15)
    assert len(raw) == isize and zlib.crc32(raw) == crc
    out.append((pos, raw))
    pos += bsize
  return out


def record_voffsets(data):
  """Decode a BAM file: (header bytes, [record bytes], [virtual offset of each record start], end voffset)."""
  blocks = bgzf_blocks(data)
  assert blocks and blocks[-1][1] == b'', 'missing EOF block'
  # stream with a map uncompressed offset -> (block file offset, within)
  starts, u = [], 0
  for off, raw in blocks:
    starts.append((u, off, len(raw)))
    u += len(raw)
  stream = b''.join(raw for _, raw in blocks)

  def voff(x):
    for us, off, ln in starts:
      if us <= x < us + ln:
        return off << 16 | (x - us)
    # the end of the data: bgzf_tell after the last record points into the still-open last block unless that
    # block filled up (then flushed: the next block, i.e. the EOF marker, at offset 0)
    for us, off, ln in reversed(starts):
      if ln:
        return off << 16 | ln if us + ln == x and ln < 0xff00 else starts[-1][1] << 16
    return starts[-1][1] << 16

  l_text = struct.unpack_from('<i', stream, 4)[0]
  p = 8 + l_text
  n_ref = struct.unpack_from('<i', stream, p)[0]
  p += 4
  for _ in range(n_ref):
    ln = struct.unpack_from('<i', stream, p)[0]
    p += 4 + ln + 4
  header = stream[:p]
  recs, vo = [], []
  while p < len(stream):
    bs = struct.unpack_from('<i', stream, p)[0]
    recs.append(stream[p:p + 4 + bs])
    vo.append(voff(p))
    p += 4 + bs
  return header, recs, vo, voff(p)


def decode(rec):
  """Attribute dict of one BAM record (the god.json keys)."""
  (_, tid, pos, l_qn, mapq, _bin, n_cig, flg, l_seq, mtid, mpos, _tlen) = struct.unpack_from('<iiiBBHHHIiii', rec, 0)
  p = 36
  qn = rec[p:p + l_qn - 1].decode()
  p += l_qn
  cig = ''.join('{}{}'.format(v >> 4, 'MIDNSHP=X'[v & 15]) for v in struct.unpack_from('<{}I'.format(n_cig), rec, p))
  p += 4 * n_cig
  seq = ''.join('=ACMGRSVTWYHKDBN'[(rec[p + i // 2] >> (4 * (1 - i % 2))) & 15] for i in range(l_seq))
  p += (l_seq + 1) // 2
  qual = ''.join(chr(q + 33) for q in rec[p:p + l_seq])
  d = {'qname': qn, 'reference_id': tid, 'pos': pos, 'cigarstring': cig, 'mapq': mapq,
       'is_reverse': 1 if flg & 0x10 else 0, 'seq': seq, 'qual': qual, 'flag': flg, 'bin': _bin}
  if flg & 1:
    d.update({'is_paired': True, 'is_proper_pair': bool(flg & 2), 'is_read1': bool(flg & 0x40),
              'is_read2': bool(flg & 0x80), 'pnext': mpos, 'rnext': mtid})
  return d


def bai(n_ref, recs, vo, vend):
  """BAI bytes for sorted decoded records with virtual offsets vo (and the end offset vend): runs of consecutive
  records in one bin are one chunk, adjacent chunks merge; linear index = first record overlapping each 16 kbp
  window, empty windows take the next window's value; pseudo-bin 37450; n_no_coor = 0.  A valid spec §5.2 index of
  the file, not claimed byte-identical to htslib's (parity unpinned)."""
  out = b'BAI\1' + struct.pack('<i', n_ref)
  ends = vo[1:] + [vend]
  i = 0
  for tid in range(n_ref):
    j = i
    while j < len(recs) and recs[j]['reference_id'] == tid:
      j += 1
    if j == i:
      out += struct.pack('<ii', 0, 0)
      continue
    bins, lin = {}, []
    for k in range(i, j):
      r = recs[k]
      ch = bins.setdefault(r['bin'], [])
      if ch and ch[-1][1] == vo[k]:
        ch[-1][1] = ends[k]
      else:
        ch.append([vo[k], ends[k]])
      w0, w1 = r['pos'] >> 14, (end_pos(r) - 1) >> 14
      if len(lin) <= w1:
        lin += [None] * (w1 + 1 - len(lin))
      for w in range(w0, w1 + 1):
        if lin[w] is None:
          lin[w] = vo[k]
    out += struct.pack('<i', len(bins) + 1)
    for b in sorted(bins):
      out += struct.pack('<Ii', b, len(bins[b])) + b''.join(struct.pack('<QQ', *c) for c in bins[b])
    out += struct.pack('<Ii', 37450, 2) + struct.pack('<QQQQ', vo[i], ends[j - 1], j - i, 0)
    nxt = ends[j - 1]
    for w in range(len(lin) - 1, -1, -1):
      if lin[w] is None:
        lin[w] = nxt
      else:
        nxt = lin[w]
    out += struct.pack('<i', len(lin)) + b''.join(struct.pack('<Q', v) for v in lin)
    i = j
  return out + struct.pack('<Q', 0)
