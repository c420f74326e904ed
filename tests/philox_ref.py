"""numpy restatement of the Philox-mode BQ corruption (test infrastructure; mh_corrupt.h corrupt_triple).

The Philox mode is this framework's counter-based stream, so its specification lives here rather than in the
reference: for base n of file f of template t (t counted inside the unit), the draw (t, f, n // 3) of Philox4x32-10
gives word w = draw[n % 3]; U1 = ((w >> 16) * 2^37 + l1) / 2^53 and U2 = ((w & 0xffff) * 2^37 + l2) / 2^53, where l1, l2
are the 37-bit values (x << 5 | y >> 27), (z << 5 | w >> 27) of the base's own draw (t, f | 0x4000 flag, n).  Then the
reference's decisions in f64 (illumina.py:156-160): bq = min(searchsorted(cum_bq[f, n], U1, 'left'), 93), substitution
when U2 < phred_p[bq], by base_rot[b][c], c = c10 % 3 with c10 = bits 10 (n % 3) .. + 9 of the triple draw's fourth
word, or, when c10 = 1023, umulhi(x, 3) of the base's draw (t, f | 0x8000 flag, n).
The device decides on the 16 high bits through its u16 tables and only draws the low bits when they matter; this
restatement always uses the full 53 bits, so agreement pins the table shortcut too."""
import numpy as np

MASK = np.uint64(0xffffffff)
ROT = {ord('A'): b'CTG', ord('C'): b'ATG', ord('T'): b'ACG', ord('G'): b'ACT'}


def philox4x32_10(c0, c1, c2, c3, k0, k1):
  """Philox4x32-10 over uint64 arrays holding 32-bit values (Salmon et al. 2011)."""
  c0, c1, c2, c3 = (np.asarray(x, np.uint64) & MASK for x in (c0, c1, c2, c3))
  k0, k1 = np.uint64(k0) & MASK, np.uint64(k1) & MASK
  for _ in range(10):
    p0 = np.uint64(0xD2511F53) * c0
    p1 = np.uint64(0xCD9E8D57) * c2
    c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & MASK, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & MASK)
    k0 = (k0 + np.uint64(0x9E3779B9)) & MASK
    k1 = (k1 + np.uint64(0xBB67AE85)) & MASK
  return c0, c1, c2, c3


def keys(seed, unit_key):
  """(k0, k1, c3) of corrupt_cfg (mh_api.hip)."""
  return seed & 0xffffffff, unit_key & 0xffffffff, ((seed >> 32) ^ (unit_key >> 32) ^ 0x636f7272) & 0xffffffff


def corrupt_reads(seqs, ts, f, cum_bq, phred, seed, unit_key):
  """Corrupted bases and qualities of the reads `seqs` (bytes, file order) of file f, template indices ts."""
  k0, k1, c3 = keys(seed, unit_key)
  lens = np.array([len(s) for s in seqs])
  L = int(lens.max()) if len(seqs) else 0
  T = np.repeat(np.asarray(ts, np.uint64), lens)
  N = np.concatenate([np.arange(l) for l in lens]).astype(np.uint64)
  th, tl = T >> np.uint64(32), T & MASK
  fw = np.uint64(f << 16)
  r = philox4x32_10(tl, th, fw | (N // np.uint64(3)), np.full_like(T, c3), k0, k1)
  k = (N % np.uint64(3)).astype(np.int64)
  w = np.choose(k, r[:3])
  lo = philox4x32_10(tl, th, fw | np.uint64(0x4000) | N, np.full_like(T, c3), k0, k1)
  l1 = ((lo[0] << np.uint64(5)) | (lo[1] >> np.uint64(27))).astype(np.float64)
  l2 = ((lo[2] << np.uint64(5)) | (lo[3] >> np.uint64(27))).astype(np.float64)
  u1 = ((w >> np.uint64(16)).astype(np.float64) * 2.0 ** 37 + l1) / 2.0 ** 53
  u2 = ((w & np.uint64(0xffff)).astype(np.float64) * 2.0 ** 37 + l2) / 2.0 ** 53
  bq = np.empty(len(N), np.int64)
  Ni = N.astype(np.int64)
  for n in range(L):
    sel = Ni == n
    bq[sel] = np.minimum(np.searchsorted(cum_bq[f, n], u1[sel], side='left'), 93)
  sub = u2 < np.asarray(phred)[bq]
  c10 = ((r[3] >> (np.uint64(10) * k.astype(np.uint64))) & np.uint64(1023)).astype(np.int64)
  ch = c10 % 3
  rej = np.nonzero(sub & (c10 == 1023))[0]
  if len(rej):
    c = philox4x32_10(tl[rej], th[rej], fw | np.uint64(0x8000) | N[rej], np.full(len(rej), c3, np.uint64), k0, k1)
    ch[rej] = ((c[0] * np.uint64(3)) >> np.uint64(32)).astype(np.int64)
  base = np.frombuffer(b''.join(seqs), np.uint8).copy()
  for i in np.nonzero(sub)[0]:
    base[i] = ROT.get(int(base[i]), b'NNN')[ch[i]]
  qual = (bq + 33).astype(np.uint8)
  out_s, out_q, o = [], [], 0
  for l in lens:
    out_s.append(base[o:o + l].tobytes())
    out_q.append(qual[o:o + l].tobytes())
    o += l
  return out_s, out_q
