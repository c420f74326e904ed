// mh_deflate.h — the parts of the device BGZF compressor (mh_deflate.hip) that run on one thread: deflate's
// length / distance code tables (RFC 1951 §3.2.5), length-limited Huffman code lengths from symbol frequencies,
// canonical codes, the dynamic block header (§3.2.7) and CRC-32 combination (RFC 1952).  __host__ __device__, so
// tests/deflate_host.cpp exercises exactly this code on the CPU (with zlib inflating the result).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mh {
namespace df {

constexpr int BLOCK = 0xff00;         // input bytes per BGZF block (htslib's BGZF_BLOCK_SIZE)
constexpr int MAX_BSIZE = 65536;      // a BGZF block, header and trailer included
constexpr int HDR = 18, TRL = 8;      // gzip member header with the BC extra field; CRC32 + ISIZE
constexpr int NLIT = 286, NDIST = 30, NCL = 19;
// MIN_MATCH: the shortest match taken.  Inside FASTQ bases (random ACGT) a 4-6-byte match costs more bits than its
// literals (~2 bits each) and cuts the parse into short steps: from 4 to 7 the golden FASTQ deflates to 4.50x instead
// of 4.30x (gzip -1: 4.39x) in 6.8x fewer parse steps.  Positions are hashed on their first HASH_BYTES bytes.
constexpr int MIN_MATCH = 7, HASH_BYTES = 4, MAX_MATCH = 258, MAX_DIST = 32768;

__host__ __device__ inline int len_code(int len) {   // 3..258 -> 0..28 (symbol 257 + code)
  if (len <= 10) return len - 3;
  if (len == 258) return 28;
  int x = len - 3, b = 31 - __builtin_clz((unsigned)x);   // x >= 8: bits 3..7
  return 4 * (b - 1) + ((x >> (b - 2)) & 3);
}
__host__ __device__ inline int len_base(int c) {
  if (c < 8) return c + 3;
  if (c == 28) return 258;
  return 3 + ((4 + (c & 3)) << (c / 4 - 1));   // c / 4 - 1 extra bits
}
__host__ __device__ inline int len_extra(int c) { return (c < 8 || c == 28) ? 0 : c / 4 - 1; }
__host__ __device__ inline int dist_code(int d) {   // 1..32768 -> 0..29
  if (d <= 4) return d - 1;
  int x = d - 1, b = 31 - __builtin_clz((unsigned)x);
  return 2 * b + ((x >> (b - 1)) & 1);
}
__host__ __device__ inline int dist_extra(int c) { return c < 4 ? 0 : c / 2 - 1; }
__host__ __device__ inline int dist_base(int c) {
  if (c < 4) return c + 1;
  const int e = c / 2 - 1;
  return 1 + ((2 + (c & 1)) << e);
}

__host__ __device__ inline uint32_t bit_reverse(uint32_t code, int len) {
  uint32_t r = 0;
  for (int i = 0; i < len; i++) {
    r = (r << 1) | (code & 1u);
    code >>= 1;
  }
  return r;
}

// Code lengths, at most `limit` bits, for the m used symbols whose keys (frequency << 9 | symbol) are in `keys`,
// sorted ascending (the caller sorts: a wave-parallel sort on the device).  len[] must be zero for unused symbols;
// A is scratch for m entries and count for 32 (LDS on the device: a thread-local array indexed at run time would be
// scratch memory, a global-memory round trip per access).  Single thread.  Huffman's algorithm in place over the frequency-sorted weights
// (Moffat & Katajainen, "In-place calculation of minimum-redundancy codes", 1995), then the depths above `limit`
// folded back with the Kraft sum kept at 1, and the lengths handed out again in frequency order.  One used symbol
// gets length 1.
__host__ __device__ inline void huffman_from_sorted(const uint32_t *keys, int m, int limit, uint8_t *len, uint32_t *A,
                                                    int32_t *count) {
  if (m == 0) return;
  if (m == 1) {
    len[keys[0] & 511u] = 1;
    return;
  }
  for (int i = 0; i < m; i++) A[i] = keys[i] >> 9;
  // first pass, left to right: internal node weights and parent pointers
  A[0] += A[1];
  int root = 0, leaf = 2;
  for (int next = 1; next < m - 1; next++) {
    if (leaf >= m || A[root] < A[leaf]) {
      A[next] = A[root];
      A[root++] = (uint32_t)next;
    } else {
      A[next] = A[leaf++];
    }
    if (leaf >= m || (root < next && A[root] < A[leaf])) {
      A[next] += A[root];
      A[root++] = (uint32_t)next;
    } else {
      A[next] += A[leaf++];
    }
  }
  // second pass, right to left: internal node depths
  A[m - 2] = 0;
  for (int next = m - 3; next >= 0; next--) A[next] = A[A[next]] + 1;
  // third pass, right to left: leaf depths
  int avail = 1, used = 0, depth = 0;
  root = m - 2;
  int nx = m - 1;
  while (avail > 0) {
    while (root >= 0 && (int)A[root] == depth) {
      used++;
      root--;
    }
    while (avail > used) {
      A[nx--] = (uint32_t)depth;
      avail--;
    }
    avail = 2 * used;
    depth++;
    used = 0;
  }
  // A[i]: the code length of the i-th least frequent symbol
  for (int b = 0; b < 32; b++) count[b] = 0;
  for (int i = 0; i < m; i++) count[A[i] > 31 ? 31 : A[i]]++;
  int over = 0;
  for (int b = limit + 1; b < 32; b++) {
    over += count[b];
    count[limit] += count[b];
    count[b] = 0;
  }
  if (over) {   // Kraft sum back to exactly 1: a leaf off the deepest level, a shallower one split in two
    uint32_t total = 0;
    for (int b = limit; b > 0; b--) total += (uint32_t)count[b] << (limit - b);
    while (total != (1u << limit)) {
      count[limit]--;
      for (int b = limit - 1; b > 0; b--)
        if (count[b]) {
          count[b]--;
          count[b + 1] += 2;
          break;
        }
      total--;
    }
  }
  int i = 0;   // the least frequent symbols get the longest codes
  for (int b = limit; b > 0; b--)
    for (int k = 0; k < count[b]; k++) len[keys[i++] & 511u] = (uint8_t)b;
}

// The keys of the used symbols of f[0..n), sorted ascending (insertion sort: for the 19-symbol code-length code).
__host__ __device__ inline int sorted_keys_small(const uint32_t *f, int n, uint32_t *keys) {
  int m = 0;
  for (int s = 0; s < n; s++)
    if (f[s]) {
      const uint32_t v = (f[s] << 9) | (uint32_t)s;
      int j = m - 1;
      while (j >= 0 && keys[j] > v) {
        keys[j + 1] = keys[j];
        j--;
      }
      keys[j + 1] = v;
      m++;
    }
  return m;
}

// Canonical codes (bit-reversed for deflate's LSB-first bit order) from lengths; count and next: 16 entries of
// scratch each.  Single thread (the device builds the two main alphabets' codes wave-wide: mh_deflate.hip).
__host__ __device__ inline void canonical_codes(const uint8_t *len, int n, uint16_t *code, int32_t *count,
                                                int32_t *next) {
  for (int b = 0; b < 16; b++) count[b] = 0;
  for (int s = 0; s < n; s++) count[len[s]]++;
  count[0] = 0;
  int c = 0;
  for (int b = 1; b < 16; b++) {
    c = (c + count[b - 1]) << 1;
    next[b] = c;
  }
  for (int s = 0; s < n; s++)
    code[s] = len[s] ? (uint16_t)bit_reverse((uint32_t)next[len[s]]++, len[s]) : 0;
}

// LSB-first bit sink over a byte buffer (single thread): the dynamic block header.
struct BitSink {
  uint8_t *out;
  uint64_t acc;
  int nacc;
  int64_t pos;
  __host__ __device__ void put(uint32_t v, int n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    while (nacc >= 8) {
      out[pos++] = (uint8_t)acc;
      acc >>= 8;
      nacc -= 8;
    }
  }
};

constexpr uint8_t CL_ORDER[NCL] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Scratch of write_dynamic_header (LDS on the device)
struct HeaderScratch {
  uint8_t seq[NLIT + NDIST];
  uint32_t rl[NLIT + NDIST];
  uint32_t cf[NCL], keys[NCL], A[NCL];
  int32_t count[32], next[16];
  uint8_t cl[NCL];
  uint16_t cc[NCL];
};

// The dynamic block's header after BFINAL/BTYPE: HLIT, HDIST, HCLEN, the code-length code and the run-length coded
// lengths of both alphabets (one sequence, §3.2.7).  Single thread.
__host__ __device__ inline void write_dynamic_header(BitSink &bs, const uint8_t *llen, const uint8_t *dlen,
                                                     HeaderScratch &H) {
  int hlit = NLIT, hdist = NDIST;
  while (hlit > 257 && llen[hlit - 1] == 0) hlit--;
  while (hdist > 1 && dlen[hdist - 1] == 0) hdist--;
  uint8_t *seq = H.seq;
  for (int i = 0; i < hlit; i++) seq[i] = llen[i];
  for (int i = 0; i < hdist; i++) seq[hlit + i] = dlen[i];
  const int total = hlit + hdist;
  // run-length symbols: value | extra << 8
  uint32_t *rl = H.rl;
  int nrl = 0;
  uint32_t *cf = H.cf;
  for (int i = 0; i < NCL; i++) cf[i] = 0;
  for (int i = 0; i < total;) {
    const uint8_t v = seq[i];
    int run = 1;
    while (i + run < total && seq[i + run] == v) run++;
    int left = run;
    if (v == 0) {
      while (left >= 11) {
        const int k = left > 138 ? 138 : left;
        rl[nrl++] = 18u | (uint32_t)(k - 11) << 8;
        cf[18]++;
        left -= k;
      }
      if (left >= 3) {
        rl[nrl++] = 17u | (uint32_t)(left - 3) << 8;
        cf[17]++;
        left = 0;
      }
    } else {
      rl[nrl++] = v;
      cf[v]++;
      left--;
      while (left >= 3) {
        const int k = left > 6 ? 6 : left;
        rl[nrl++] = 16u | (uint32_t)(k - 3) << 8;
        cf[16]++;
        left -= k;
      }
    }
    while (left-- > 0) {
      rl[nrl++] = v;
      cf[v]++;
    }
    i += run;
  }
  uint8_t *cl = H.cl;
  uint16_t *cc = H.cc;
  for (int i = 0; i < NCL; i++) cl[i] = 0;
  huffman_from_sorted(H.keys, sorted_keys_small(cf, NCL, H.keys), 7, cl, H.A, H.count);
  canonical_codes(cl, NCL, cc, H.count, H.next);
  int hclen = NCL;
  while (hclen > 4 && cl[CL_ORDER[hclen - 1]] == 0) hclen--;
  bs.put((uint32_t)(hlit - 257), 5);
  bs.put((uint32_t)(hdist - 1), 5);
  bs.put((uint32_t)(hclen - 4), 4);
  for (int i = 0; i < hclen; i++) bs.put(cl[CL_ORDER[i]], 3);
  for (int i = 0; i < nrl; i++) {
    const uint32_t s = rl[i] & 0xffu, x = rl[i] >> 8;
    bs.put(cc[s], cl[s]);
    if (s == 16) bs.put(x, 2);
    else if (s == 17) bs.put(x, 3);
    else if (s == 18) bs.put(x, 7);
  }
}

// ---- CRC-32 (RFC 1952, reflected polynomial 0xEDB88320) ------------------------------------------------------------
constexpr uint32_t CRC_POLY = 0xedb88320u;

// a * b modulo the CRC polynomial (reflected bit order)
__host__ __device__ constexpr inline uint32_t crc_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ CRC_POLY : b >> 1;
  }
  return p;
}
// x^(8 n) modulo the polynomial: the operator that appends n zero bytes
__host__ __device__ inline uint32_t crc_x8n(uint64_t n) {
  uint32_t p = 1u << 31;          // x^0
  uint32_t sq = 1u << 23;          // x^8
  while (n) {
    if (n & 1) p = crc_multmodp(sq, p);
    sq = crc_multmodp(sq, sq);
    n >>= 1;
  }
  return p;
}
// crc32(A || B) from crc32(A), crc32(B) and len(B)
__host__ __device__ inline uint32_t crc_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return crc_multmodp(crc_x8n(len_b), crc_a) ^ crc_b;
}

// CRC-32 of a block by segments (the device: one segment per thread).  The raw CRC (register starting at 0, no final
// inversion) is linear, so raw(block) = XOR over segments i of raw(segment i) * x^(8 (n - end_i)), and
// crc32 = ~(raw(block) ^ 0xffffffff * x^(8 n)).  With segments of CRC_SEG bytes, n = q CRC_SEG + r: a whole segment
// i < q is scaled by x^(8 CRC_SEG (q - 1 - i)) and then, all together, by x^(8 r); the partial segment q is not
// scaled.  The powers are compile-time tables.  CRC_SEG = 132 bytes (33 words): lanes' word loads at 132-byte
// strides fall in different LDS banks (128 put every lane on one bank).
constexpr int CRC_SEG = 132;
constexpr int CRC_NSEG = (BLOCK + CRC_SEG - 1) / CRC_SEG;   // 495 (<= 512 threads)
struct CrcPowers {
  uint32_t seg[CRC_NSEG + 1];   // x^(8 CRC_SEG j)
  uint32_t byte[CRC_SEG];       // x^(8 r)
};
constexpr CrcPowers make_crc_powers() {
  CrcPowers t{};
  uint32_t p = 1u << 31;   // x^0
  for (int r = 0; r < CRC_SEG; r++) {
    t.byte[r] = p;
    p = crc_multmodp(1u << 23, p);   // * x^8
  }
  uint32_t q = 1u << 31;
  for (int j = 0; j <= CRC_NSEG; j++) {
    t.seg[j] = q;
    q = crc_multmodp(p, q);          // * x^(8 CRC_SEG)
  }
  return t;
}
// the raw CRC register after byte b (table of 256 entries: the standard reflected table)
__host__ __device__ inline uint32_t crc_raw_byte(uint32_t c, uint32_t b, const uint32_t *tab) {
  return tab[(c ^ b) & 0xffu] ^ (c >> 8);
}
// crc32 of n bytes by the segment method (host restatement of the device's, checked against the direct CRC)
__host__ inline uint32_t crc32_segments(const uint8_t *b, int n, const CrcPowers &P, const uint32_t *tab) {
  const int q = n / CRC_SEG, r = n - q * CRC_SEG;
  uint32_t acc = 0, tail = 0;
  for (int i = 0; i * CRC_SEG < n; i++) {
    const int a = i * CRC_SEG, e = a + CRC_SEG < n ? a + CRC_SEG : n;
    uint32_t c = 0;
    for (int k = a; k < e; k++) c = crc_raw_byte(c, b[k], tab);
    if (i < q) acc ^= crc_multmodp(P.seg[q - 1 - i], c);
    else tail = c;
  }
  const uint32_t raw = crc_multmodp(P.byte[r], acc) ^ tail;
  return ~(crc_multmodp(crc_multmodp(P.seg[q], P.byte[r]), 0xffffffffu) ^ raw);
}

}  // namespace df
}  // namespace mh
