// mh_corrupt.h — the empirical-BQ corruption of one base (illumina.corrupt_single_read, illumina.py:140-162),
// shared by the fused emission (mh_emit.hip) and standalone corrupt-reads (mh_corrupt.hip).
//
// Arithmetic: U1, U2 are 53-bit uniforms and the decisions are the reference's f64 ones, bq =
// min(searchsorted(cum_bq[mate, n, :], U1, side='left'), 93) and substitution when U2 < phred_p[bq].  Word sources:
//   exact mode   the reference's own MT19937 stream (mh_corrupt.hip: rand(n), rand(n), randint(0, 3, n) per mate),
//                U = numpy's ((a >> 5) * 2^26 + (b >> 6)) / 2^53, compared in f64
//   Philox mode  Philox4x32-10 keyed by (seed, unit), one draw per base pair, counter (template, file, pair): each
//                base gets the high 32 bits h of U1 and of U2 (U = (h * 2^21 + l) / 2^53).  The decisions are taken
//                on h against u32 tables F = floor(threshold * 2^32): F < h decides "below", F > h "not below";
//                only F == h needs the low 21 bits, which then come from a second draw (flag 0x4000) and the f64
//                comparison runs — the same outcome as comparing the full 53-bit U in f64, at 32-bit cost.
//                The replacement base comes from a third counter (flag 0x8000), umulhi(word, 3).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mh {

constexpr int CG_BUCKETS = 256;   // search-guide buckets per BQ row: bucket k = draws in [k / 256, (k + 1) / 256)

struct CorruptCfg {
  int32_t enable;
  const double *cum;     // [2][max_bp][n_bq] cumulative BQ tables (the model's f64 cum_bq_mat)
  const double *phred;   // [100]
  int32_t max_bp, n_bq;
  uint32_t k0, k1, c3;   // Philox key and the constant counter word
  int64_t t_base;        // index of the launch's first template inside its unit (slices: mh_emit_reads_range)
  const uint16_t *guide = nullptr;   // [2][max_bp][CG_BUCKETS + 1]: entries of the row below k / CG_BUCKETS
  const uint32_t *F = nullptr;       // [2][max_bp][n_bq]: min(floor(cum * 2^32), 2^32 - 1)
  const uint32_t *Fp = nullptr;      // [100]: min(floor(phred_p * 2^32), 2^32 - 1)
};

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    // one 32x32 -> 64 multiply per product (v_mad_u64_u32) instead of separate mul_hi and mul_lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// numpy's legacy double from two consecutive 32-bit words (random_standard_uniform / rk_double)
__device__ __forceinline__ double mt_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// np.searchsorted(cum_bq[f, n, :], u) (side='left'), clamped to 93 (illumina.py:156); the guide narrows the search
// to [g[k], g[k + 1]] for u in bucket k (exact: g[k] counts the entries below k / CG_BUCKETS)
__device__ __forceinline__ uint32_t bq_search(const double *cum, const uint16_t *guide, int32_t max_bp, int32_t n_bq,
                                              int f, int n, double u) {
  const int64_t ri = (int64_t)f * max_bp + n;
  const double *row = cum + ri * n_bq;
  int lo = 0, hi = n_bq;
  if (guide) {
    const uint16_t *g = guide + ri * (CG_BUCKETS + 1) + (int)(u * CG_BUCKETS);
    lo = g[0];
    hi = g[1];
  }
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (row[mid] < u) lo = mid + 1; else hi = mid;
  }
  return lo < 93 ? lo : 93;
}

// base_rot.get(b, 'NNN')[c] (illumina.py:131-136, 160)
__device__ __forceinline__ uint8_t rot_base(uint8_t x, uint32_t c) {
  const char *rot = x == 'A' ? "CTG" : x == 'C' ? "ATG" : x == 'T' ? "ACG" : x == 'G' ? "ACT" : "NNN";
  return (uint8_t)rot[c];
}

// Philox mode, one base: h1 / h2 the high words of U1 / U2; returns bq and sets *sub.  `ex` supplies the low words
// (second draw) when h lands exactly on a table value.
template <typename Ex>
__device__ __forceinline__ uint32_t corrupt_base32(const CorruptCfg &cc, int f, int n, uint32_t h1, uint32_t h2,
                                                   bool *sub, Ex ex) {
  const int64_t ri = (int64_t)f * cc.max_bp + n;
  const uint32_t *F = cc.F + ri * cc.n_bq;
  const uint16_t *g = cc.guide + ri * (CG_BUCKETS + 1) + (h1 >> 24);
  int lo = g[0];
  const int hb = g[1];
  int hi = hb;
  while (lo < hi) {   // first entry with F >= h1 (entries below k * 2^24 are below every h1 of bucket k)
    const int mid = (lo + hi) >> 1;
    if (F[mid] < h1) lo = mid + 1; else hi = mid;
  }
  uint32_t bq;
  if (lo < hb && F[lo] == h1) {   // a threshold inside [h1, h1 + 1) / 2^32: the full 53 bits decide
    const uint2 l = ex();
    bq = bq_search(cc.cum, cc.guide, cc.max_bp, cc.n_bq, f, n,
                   ((double)h1 * 2097152.0 + (double)(l.x >> 11)) * (1.0 / 9007199254740992.0));
    *sub = ((double)h2 * 2097152.0 + (double)(l.y >> 11)) * (1.0 / 9007199254740992.0) < cc.phred[bq];
    return bq;
  }
  bq = lo < 93 ? lo : 93;
  const uint32_t fp = cc.Fp[bq];
  if (h2 == fp) {
    const uint2 l = ex();
    *sub = ((double)h2 * 2097152.0 + (double)(l.y >> 11)) * (1.0 / 9007199254740992.0) < cc.phred[bq];
  } else {
    *sub = h2 < fp;
  }
  return bq;
}

// Philox mode: bases n0 and n0 + 1 (n0 even; cnt = 1 or 2 of them) of file f of template t (corruption in place,
// qualities to q).  Draw (t, f, n0 / 2): words x, y are base n0's h1, h2; z, w base n0 + 1's.
__device__ __forceinline__ void corrupt_pair(const CorruptCfg &cc, int64_t t, int f, int n0, int cnt, uint8_t *b,
                                             uint8_t *q) {
  t += cc.t_base;
  const uint2 key = make_uint2(cc.k0, cc.k1);
  const uint32_t cw = ((uint32_t)f << 16) | ((uint32_t)n0 >> 1);
  const uint4 r = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw, cc.c3), key);
  bool sub[2] = {false, false};
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (i >= cnt) break;
    const uint32_t bq = corrupt_base32(cc, f, n0 + i, i ? r.z : r.x, i ? r.w : r.y, &sub[i], [&]() {
      const uint4 l = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw | 0x4000u, cc.c3), key);
      return i ? make_uint2(l.z, l.w) : make_uint2(l.x, l.y);
    });
    q[i] = (uint8_t)(bq + 33);
  }
  if (sub[0] || sub[1]) {   // rare: the replacement bases (randint(0, 3))
    const uint4 c = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw | 0x8000u, cc.c3), key);
    if (sub[0]) b[0] = rot_base(b[0], __umulhi(c.x, 3u));
    if (sub[1]) b[1] = rot_base(b[1], __umulhi(c.y, 3u));
  }
}

}  // namespace mh
