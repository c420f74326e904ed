// mh_corrupt.h — the empirical-BQ corruption of one base (illumina.corrupt_single_read, illumina.py:140-162),
// shared by the fused emission (mh_emit.hip) and standalone corrupt-reads (mh_corrupt.hip).
//
// Arithmetic is the reference's in both RNG modes: U1, U2 are 53-bit doubles built like numpy's rand()
// ((a >> 5) * 2^26 + (b >> 6)) / 2^53 from two 32-bit words, bq = min(searchsorted(cum_bq[mate, n, :], U1,
// side='left'), 93) over the f64 table, substitution when U2 < phred_p[bq] (f64).  Only the word source differs:
//   Philox mode  words from Philox4x32-10 keyed by (seed, unit), counter (template, file, base): one draw per base;
//                the replacement base from a second counter, umulhi(word, 3)
//   exact mode   the reference's own MT19937 stream (mh_corrupt.hip: rand(n), rand(n), randint(0, 3, n) per mate)
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

// Philox mode: bases n0 and n0 + 1 (cnt = 1 or 2 of them) of file f of template t.  Base n draws counter
// (t, f, n): words x, y make U1, words z, w make U2; a substituted base draws its replacement from a second counter
// (bit 15 of the position word set).
__device__ __forceinline__ void corrupt_pair(const CorruptCfg &cc, int64_t t, int f, int n0, int cnt, uint8_t *b,
                                             uint8_t *q) {
  t += cc.t_base;
  const uint2 key = make_uint2(cc.k0, cc.k1);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (i >= cnt) break;
    const uint32_t cw = ((uint32_t)f << 16) | (uint32_t)(n0 + i);
    const uint4 r = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw, cc.c3), key);
    const uint32_t bq = bq_search(cc.cum, cc.guide, cc.max_bp, cc.n_bq, f, n0 + i, mt_double(r.x, r.y));
    q[i] = (uint8_t)(bq + 33);
    if (mt_double(r.z, r.w) < cc.phred[bq]) {   // rare: the replacement base (randint(0, 3))
      const uint4 c = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw | 0x8000u, cc.c3), key);
      b[i] = rot_base(b[i], __umulhi(c.x, 3u));
    }
  }
}

}  // namespace mh
