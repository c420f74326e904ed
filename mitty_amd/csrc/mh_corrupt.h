// mh_corrupt.h — the empirical-BQ corruption of one base (illumina.corrupt_single_read, illumina.py:139-162) driven
// by Philox4x32-10, shared by the fused emission (mh_emit.hip) and standalone corrupt-reads (mh_corrupt.hip).
// Counter = (template index, file, base): output independent of launch geometry, GPU count and slicing.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mh {

constexpr int CG_BUCKETS = 256;   // search-guide buckets per BQ row: bucket k = draws in [k / 256, (k + 1) / 256)

struct CorruptCfg {
  int32_t enable;
  const float *cum;      // [2][max_bp][n_bq] cumulative BQ tables (f32)
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

// illumina.corrupt_single_read (illumina.py:155-160) for bases n0 and n0 + 1 (n0 even; cnt = 1 or 2 of them),
// Philox-driven: one draw per pair, counter (t, f, n0 / 2): words x, y are base n0's U1 and U2, z, w base n0 + 1's;
// a substituted base draws its replacement from a second counter (bit 15 of the position word set).
__device__ __forceinline__ uint32_t corrupt_bq(const CorruptCfg &cc, int f, int n, uint32_t w) {
  const float u1 = (float)(w >> 8) * (1.0f / 16777216.0f);
  const int64_t ri = (int64_t)f * cc.max_bp + n;
  const float *row = cc.cum + ri * cc.n_bq;
  int lo = 0, hi = cc.n_bq;                 // np.searchsorted(bq_mat[n, :], U1) (side='left')
  if (cc.guide) {                           // the answer lies in [g[k], g[k + 1]] for u1's bucket k
    const uint16_t *g = cc.guide + ri * (CG_BUCKETS + 1) + (w >> 24);
    lo = g[0];
    hi = g[1];
  }
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (row[mid] < u1) lo = mid + 1; else hi = mid;
  }
  return lo < 93 ? lo : 93;
}

__device__ __forceinline__ void corrupt_pair(const CorruptCfg &cc, int64_t t, int f, int n0, int cnt, uint8_t *b,
                                             uint8_t *q) {
  t += cc.t_base;
  const uint32_t cw = ((uint32_t)f << 16) | ((uint32_t)n0 >> 1);
  const uint2 key = make_uint2(cc.k0, cc.k1);
  const uint4 r = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw, cc.c3), key);
  const uint32_t wu1[2] = {r.x, r.z}, wu2[2] = {r.y, r.w};
  bool sub[2] = {false, false};
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (i >= cnt) break;
    const uint32_t bq = corrupt_bq(cc, f, n0 + i, wu1[i]);
    sub[i] = (double)wu2[i] * (1.0 / 4294967296.0) < cc.phred[bq];
    q[i] = (uint8_t)(bq + 33);
  }
  if (sub[0] || sub[1]) {   // rare: the replacement bases (randint(0, 3))
    const uint4 c = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), cw | 0x8000u, cc.c3), key);
    const uint32_t wc[2] = {c.x, c.y};
#pragma unroll
    for (int i = 0; i < 2; i++) {
      if (!sub[i]) continue;
      const uint32_t ch = __umulhi(wc[i], 3u);
      const uint8_t x = b[i];
      const char *rot = x == 'A' ? "CTG" : x == 'C' ? "ATG" : x == 'T' ? "ACG" : x == 'G' ? "ACT" : "NNN";
      b[i] = (uint8_t)rot[ch];
    }
  }
}

}  // namespace mh
