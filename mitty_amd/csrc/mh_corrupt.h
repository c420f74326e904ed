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

// illumina.corrupt_single_read for one base (illumina.py:155-160), Philox-driven.
__device__ __forceinline__ void corrupt_base(const CorruptCfg &cc, int64_t t, int f, int n, uint8_t &b, uint8_t &q) {
  t += cc.t_base;
  uint4 r = philox4x32_10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), ((uint32_t)f << 16) | (uint32_t)n, cc.c3),
                          make_uint2(cc.k0, cc.k1));
  const float u1 = (float)(r.x >> 8) * (1.0f / 16777216.0f);
  const int64_t ri = (int64_t)f * cc.max_bp + n;
  const float *row = cc.cum + ri * cc.n_bq;
  int lo = 0, hi = cc.n_bq;                 // np.searchsorted(bq_mat[n, :], U1) (side='left')
  if (cc.guide) {                           // the answer lies in [g[k], g[k + 1]] for u1's bucket k
    const uint16_t *g = cc.guide + ri * (CG_BUCKETS + 1) + (r.x >> 24);
    lo = g[0];
    hi = g[1];
  }
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (row[mid] < u1) lo = mid + 1; else hi = mid;
  }
  const int bq = lo < 93 ? lo : 93;
  const double u2 = (double)r.y * (1.0 / 4294967296.0);
  if (u2 < cc.phred[bq]) {
    const uint32_t ch = __umulhi(r.z, 3u);  // randint(0, 3)
    const char *rot = b == 'A' ? "CTG" : b == 'C' ? "ATG" : b == 'T' ? "ACG" : b == 'G' ? "ACT" : "NNN";
    b = (uint8_t)rot[ch];
  }
  q = (uint8_t)(bq + 33);
}

}  // namespace mh
