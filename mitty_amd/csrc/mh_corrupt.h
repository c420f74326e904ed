// mh_corrupt.h — the empirical-BQ corruption of one base (illumina.corrupt_single_read, illumina.py:140-162),
// shared by the fused emission (mh_emit.hip) and standalone corrupt-reads (mh_corrupt.hip).
//
// Arithmetic: U1, U2 are 53-bit uniforms and the decisions are the reference's f64 ones, bq =
// min(searchsorted(cum_bq[mate, n, :], U1, side='left'), 93) and substitution when U2 < phred_p[bq].  Word sources:
//   exact mode   the reference's own MT19937 stream (mh_corrupt.hip: rand(n), rand(n), randint(0, 3, n) per mate),
//                U = numpy's ((a >> 5) * 2^26 + (b >> 6)) / 2^53, compared in f64
//   Philox mode  Philox4x32-10 keyed by (seed, unit), one draw per three bases, counter (template, file, triple):
//                base k of the triple takes word k (x, y, z): h1 = its high 16 bits (the top of U1), h2 = its low
//                16 bits (the top of U2), U = (h * 2^37 + l) / 2^53; word w holds the three bases' replacement
//                choices, 10 bits each (c < 1023: randint(0, 3) = c % 3, exact since 1023 = 3 * 341; c = 1023: the
//                base's own draw (t, f | 0x8000, n), umulhi(x, 3)).  Decisions are taken on h against u16 tables
//                T = floor(x * 2^16) (clamped to 65535): T < h decides "below", T > h "not below"; only T == h needs
//                the low 37 bits, which then come from a per-base draw (flag 0x4000) and the f64 comparison runs —
//                the outcome of comparing the full 53-bit U in f64.  The BQ search is one byte per draw:
//                bk[row][h1 >> 8] holds the entries below the bucket (capped at 93) and a flag when a threshold
//                falls inside it (then the row's T entries from there are walked).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mh {

constexpr int CG_BUCKETS = 256;   // search-guide buckets per BQ row: bucket k = draws in [k / 256, (k + 1) / 256)
constexpr int CB_ROW = 256;       // Philox mode: bucket-table bytes per BQ row (h1 >> 8)
constexpr int CF_SHIFT = 6;       // Philox mode, the row pass's fine table: bucket h1 >> 6 (1024 per row)
constexpr int CF_ROW = 65536 >> CF_SHIFT;

struct CorruptCfg {
  int32_t enable;
  const double *cum;     // [2][max_bp][n_bq] cumulative BQ tables (the model's f64 cum_bq_mat)
  const double *phred;   // [100]
  int32_t max_bp, n_bq;
  uint32_t k0, k1, c3;   // Philox key and the constant counter word
  int64_t t_base;        // index of the launch's first template inside its unit (slices: mh_emit_reads_range)
  const uint16_t *guide = nullptr;   // [2][max_bp][CG_BUCKETS + 1]: entries of the row below k / CG_BUCKETS
  const uint8_t *bk = nullptr;       // [2][max_bp][CB_ROW]: min(entries below k / 256, 93) | 0x80 (one inside)
  const uint16_t *T16 = nullptr;     // [2][max_bp][n_bq]: min(floor(cum * 2^16), 65535)
  const uint16_t *Fp16 = nullptr;    // [100]: min(floor(phred_p * 2^16), 65535)
  const uint8_t *bkf = nullptr;      // [2][max_bp][CF_ROW]: bk's entries over 1024 buckets (the row pass: a threshold
                                     // inside the draw's bucket for ~2.2 % of draws instead of ~7 %)
};

// a ^ b ^ k in one VALU instruction (gfx950 v_bitop3_b32, truth table 0x96; the compiler emits two v_xor_b32 for
// a ^ b ^ k).  The builtin, not inline asm: the compiler then knows the instruction's hazards (the asm form was
// padded with s_nop, ~38 per block of the corruption rows) and schedules around it.
__device__ __forceinline__ uint32_t xor3_vvs(uint32_t a, uint32_t b, uint32_t k) {
  return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
}

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    // one 32x32 -> 64 multiply per product (v_mad_u64_u32) instead of separate mul_hi and mul_lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(xor3_vvs(hi1, c.y, k.x), lo1, xor3_vvs(hi0, c.w, k.y), lo0);
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
  // the three replacements packed little-endian in a word (no table load): "CTG", "ATG", "ACG", "ACT", "NNN"
  const uint32_t rot = x == 'A' ? 0x475443u : x == 'C' ? 0x475441u : x == 'T' ? 0x474341u : x == 'G' ? 0x544341u
                                                                                                    : 0x4e4e4eu;
  return (uint8_t)(rot >> (8 * c));
}

// Philox mode, the BQ step from global memory: entries of row (f, n) below h1 (capped at 93) and whether one equals
// h1 (then the low bits decide), from the bucket entry e = bk[f][n][h1 >> 8] and, for a flagged bucket, a walk over
// the row's T16 from the bucket's first entry.
__device__ __forceinline__ uint32_t bq_walk_g(const CorruptCfg &cc, int f, int n, uint32_t h1, bool *amb) {
  const uint32_t e = cc.bk[((int64_t)f * cc.max_bp + n) * CB_ROW + (h1 >> 8)];
  uint32_t bq = e & 0x7fu;
  *amb = false;
  if (e & 0x80u) {
    const uint16_t *T = cc.T16 + ((int64_t)f * cc.max_bp + n) * cc.n_bq;
    const uint32_t lim = cc.n_bq < 93 ? (uint32_t)cc.n_bq : 93u;
    uint32_t v = bq < lim ? T[bq] : 0xffffffffu;
    while (v < h1) {
      bq++;
      v = bq < lim ? T[bq] : 0xffffffffu;
    }
    *amb = v == h1;
  }
  return bq;
}

// Philox mode, the rare tails out of line (the hot loop stays small): the f64 decisions with the base's low bits
// (draw (t, f | 0x4000, n)) when h1 lands on a BQ threshold (amb) or h2 on Fp16[bq]; returns bq | sub << 8.
__device__ __forceinline__ uint32_t cq_exact_body(const double *cum, const double *phred, const uint16_t *guide,
                                                  int32_t max_bp, int32_t n_bq, uint32_t k0, uint32_t k1, uint32_t c3,
                                                  uint32_t tl, uint32_t th, int f, int n, uint32_t w, uint32_t bq,
                                                  uint32_t amb) {
  const uint4 l = philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x4000u | (uint32_t)n, c3), make_uint2(k0, k1));
  if (amb) {
    const double u1 = ((double)(w >> 16) * 137438953472.0 + (double)(((uint64_t)l.x << 5) | (l.y >> 27))) *
                      (1.0 / 9007199254740992.0);
    bq = bq_search(cum, guide, max_bp, n_bq, f, n, u1);
  }
  const double u2 = ((double)(w & 0xffffu) * 137438953472.0 + (double)(((uint64_t)l.z << 5) | (l.w >> 27))) *
                    (1.0 / 9007199254740992.0);
  return bq | (u2 < phred[bq] ? 0x100u : 0u);
}
static __device__ __noinline__ uint32_t cq_exact(const double *cum, const double *phred, const uint16_t *guide,
                                                 int32_t max_bp, int32_t n_bq, uint32_t k0, uint32_t k1, uint32_t c3,
                                                 uint32_t tl, uint32_t th, int f, int n, uint32_t w, uint32_t bq,
                                                 uint32_t amb) {
  return cq_exact_body(cum, phred, guide, max_bp, n_bq, k0, k1, c3, tl, th, f, n, w, bq, amb);
}

// Philox mode: bases n0 .. n0 + cnt - 1 (n0 = 3 * triple, cnt <= 3) of file f of template t (t without t_base):
// b[] corrupted in place, qualities (bq + 33) to q[].  walk(n, h1, &amb) -> the BQ step (entries below h1, capped
// at 93; amb when one equals h1), fp(bq) -> Fp16[bq].
template <typename BK, typename FP>
__device__ __forceinline__ void corrupt_triple(const CorruptCfg &cc, int64_t t, int f, int n0, int cnt, uint8_t *b,
                                               uint8_t *q, BK walk, FP fp) {
  t += cc.t_base;
  const uint32_t tl = (uint32_t)t, th = (uint32_t)(t >> 32);
  const uint4 r = philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | ((uint32_t)n0 / 3u), cc.c3),
                                make_uint2(cc.k0, cc.k1));
#pragma unroll
  for (int k = 0; k < 3; k++) {   // (selects, not an indexed array: that would be placed in scratch)
    if (k < cnt) {
      const int n = n0 + k;
      const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : r.z;
      bool amb;
      uint32_t bq = walk(n, w >> 16, &amb);
      const uint32_t p = fp(bq);
      bool s;
      if (amb || (w & 0xffffu) == p) {   // U1 or U2 within 2^-16 of a threshold: the full 53 bits decide
        const uint32_t x = cq_exact(cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq, cc.k0, cc.k1, cc.c3, tl, th, f, n,
                                    w, bq, amb);
        bq = x & 0xffu;
        s = x >> 8;
      } else {
        s = (w & 0xffffu) < p;
      }
      q[k] = (uint8_t)(bq + 33);
      if (s) {   // randint(0, 3): the triple's 10 choice bits, or (rejected) the base's own draw
        uint32_t c10 = (r.w >> (10 * k)) & 1023u;
        if (c10 == 1023u)
          c10 = __umulhi(philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)n, cc.c3),
                                       make_uint2(cc.k0, cc.k1)).x, 3u);
        b[k] = rot_base(b[k], c10 % 3u);
      }
    }
  }
}

// corrupt_triple with the tables read from global memory
__device__ __forceinline__ void corrupt_triple_g(const CorruptCfg &cc, int64_t t, int f, int n0, int cnt, uint8_t *b,
                                                 uint8_t *q) {
  corrupt_triple(
      cc, t, f, n0, cnt, b, q,
      [&](int n, uint32_t h1, bool *amb) -> uint32_t { return bq_walk_g(cc, f, n, h1, amb); },
      [&](uint32_t bq) -> uint32_t { return cc.Fp16[bq]; });
}

}  // namespace mh
