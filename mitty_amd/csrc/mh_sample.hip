// mh_sample.hip — template sampling on the device (reference illumina.generate_reads, illumina.py:43-110).
//
// Parity mode (MH_RNG_MITTY) reproduces numpy's legacy RandomState streams word for word:
//   seed -> RS(seed).randint(SEED_MAX, 4) = (tloc, tlen, shuffle, file_order) seeds        (host, 4 words)
//   k_mt_streams     one 256-thread workgroup per MT19937 stream; the 624-word state lives in LDS and is
//                    advanced in the three dependency phases of the twist ([0,227) [227,454) [454,624)),
//                    tempered words streamed to HBM (tloc: 2n words, tlen: 2n words, file order: n/4 words)
//   scan(geometric)  ts = cumsum(ceil(log1p(-U)/log(1-p))) + p_min + 1, the geometric draw computed inside the
//                    scan's Load; a draw whose quotient lies within 1e-9 of an integer is flagged and recomputed
//                    with the host libm (the reference's libm) before the scan is redone
//   k_shuffle_decode Fisher-Yates swap indices j_i = random_interval(i), i = n-1..1: one workgroup per stream
//                    fuses MT19937 with a block-parallel rejection decode (fixed-point on the accept prefix,
//                    exact; sequential fallback for the rare non-converging chunk)
//   k_perm_*         the permutation those swaps produce, without replaying them: bucket the steps by target j,
//                    then for each output slot p chase  q = j_p -> next step with the same target -> ...
//                    (see perm_chase below); ts_shuf[p] = ts[q]
//   k_tlen + scan    tl = searchsorted(cum_tlen (LDS), U) clipped to rlen; keep te < p_max; compaction
//   k_file_order     fo0[k] = byte (k & 3) of word k >> 2, & 1  (randint(2, dtype=int8) buffering)
#include <cmath>

#include "mh_internal.h"
#include "mh_scan.h"

namespace mh {

namespace {

constexpr uint32_t MT_UP = 0x80000000u, MT_LO = 0x7fffffffu, MT_A = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
  uint32_t y = (a & MT_UP) | (b & MT_LO);
  return (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}

__device__ void mt_seed_lds(uint32_t *st, uint32_t seed) {
  if (threadIdx.x == 0) {
    uint32_t v = seed;
    st[0] = v;
    for (int i = 1; i < 624; i++) {
      v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
      st[i] = v;
    }
  }
  __syncthreads();
}

// One twist: o (old state) -> nw (new state), calling emit(k, tempered word) for k = 0..623.
// Requires blockDim.x >= 227.
template <typename Emit>
__device__ __forceinline__ void mt_twist_block(const uint32_t *o, uint32_t *nw, Emit emit) {
  const int t = threadIdx.x;
  if (t < 227) {
    uint32_t v = o[t + 397] ^ mt_mix(o[t], o[t + 1]);
    nw[t] = v;
    emit(t, mt_temper(v));
  }
  __syncthreads();
  if (t < 227) {
    int i = 227 + t;
    uint32_t v = nw[i - 227] ^ mt_mix(o[i], o[i + 1]);
    nw[i] = v;
    emit(i, mt_temper(v));
  }
  __syncthreads();
  if (t < 170) {
    int i = 454 + t;
    uint32_t nxt = (i < 623) ? o[i + 1] : nw[0];
    uint32_t v = nw[i - 227] ^ mt_mix(o[i], nxt);
    nw[i] = v;
    emit(i, mt_temper(v));
  }
  __syncthreads();
}

struct MTJob {
  uint32_t *out;
  int64_t count;
  uint32_t seed;
};
struct MTJobs {
  MTJob j[8];
};

__global__ void __launch_bounds__(256) k_mt_streams(MTJobs jobs) {
  __shared__ uint32_t st[2][624];
  const MTJob job = jobs.j[blockIdx.x];
  mt_seed_lds(st[0], job.seed);
  int cur = 0;
  for (int64_t base = 0; base < job.count; base += 624) {
    uint32_t *out = job.out;
    int64_t cnt = job.count;
    mt_twist_block(st[cur], st[cur ^ 1], [&](int k, uint32_t w) {
      if (base + k < cnt) out[base + k] = w;
    });
    cur ^= 1;
  }
}

// ---- Fisher-Yates swap indices -------------------------------------------------------------------------------
constexpr int SD_THREADS = 640;   // 10 waves: one tempered word per thread per twist
constexpr int SD_WAVES = SD_THREADS / 64;

__device__ __forceinline__ uint32_t interval_mask(uint32_t m) {
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
  return m;
}

// j[i] = random_interval(i) for i = n-1 .. 1 (j[0] = 0), MT19937 seeded with `seed`.
__global__ void __launch_bounds__(SD_THREADS) k_shuffle_decode(uint32_t seed, int64_t n, uint32_t *j) {
  __shared__ uint32_t st[2][624];
  __shared__ uint32_t words[624];
  __shared__ int32_t wave_cnt[SD_WAVES];
  __shared__ int64_t s_i0;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) {
    s_i0 = n - 1;
    if (n > 0) j[0] = 0;
  }
  mt_seed_lds(st[0], seed);
  int cur = 0;
  int64_t i0 = n - 1;
  while (i0 >= 1) {
    mt_twist_block(st[cur], st[cur ^ 1], [&](int k, uint32_t w) { words[k] = w; });
    cur ^= 1;
    // decode the 624 words: lane t holds word t; A = accepted words before t in this twist
    const bool have = t < 624;
    const uint32_t w = have ? words[t] : 0u;
    int32_t A = t;   // first guess: everything before accepted (decisions barely depend on A while i0 >> 624)
    bool acc = false;
    uint32_t v = 0;
    bool converged = false;
    for (int it = 0; it < 16; it++) {
      int64_t i = i0 - A;
      acc = have && i >= 1 && ((v = (w & interval_mask((uint32_t)i))) <= (uint32_t)i);
      uint64_t bal = __ballot(acc);
      if (lane == 0) wave_cnt[wave] = __popcll(bal);
      __syncthreads();
      int32_t pre = 0;
      for (int q = 0; q < wave; q++) pre += wave_cnt[q];
      int32_t A2 = pre + (int32_t)__popcll(bal & ((lane ? (~0ull >> (64 - lane)) : 0ull)));
      int same = __syncthreads_and(A2 == A);
      A = A2;
      if (same) { converged = true; break; }
    }
    if (!converged) {
      // exact sequential decode of this twist (rare: only when i0 is comparable to 624)
      if (t == 0) {
        int64_t ii = i0;
        for (int k = 0; k < 624 && ii >= 1; k++) {
          uint32_t vv = words[k] & interval_mask((uint32_t)ii);
          if (vv <= (uint32_t)ii) { j[ii] = vv; ii--; }
        }
        s_i0 = ii;
      }
      __syncthreads();
      i0 = s_i0;
      __syncthreads();
      continue;
    }
    if (acc) j[i0 - A] = v;
    int32_t tot = 0;
    for (int q = 0; q < SD_WAVES; q++) tot += wave_cnt[q];
    i0 -= tot;
    __syncthreads();
  }
}

// ---- permutation from swap indices -------------------------------------------------------------------------
__global__ void k_perm_hist(int64_t n, const uint32_t *j, int32_t *cnt) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  atomicAdd(&cnt[s == 0 ? 0 : j[s]], 1);
}
struct LoadCnt {
  const int32_t *cnt;
  __device__ int64_t operator()(int64_t i) const { return cnt[i]; }
};
struct StoreStart {
  int32_t *start;
  __device__ void operator()(int64_t i, int64_t, int64_t excl) const { start[i] = (int32_t)excl; }
};
__global__ void k_perm_scatter(int64_t n, const uint32_t *j, const int32_t *start, int32_t *fill, int32_t *entries) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint32_t b = s == 0 ? 0 : j[s];
  int32_t slot = atomicAdd(&fill[b], 1);
  entries[start[b] + slot] = (int32_t)s;
}

// Smallest step s' > after in bucket b, or -1.
__device__ __forceinline__ int64_t bucket_next(const int32_t *start, const int32_t *entries, int64_t b,
                                               int64_t after) {
  int64_t best = -1;
  for (int32_t e = start[b]; e < start[b + 1]; e++) {
    int64_t s = entries[e];
    if (s > after && (best < 0 || s < best)) best = s;
  }
  return best;
}

// Fisher-Yates (for i = n-1..1: swap(x[i], x[j_i])) composes to a_final[p] = x[tau_{n-1}(...tau_1(p))] with
// tau_i = (i j_i).  Following p through tau_1, tau_2, ...: nothing moves it before step p; step p sends it to
// j_p; afterwards it moves only when a later step i targets its current slot q (j_i == q), landing on q = i.
// So q = j_p, then repeatedly the smallest later step whose target is the current slot.
__global__ void k_perm_gather(int64_t n, const uint32_t *j, const int32_t *start, const int32_t *entries,
                              const int64_t *ts, int64_t *out) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  int64_t jp = p == 0 ? 0 : j[p];
  int64_t c = bucket_next(start, entries, jp, p);   // smallest step > p that targets j_p
  int64_t q;
  if (c < 0) {
    q = jp;
  } else {
    for (;;) {
      int64_t c2 = bucket_next(start, entries, c, c);
      if (c2 < 0) break;
      c = c2;
    }
    q = c;
  }
  out[p] = ts[q];
}

// ---- geometric + cumsum ------------------------------------------------------------------------------------
__device__ __forceinline__ double mt_double(const uint32_t *w, int64_t k) {
  int32_t a = (int32_t)(w[2 * k] >> 5), b = (int32_t)(w[2 * k + 1] >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

struct GeoFlags {
  int64_t *idx;
  uint32_t *count;
  uint32_t cap;
};

__device__ __forceinline__ int64_t geometric_draw(double U, double p, double log_q, GeoFlags fl, int64_t k) {
  if (p >= 0.333333333333333333333333) {            // numpy legacy_random_geometric_search
    double sum = p, prod = p, q = 1.0 - p;
    int64_t X = 1;
    while (U > sum) { prod *= q; sum += prod; X++; }
    return X;
  }
  double qv = log1p(-U) / log_q;                      // numpy legacy_random_geometric_inversion
  double r = rint(qv);
  if (fabs(qv - r) <= 1e-9 * fmax(1.0, fabs(qv))) {   // ceil() could differ from the host libm: flag
    uint32_t s = atomicAdd(fl.count, 1u);
    if (s < fl.cap) fl.idx[s] = k;
  }
  return (int64_t)ceil(qv);
}

struct LoadGeo {
  const uint32_t *w; double p, log_q; GeoFlags fl;
  __device__ int64_t operator()(int64_t k) const { return geometric_draw(mt_double(w, k), p, log_q, fl, k); }
};
struct LoadArr {
  const int64_t *a;
  __device__ int64_t operator()(int64_t k) const { return a[k]; }
};
__global__ void k_geo_array(int64_t n, const uint32_t *w, double p, double log_q, GeoFlags fl, int64_t *g) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) g[k] = geometric_draw(mt_double(w, k), p, log_q, fl, k);
}
struct StoreTs {
  int64_t *ts; int64_t add;
  __device__ void operator()(int64_t k, int64_t incl, int64_t) const { ts[k] = incl + add; }
};

// ---- template length, compaction, file order ----------------------------------------------------------------
__global__ void __launch_bounds__(256) k_tlen(int64_t n, const uint32_t *w, const double *cum_tlen, int32_t n_tlen,
                                              int64_t rlen, int64_t p_max, const int64_t *ts, int64_t *te,
                                              uint8_t *keep) {
  extern __shared__ __attribute__((aligned(16))) double s_cum[];
  for (int i = threadIdx.x; i < n_tlen; i += blockDim.x) s_cum[i] = cum_tlen[i];
  __syncthreads();
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double u = mt_double(w, k);
  int32_t lo = 0, hi = n_tlen;                        // searchsorted(side='left')
  while (lo < hi) {
    int32_t mid = (lo + hi) >> 1;
    if (s_cum[mid] < u) lo = mid + 1; else hi = mid;
  }
  int64_t tl = lo < rlen ? rlen : lo;                 // tl.clip(rlen)
  int64_t e = ts[k] + tl;
  te[k] = e;
  keep[k] = e < p_max;
}
struct LoadKeep {
  const uint8_t *keep;
  __device__ int64_t operator()(int64_t k) const { return keep[k]; }
};
struct StoreCompact {
  const uint8_t *keep; const int64_t *ts, *te; int64_t *pos0, *pos1; int64_t rlen;
  __device__ void operator()(int64_t k, int64_t, int64_t excl) const {
    if (!keep[k]) return;
    pos0[excl] = ts[k];
    pos1[excl] = te[k] - rlen;
  }
};
__global__ void k_file_order(int64_t m, const uint32_t *w, int8_t *fo0) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < m) fo0[k] = (int8_t)((w[k >> 2] >> (8 * (k & 3))) & 1u);
}

// ---- Philox4x32-10 fast mode ------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}
__global__ void k_philox_words(uint32_t *out, int64_t count, uint64_t key, uint32_t stream) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one uint4 per thread
  if (q * 4 >= count) return;
  uint4 r = philox4x32(make_uint4((uint32_t)q, (uint32_t)(q >> 32), stream, 0x6d697479u),
                       make_uint2((uint32_t)key, (uint32_t)(key >> 32)));
  uint32_t v[4] = {r.x, r.y, r.z, r.w};
  for (int e = 0; e < 4; e++)
    if (q * 4 + e < count) out[q * 4 + e] = v[e];
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
void HostMT::seed(uint32_t s) {
  key[0] = s;
  for (int i = 1; i < 624; i++) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + (uint32_t)i;
  pos = 624;
}
uint32_t HostMT::next() {
  if (pos == 624) {
    int i;
    uint32_t y;
    for (i = 0; i < 624 - 397; i++) {
      y = (key[i] & MT_UP) | (key[i + 1] & MT_LO);
      key[i] = key[i + 397] ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
    }
    for (; i < 623; i++) {
      y = (key[i] & MT_UP) | (key[i + 1] & MT_LO);
      key[i] = key[i + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
    }
    y = (key[623] & MT_UP) | (key[0] & MT_LO);
    key[623] = key[396] ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
    pos = 0;
  }
  uint32_t y = key[pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
double HostMT::next_double() {
  int32_t a = (int32_t)(next() >> 5), b = (int32_t)(next() >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
uint64_t HostMT::interval(uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = max, v;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  if (max <= 0xffffffffull) {
    while ((v = (next() & mask)) > max) {}
  } else {
    while ((v = ((((uint64_t)next()) << 32 | next()) & mask)) > max) {}
  }
  return v;
}

int32_t sample_templates(mh_ctx *ctx, int64_t p_min, int64_t p_max, double p, int32_t rlen, const double *cum_tlen,
                         int32_t n_tlen, uint64_t seed, int32_t rng_mode, int64_t *out_n) {
  if (seed > 0xffffffffull)
    return arg_fail(ctx, MH_E_SEED, "Seed value " + std::to_string(seed) + " is out of range 0 - 4294967295");
  if (n_tlen <= 0 || n_tlen > 8192) return arg_fail(ctx, MH_E_ARG, "cum_tlen must have 1..8192 entries");
  if (rng_mode != MH_RNG_MITTY && rng_mode != MH_RNG_PHILOX) return arg_fail(ctx, MH_E_ARG, "unknown rng_mode");
  hipStream_t st = ctx->stream;
  HostMT sr;
  sr.seed((uint32_t)seed);
  uint32_t s_tloc = (uint32_t)sr.interval(0xfffffffeull), s_tlen = (uint32_t)sr.interval(0xfffffffeull);
  uint32_t s_shuf = (uint32_t)sr.interval(0xfffffffeull), s_fo = (uint32_t)sr.interval(0xfffffffeull);

  int64_t n = (int64_t)((double)(p_max - p_min) * p * 1.2);   // int((p_max - p_min) * p * 1.2)
  if (n < 0) n = 0;
  if (n > ((int64_t)1 << 31) - 2) return arg_fail(ctx, MH_E_ARG, "region too large for one work unit (2^31 draws)");
  const int64_t nn = n > 0 ? n : 1;
  const int64_t n_fo_words = (n + 3) / 4 + 1;

  stage_begin(ctx, "sample");
  // scratch layout: 0 tloc words, 1 tlen words, 2 fo words, 3 j, 4 ts, 5 ts_shuf, 6 te, 7 keep, 8 cnt/fill,
  //                 9 start, 10 entries, 11 geo flags, 12 g (rare path)
  MH_TRY(ensure(ctx, ctx->s[0], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[1], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[2], 4 * n_fo_words));
  MH_TRY(ensure(ctx, ctx->s[3], 4 * nn));
  MH_TRY(ensure(ctx, ctx->s[4], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[5], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[6], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[7], nn));
  MH_TRY(ensure(ctx, ctx->s[8], 4 * (nn + 1)));
  MH_TRY(ensure(ctx, ctx->s[9], 4 * (nn + 1)));
  MH_TRY(ensure(ctx, ctx->s[10], 4 * nn));
  MH_TRY(ensure(ctx, ctx->s[11], 8 * 1024));
  MH_TRY(ensure(ctx, ctx->s[13], 8 * 1024));
  MH_TRY(ensure(ctx, ctx->d_small, 256));
  MH_TRY(ensure(ctx, ctx->scan_partials, 16 * scan_partials_count(nn) + 64));
  MH_TRY(ensure(ctx, ctx->t_pos0, 8 * nn));
  MH_TRY(ensure(ctx, ctx->t_pos1, 8 * nn));
  MH_TRY(ensure(ctx, ctx->t_fo0, nn));
  uint32_t *w_tloc = (uint32_t *)ctx->s[0].p, *w_tlen = (uint32_t *)ctx->s[1].p, *w_fo = (uint32_t *)ctx->s[2].p;
  uint32_t *jarr = (uint32_t *)ctx->s[3].p;
  int64_t *ts = (int64_t *)ctx->s[4].p, *ts_shuf = (int64_t *)ctx->s[5].p, *te = (int64_t *)ctx->s[6].p;
  uint8_t *keep = (uint8_t *)ctx->s[7].p;
  int32_t *cnt = (int32_t *)ctx->s[8].p, *start = (int32_t *)ctx->s[9].p, *entries = (int32_t *)ctx->s[10].p;
  int64_t *flag_idx = (int64_t *)ctx->s[11].p;
  double *d_cum = (double *)ctx->s[13].p;
  char *small = (char *)ctx->d_small.p;
  int64_t *tot = (int64_t *)small;
  uint32_t *flag_cnt = (uint32_t *)(small + 32);
  HIPCHK(ctx, hipMemsetAsync(small, 0, 256, st));
  HIPCHK(ctx, hipMemcpyAsync(d_cum, cum_tlen, 8 * n_tlen, hipMemcpyHostToDevice, st));

  if (n == 0) {
    stage_end(ctx);
    ctx->n_tpl = 0;
    ctx->rlen = rlen;
    ctx->have_tpl = true;
    *out_n = 0;
    return MH_OK;
  }

  // 1. word streams
  if (rng_mode == MH_RNG_MITTY) {
    MTJobs jobs{};
    jobs.j[0] = MTJob{w_tloc, 2 * n, s_tloc};
    jobs.j[1] = MTJob{w_tlen, 2 * n, s_tlen};
    jobs.j[2] = MTJob{w_fo, n_fo_words, s_fo};
    stage_begin(ctx, "sample_mt_streams");
    hipLaunchKernelGGL(k_mt_streams, dim3(3), dim3(256), 0, st, jobs);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    stage_begin(ctx, "sample_shuffle_decode");
    hipLaunchKernelGGL(k_shuffle_decode, dim3(1), dim3(SD_THREADS), 0, st, s_shuf, n, jarr);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  } else {
    uint64_t key = ((uint64_t)s_tloc << 32) | s_tlen;
    hipLaunchKernelGGL(k_philox_words, dim3(grid_for((2 * n + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st, w_tloc,
                       2 * n, key, 1u);
    hipLaunchKernelGGL(k_philox_words, dim3(grid_for((2 * n + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st, w_tlen,
                       2 * n, key, 2u);
    hipLaunchKernelGGL(k_philox_words, dim3(grid_for((n_fo_words + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st, w_fo,
                       n_fo_words, key, 3u);
    HIPCHK(ctx, hipGetLastError());
  }

  // 2. ts = cumsum(geometric) + p_min + 1
  const double log_q = std::log(1.0 - p);
  GeoFlags fl{flag_idx, flag_cnt, 1024};
  stage_begin(ctx, "sample_geometric_scan");
  HIPCHK(ctx, device_scan<int64_t>(st, n, LoadGeo{w_tloc, p, log_q, fl}, StoreTs{ts, p_min + 1}, OpSum{}, (int64_t)0,
                                   (int64_t *)ctx->scan_partials.p, tot));
  stage_end(ctx);
  uint32_t nflag = 0;
  HIPCHK(ctx, hipMemcpyAsync(&nflag, flag_cnt, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (nflag > 0) {
    // rare exact path: materialise the draws, recompute the flagged ones with the host libm, rescan
    MH_TRY(ensure(ctx, ctx->s[12], 8 * nn));
    int64_t *g = (int64_t *)ctx->s[12].p;
    HIPCHK(ctx, hipMemsetAsync(flag_cnt, 0, 4, st));
    hipLaunchKernelGGL(k_geo_array, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, w_tloc, p, log_q, fl, g);
    HIPCHK(ctx, hipMemcpyAsync(&nflag, flag_cnt, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    if (nflag > 1024) {
      stage_end(ctx);
      return arg_fail(ctx, MH_E_ARG, "too many near-integer geometric quotients (p too coarse?)");
    }
    std::vector<int64_t> idx(nflag);
    HIPCHK(ctx, hipMemcpy(idx.data(), flag_idx, 8 * nflag, hipMemcpyDeviceToHost));
    for (int64_t k : idx) {
      uint32_t ww[2];
      HIPCHK(ctx, hipMemcpy(ww, w_tloc + 2 * k, 8, hipMemcpyDeviceToHost));
      double U = (((int32_t)(ww[0] >> 5)) * 67108864.0 + ((int32_t)(ww[1] >> 6))) / 9007199254740992.0;
      int64_t gv = (int64_t)std::ceil(std::log1p(-U) / std::log(1.0 - p));
      HIPCHK(ctx, hipMemcpy(g + k, &gv, 8, hipMemcpyHostToDevice));
    }
    HIPCHK(ctx, device_scan<int64_t>(st, n, LoadArr{g}, StoreTs{ts, p_min + 1}, OpSum{}, (int64_t)0,
                                     (int64_t *)ctx->scan_partials.p, tot));
  }

  // 3. shuffle
  const int64_t *ts_use = ts;
  if (rng_mode == MH_RNG_MITTY && n > 1) {
    stage_begin(ctx, "sample_permutation");
    HIPCHK(ctx, hipMemsetAsync(cnt, 0, 4 * (n + 1), st));
    hipLaunchKernelGGL(k_perm_hist, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, jarr, cnt);
    HIPCHK(ctx, device_scan<int64_t>(st, n + 1, LoadCnt{cnt}, StoreStart{start}, OpSum{}, (int64_t)0,
                                     (int64_t *)ctx->scan_partials.p, tot + 1));
    HIPCHK(ctx, hipMemsetAsync(cnt, 0, 4 * (n + 1), st));
    hipLaunchKernelGGL(k_perm_scatter, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, jarr, start, cnt,
                       entries);
    hipLaunchKernelGGL(k_perm_gather, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, jarr, start, entries,
                       ts, ts_shuf);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    ts_use = ts_shuf;
  }

  // 4. template lengths, keep te < p_max, compaction
  stage_begin(ctx, "sample_tlen_compact");
  hipLaunchKernelGGL(k_tlen, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 8 * n_tlen, st, n, w_tlen, d_cum, n_tlen,
                     (int64_t)rlen, p_max, ts_use, te, keep);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, device_scan<int64_t>(st, n, LoadKeep{keep},
                                   StoreCompact{keep, ts_use, te, (int64_t *)ctx->t_pos0.p, (int64_t *)ctx->t_pos1.p,
                                                (int64_t)rlen},
                                   OpSum{}, (int64_t)0, (int64_t *)ctx->scan_partials.p, tot + 2));
  stage_end(ctx);
  int64_t m = 0;
  HIPCHK(ctx, hipMemcpyAsync(&m, tot + 2, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  // 5. file order
  if (m > 0) {
    hipLaunchKernelGGL(k_file_order, dim3(grid_for(m, 256, INT32_MAX)), dim3(256), 0, st, m, w_fo,
                       (int8_t *)ctx->t_fo0.p);
    HIPCHK(ctx, hipGetLastError());
  }
  stage_end(ctx);
  ctx->n_tpl = m;
  ctx->rlen = rlen;
  ctx->have_tpl = true;
  *out_n = m;
  return MH_OK;
}

}  // namespace mh
