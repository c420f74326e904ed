// mh_sample.hip — template sampling on the device (reference illumina.generate_reads, illumina.py:43-110).
//
// Parity mode (MH_RNG_MITTY) reproduces numpy's legacy RandomState streams word for word.
// Per work unit:  seed -> RS(seed).randint(SEED_MAX, 4) = (tloc, tlen, shuffle, file_order) stream seeds (host).
//   k_mt_segments     every MT19937 stream of every unit in the batch is cut into segments of SEG_WORDS outputs;
//                     one 256-thread workgroup per segment jumps to the segment start (W_J = XOR_{g_k=1} W_k with
//                     g = x^J mod P from mh_jump.cpp, the stream's first 20.6k words built in LDS) and then twists
//                     its segment (three dependency phases of 227/227/170 words) — no sequential chain over a
//                     stream, all segments of all units run at once
//   k_shuffle_decode2 Fisher-Yates swap indices j_i = random_interval(i), i = n-1..1, one 1024-thread workgroup
//                     per unit, 4096 words per step: each thread decides its 4 words given the accepted count
//                     before it, the block fixes that count by iterating scan -> decide to its (unique) fixed
//                     point (2 rounds while i >> 4096; bounded, with an exact sequential fallback)
//   scan(geometric)   ts = cumsum(ceil(log1p(-U)/log(1-p))) + p_min + 1 (numpy legacy inversion, pinned against
//                     numpy), computed inside the scan's Load; quotients within 1e-12 of an integer are flagged
//                     and the unit is redone with those draws recomputed by the host libm
//   k_perm_*          the permutation the swaps produce, without replaying them: steps radix-sorted by target,
//                     then a chase per step (see k_perm_heads)
//   k_tlen + scan     tl = searchsorted(cum_tlen (LDS), U) clipped to rlen; keep te < p_max; compaction
//   file order        fo0[k] = byte (k & 3) of word k >> 2, & 1 (randint(2, dtype=int8) buffering), written
//                     by the compaction's store
// The single-stream decode (k_shuffle_decode: MT19937 fused with the decode in one workgroup) remains as the exact
// fallback for a unit whose decode ran out of pre-generated words.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>


#include "mh_device.h"
#include "mh_internal.h"
#include "mh_scan.h"
#include "mh_sort.h"


namespace mh {

namespace jump {
void jump_poly_words(uint64_t L, int64_t k, uint32_t *out624);
}

namespace {

constexpr uint32_t MT_UP = 0x80000000u, MT_LO = 0x7fffffffu, MT_A = 0x9908b0dfu;
constexpr int64_t SEG_WORDS_DEFAULT = 624 * 640;   // outputs per segment (twice as long: within noise, round 5)
static int64_t seg_words() { return SEG_WORDS_DEFAULT; }

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
  lds_barrier();
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
  lds_barrier();
  if (t < 227) {
    int i = 227 + t;
    uint32_t v = nw[i - 227] ^ mt_mix(o[i], o[i + 1]);
    nw[i] = v;
    emit(i, mt_temper(v));
  }
  lds_barrier();
  if (t < 170) {
    int i = 454 + t;
    uint32_t nxt = (i < 623) ? o[i + 1] : nw[0];
    uint32_t v = nw[i - 227] ^ mt_mix(o[i], nxt);
    nw[i] = v;
    emit(i, mt_temper(v));
  }
  lds_barrier();
}

// ---- jump-ahead segments ---------------------------------------------------------------------------------------
struct SegJob {
  uint32_t *out;      // the stream's output array
  int64_t start;      // first output index of this segment
  int64_t count;      // outputs to produce
  uint32_t seed;
  int32_t k;          // segment index: start = k * SEG_WORDS, jump polynomial polys[k]
};

constexpr int CB_WORDS = 2048;   // circular window of the extended sequence x_i (jump), then the two twist states
constexpr int CB_MASK = CB_WORDS - 1;
constexpr int JW = 208;          // jump lanes: lane w accumulates state words w, w + 208, w + 416
constexpr int CB_ZERO = 2 * CB_WORDS;   // 624 zero words: the target of a batch's unused bit slots
constexpr int JB = 16;                  // set bits per batch of the jump

// The jump W_J[w] = XOR over set bits k of g of x_{k+w} walks the polynomial's bits in increasing k, so x is
// generated 624 words at a time into a 2048-word circular window just ahead of the bits that need it.  The window
// is stored twice (slot s and s + 2048), so x_{k+w}, x_{k+w+208}, x_{k+w+416} sit at (k mod 2048) + w + {0, 208,
// 416} with no wrap: one address add per set bit (the three reads use immediate offsets), and a batch's unused
// bit slots read a zero block instead of being masked out.  26 KB of LDS.
__global__ void __launch_bounds__(256) k_mt_segments(const SegJob *jobs, const uint32_t *polys) {
  __shared__ uint32_t cb[2 * CB_WORDS + 624];
  __shared__ uint32_t gp[624];
  const SegJob job = jobs[blockIdx.x];
  const int t = threadIdx.x;
  mt_seed_lds(cb, job.seed);   // x_0 .. x_623
  if (job.k > 0) {
    const uint32_t *g = polys + (int64_t)job.k * 624;
    for (int i = t; i < 624; i += 256) {
      gp[i] = g[i];
      cb[CB_WORDS + i] = cb[i];   // mirror of x_0 .. x_623
      cb[CB_ZERO + i] = 0u;
    }
    lds_barrier();
    const int w = t < JW ? t : 0;   // lanes >= 208 compute lane 0's words and discard them
    uint32_t a0 = 0, a1 = 0, a2 = 0;
    int32_t G = 624;   // x_0 .. x_{G-1} exist (the last CB_WORDS of them in the window)
    for (int pw = 0; pw < 624; pw++) {
      const int kb = pw * 32;
      // bits kb .. kb+31 read x up to x_{kb+31+623}.  Overwritten slots hold x_{G-2048} .. x_{G-1425}, older than
      // any x still needed (>= x_{kb} >= x_{G-654}) by this or a lagging wave (>= x_{G-1278}).
      while (G <= kb + 31 + 623) {   // G and kb are uniform: every wave takes the same barriers
#pragma unroll
        for (int ph = 0; ph < 3; ph++) {
          if (t < (ph < 2 ? 227 : 170)) {
            const int i = G + 227 * ph + t;
            const uint32_t v = cb[(i - 227) & CB_MASK] ^ mt_mix(cb[(i - 624) & CB_MASK], cb[(i - 623) & CB_MASK]);
            cb[i & CB_MASK] = v;
            cb[(i & CB_MASK) + CB_WORDS] = v;
          }
          lds_barrier();
        }
        G += 624;
      }
      uint32_t m = __builtin_amdgcn_readfirstlane(gp[pw]);   // uniform: the bit walk stays in scalar registers
      const int base = kb & CB_MASK;
      for (int nleft = __builtin_popcount(m); nleft > 0; nleft -= JB) {   // JB set bits per batch: 3 * JB LDS reads
        int off[JB];
#pragma unroll
        for (int u = 0; u < JB; u++) {
          off[u] = u < nleft ? base + __builtin_ctz(m) : CB_ZERO;
          m &= m - 1u;
        }
        uint32_t v0[JB], v1[JB], v2[JB];
#pragma unroll
        for (int u = 0; u < JB; u++) {
          const uint32_t *q = cb + off[u] + w;
          v0[u] = q[0];
          v1[u] = q[JW];
          v2[u] = q[2 * JW];
        }
#pragma unroll
        for (int u = 0; u < JB; u++) {
          a0 ^= v0[u];
          a1 ^= v1[u];
          a2 ^= v2[u];
        }
      }
    }
    lds_barrier();
    if (t < JW) {
      cb[t] = a0;
      cb[t + JW] = a1;
      cb[t + 2 * JW] = a2;
    }
    lds_barrier();
  }
  uint32_t *st0 = cb, *st1 = cb + 624;
  uint32_t *out = job.out + job.start;
  const int64_t cnt = job.count;
  for (int64_t base = 0; base < cnt; base += 624) {
    mt_twist_block(st0, st1, [&](int k, uint32_t w) {
      if (base + k < cnt) out[base + k] = w;
    });
    uint32_t *tmp = st0; st0 = st1; st1 = tmp;
  }
}

// ---- Fisher-Yates swap indices -------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t interval_mask(uint32_t m) {
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
  return m;
}

struct DecJob {
  const uint32_t *words;   // the unit's shuffle stream (tempered outputs)
  int64_t n_words;
  int64_t n;               // draws: i = n-1 .. 1
  uint32_t *j;
  int64_t *status;         // remaining i0 (0 = complete)
};

constexpr int DC_THREADS = 256;
constexpr int DC_WAVES = DC_THREADS / 64;
constexpr int DC_PER = 4;
constexpr int DC_CHUNK = DC_THREADS * DC_PER;

__global__ void __launch_bounds__(DC_THREADS) k_shuffle_decode2(const DecJob *jobs) {
  __shared__ int32_t wsum[DC_WAVES];
  __shared__ int32_t s_tot;
  const DecJob job = jobs[blockIdx.x];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0 && job.n > 0) job.j[0] = 0;
  int64_t i0 = job.n - 1;
  int64_t base = 0;
  float ratio = 0.75f;
  // words of the current chunk; the next chunk's are loaded one step ahead (hides the HBM latency per step)
  uint4 nxt = make_uint4(0, 0, 0, 0);
  if (DC_PER * t + 3 < job.n_words) nxt = *(const uint4 *)(job.words + DC_PER * t);
  while (i0 >= 1 && base < job.n_words) {
    uint32_t w[DC_PER] = {nxt.x, nxt.y, nxt.z, nxt.w};
    bool valid[DC_PER];
#pragma unroll
    for (int e = 0; e < DC_PER; e++) valid[e] = base + DC_PER * t + e < job.n_words;
    {
      const int64_t nb = base + DC_CHUNK + DC_PER * t;
      if (nb + 3 < job.n_words) nxt = *(const uint4 *)(job.words + nb);
    }
    int32_t A = (int32_t)(ratio * (float)(DC_PER * t));
    int32_t cnt = 0;
    uint32_t v[DC_PER];
    bool acc[DC_PER];
    bool converged = false;
    for (int it = 0; it < 24; it++) {
      cnt = 0;
#pragma unroll
      for (int e = 0; e < DC_PER; e++) {
        const int64_t i = i0 - A - cnt;
        v[e] = (i >= 1) ? (w[e] & interval_mask((uint32_t)i)) : 0u;
        acc[e] = valid[e] && i >= 1 && v[e] <= (uint32_t)i;
        cnt += acc[e];
      }
      // exclusive block scan of cnt
      int32_t incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        int32_t o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
      }
      if (lane == 63) wsum[wave] = incl;
      __syncthreads();
      int32_t pre = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < DC_WAVES; q++) {
        const int32_t s = wsum[q];
        pre += q < wave ? s : 0;
        tot += s;
      }
      const int32_t A2 = pre + incl - cnt;
      const int same = __syncthreads_and(A2 == A);
      A = A2;
      if (t == 0) s_tot = tot;
      if (same) {
        converged = true;
        break;
      }
    }
    if (!converged) {
      // exact sequential decode of this chunk (only when i0 is comparable to the chunk size)
      __syncthreads();
      if (t == 0) {
        int64_t ii = i0;
        for (int64_t k = 0; k < DC_CHUNK && base + k < job.n_words && ii >= 1; k++) {
          const uint32_t vv = job.words[base + k] & interval_mask((uint32_t)ii);
          if (vv <= (uint32_t)ii) { job.j[ii] = vv; ii--; }
        }
        s_tot = (int32_t)(i0 - ii);
      }
      __syncthreads();
    } else {
      int32_t a = 0;
#pragma unroll
      for (int e = 0; e < DC_PER; e++) {
        if (acc[e]) job.j[i0 - A - a] = v[e];
        a += acc[e];
      }
    }
    __syncthreads();
    const int32_t tot = s_tot;
    i0 -= tot;
    base += DC_CHUNK;
    ratio = (float)tot / (float)DC_CHUNK;
    __syncthreads();
  }
  if (t == 0) *job.status = i0 < 1 ? 0 : i0;
}

// ---- chunk-parallel decode ---------------------------------------------------------------------------------------
// Every DC_CHUNK-word chunk of every unit's shuffle stream is decoded by its own workgroup, given the draw index i0
// the sequential decode would have at the chunk's first word (start[c]).  Those starts are a prefix sum of the
// chunks' accept counts, which depend on the starts only through words whose masked value lies between a guessed
// and the true i0, so the host iterates count passes (changed chunks only) from an expectation-based guess to the
// fixed point, where every start equals the sequential one; one write pass then emits all swap indices.
struct ChunkJob {
  const uint32_t *words;   // the unit's shuffle stream
  int64_t n_words;
  int64_t base;            // first word of the chunk
  uint32_t *j;             // the unit's swap-index array
  int32_t tail;            // 1: part of the unit's tail (k_decode_tail decodes it; count passes skip it)
  int32_t size;            // words in the chunk (a multiple of 64, at most DC_CHUNK)
};

constexpr int32_t DC_BIG = 1 << 30;

// Per chunk: the accept count and the margin [dlo, dhi]: for every start shift d in it, no accept decision and no
// interval mask of the chunk changes (all i shift by d), so the count stays valid.  dhi = 0 once i reached 0.
template <bool WRITE>
__device__ void decode_chunk(const ChunkJob *jobs, int32_t c, const int64_t *start, int32_t *count, int32_t *margin,
                             int32_t *wsum, int32_t *wlo, int32_t *whi, int32_t &s_tot) {
  const ChunkJob job = jobs[c];
  const int64_t i0 = start[c];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (job.tail) {   // never queued; its count is not needed (the tail follows every bulk chunk of the unit)
    if (!WRITE && t == 0) {
      count[c] = 0;
      margin[2 * c] = -DC_BIG;
      margin[2 * c + 1] = DC_BIG;
    }
    return;
  }
  if (i0 < 1) {
    if (t == 0) {
      count[c] = 0;
      margin[2 * c] = -DC_BIG;
      margin[2 * c + 1] = 0;
    }
    return;
  }
  const int64_t base = job.base;
  uint32_t w[DC_PER];
  bool valid[DC_PER];
  if (base + DC_PER * t + 3 < job.n_words) {
    const uint4 q = *(const uint4 *)(job.words + base + DC_PER * t);
    w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < DC_PER; e++) w[e] = base + DC_PER * t + e < job.n_words ? job.words[base + DC_PER * t + e] : 0u;
  }
#pragma unroll
  for (int e = 0; e < DC_PER; e++) valid[e] = DC_PER * t + e < job.size && base + DC_PER * t + e < job.n_words;
  // first guess of the accepts before this thread's words: the acceptance rate at i0
  const uint32_t m0 = interval_mask((uint32_t)i0);
  int32_t A = (int32_t)((float)(i0 + 1) / ((float)m0 + 1.0f) * (float)(DC_PER * t));
  int32_t cnt = 0;
  uint32_t v[DC_PER];
  bool acc[DC_PER];
  bool converged = false;
  for (int it = 0; it < 24; it++) {
    cnt = 0;
#pragma unroll
    for (int e = 0; e < DC_PER; e++) {
      const int64_t i = i0 - A - cnt;
      v[e] = (i >= 1) ? (w[e] & interval_mask((uint32_t)i)) : 0u;
      acc[e] = valid[e] && i >= 1 && v[e] <= (uint32_t)i;
      cnt += acc[e];
    }
    int32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      int32_t o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int32_t pre = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < DC_WAVES; q++) {
      const int32_t s = wsum[q];
      pre += q < wave ? s : 0;
      tot += s;
    }
    const int32_t A2 = pre + incl - cnt;
    const int same = __syncthreads_and(A2 == A);
    A = A2;
    if (t == 0) s_tot = tot;
    if (same) {
      converged = true;
      break;
    }
  }
  if (!converged) {   // exact sequential decode of the chunk (i0 comparable to the chunk size)
    __syncthreads();
    if (t == 0) {
      int64_t ii = i0;
      int64_t lo = -DC_BIG, hi = DC_BIG;
      for (int64_t k = 0; k < job.size && base + k < job.n_words; k++) {
        if (ii < 1) { hi = 0; break; }
        const uint32_t m = interval_mask((uint32_t)ii);
        const uint32_t vv = job.words[base + k] & m;
        lo = max(lo, (int64_t)(m >> 1) + 1 - ii);
        hi = min(hi, (int64_t)m - ii);
        if (vv <= (uint32_t)ii) {
          lo = max(lo, (int64_t)vv - ii);
          if (WRITE) job.j[ii] = vv;
          ii--;
        } else {
          hi = min(hi, (int64_t)vv - ii - 1);
        }
      }
      count[c] = (int32_t)(i0 - ii);
      margin[2 * c] = (int32_t)lo;
      margin[2 * c + 1] = (int32_t)hi;
    }
    return;
  }
  // margins of this thread's words, then block min / max
  int64_t lo = -DC_BIG, hi = DC_BIG;
  {
    int32_t a = 0;
#pragma unroll
    for (int e = 0; e < DC_PER; e++) {
      if (!valid[e]) continue;
      const int64_t i = i0 - A - a;
      if (i < 1) { hi = 0; continue; }
      const uint32_t m = interval_mask((uint32_t)i);
      lo = max(lo, (int64_t)(m >> 1) + 1 - i);
      hi = min(hi, (int64_t)m - i);
      if (acc[e]) lo = max(lo, (int64_t)v[e] - i); else hi = min(hi, (int64_t)v[e] - i - 1);
      if (WRITE && acc[e]) job.j[i] = v[e];
      a += acc[e];
    }
  }
  int32_t l32 = (int32_t)max(lo, (int64_t)-DC_BIG), h32 = (int32_t)min(hi, (int64_t)DC_BIG);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    l32 = max(l32, __shfl_xor(l32, d, 64));
    h32 = min(h32, __shfl_xor(h32, d, 64));
  }
  if (lane == 0) { wlo[wave] = l32; whi[wave] = h32; }
  __syncthreads();
  if (t == 0) {
    int32_t L = -DC_BIG, H = DC_BIG;
    for (int q = 0; q < DC_WAVES; q++) { L = max(L, wlo[q]); H = min(H, whi[q]); }
    count[c] = s_tot;
    margin[2 * c] = L;
    margin[2 * c + 1] = H;
  }
}

// Chunks todo[0 .. *n_todo) (all chunks when todo == nullptr), strided over the grid; the list and its length are
// device-resident, written by k_decode_resolve, so passes chain on the stream without host round trips.
template <bool WRITE>
__global__ void __launch_bounds__(DC_THREADS) k_decode_chunks(const ChunkJob *jobs, const int32_t *todo,
                                                              const int32_t *n_todo, int32_t n_all,
                                                              const int64_t *start, int32_t *count,
                                                              int32_t *margin) {
  __shared__ int32_t wsum[DC_WAVES];
  __shared__ int32_t wlo[DC_WAVES], whi[DC_WAVES];
  __shared__ int32_t s_tot;
  const int32_t n = todo ? *n_todo : n_all;
  for (int32_t i = blockIdx.x; i < n; i += gridDim.x) {
    decode_chunk<WRITE>(jobs, todo ? todo[i] : i, start, count, margin, wsum, wlo, whi, s_tot);
    __syncthreads();
  }
}

// After a count pass: per unit, the starts the counts imply (s = n - 1 - accepts before the chunk), and the chunks
// whose count was taken at a start outside their margin, which are queued for the next pass at the implied start.
// Tiles of up to DR_TILE chunks never cross a unit; k_decode_resolve (one workgroup per tile) adds the unit's earlier
// tiles as its carry.
constexpr int DR_THREADS = 256, DR_PER = 8, DR_TILE = DR_THREADS * DR_PER;
struct DecTile {
  int32_t unit, begin, end, first_tile;   // chunks [begin, end); first_tile = the unit's first tile index
};

__device__ __forceinline__ int64_t block_sum_dr(int64_t v, int64_t *wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if (lane == 0) wsum[wave] = v;
  __syncthreads();
  int64_t tot = 0;
#pragma unroll
  for (int q = 0; q < DR_THREADS / 64; q++) tot += wsum[q];
  return tot;
}

// One launch per pass: every tile sums its unit's earlier tiles itself (a unit spans a few tiles), appends the chunks
// to requeue to *n_todo, and zeroes *n_next, the counter the next pass appends to (the two alternate by pass).
__global__ void __launch_bounds__(DR_THREADS) k_decode_resolve(const DecTile *tiles, const int64_t *n_draws,
                                                               const int32_t *count, const int32_t *margin,
                                                               int64_t *s0, int64_t *s1, int32_t *todo,
                                                               int32_t *n_todo, int32_t *n_next, int64_t *rem) {
  __shared__ int64_t wsum[DR_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const DecTile tl = tiles[blockIdx.x];
  if (blockIdx.x == 0 && t == 0) *n_next = 0;
  int64_t before = 0;
  for (int32_t k = tl.first_tile; k < (int32_t)blockIdx.x; k++) {   // every load of a tile issued back to back
    const int32_t b = tiles[k].begin + t * DR_PER, e = tiles[k].end;
    int32_t cb[DR_PER];
#pragma unroll
    for (int q = 0; q < DR_PER; q++) cb[q] = b + q < e ? count[b + q] : 0;
#pragma unroll
    for (int q = 0; q < DR_PER; q++) before += cb[q];
  }
  const int64_t carry = n_draws[tl.unit] - 1 - block_sum_dr(before, wsum);
  __syncthreads();   // wsum is reused by the scan below
  const int32_t c0 = tl.begin + t * DR_PER;
  int32_t cv[DR_PER];
  int64_t loc = 0;
#pragma unroll
  for (int k = 0; k < DR_PER; k++) {
    cv[k] = c0 + k < tl.end ? count[c0 + k] : 0;
    loc += cv[k];
  }
  int64_t incl = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int64_t pre = 0;
#pragma unroll
  for (int q = 0; q < DR_THREADS / 64; q++) pre += q < wave ? wsum[q] : 0;
  int64_t s = carry - (pre + incl - loc);
  // every load first, then one queue append per wave (an atomic round trip per chunk would serialise the kernel)
  int64_t o0[DR_PER];
  int32_t mlo[DR_PER], mhi[DR_PER];
#pragma unroll
  for (int k = 0; k < DR_PER; k++) {
    const int32_t c = c0 + k < tl.end ? c0 + k : tl.begin;
    o0[k] = s0[c];
    mlo[k] = margin[2 * c];
    mhi[k] = margin[2 * c + 1];
  }
  uint32_t rq = 0;
#pragma unroll
  for (int k = 0; k < DR_PER; k++) {
    const int32_t c = c0 + k;
    if (c < tl.end) {
      const int64_t sv = s > 0 ? s : 0;
      s1[c] = sv;
      const int64_t d = sv - o0[k];
      if (d < mlo[k] || d > mhi[k]) {
        s0[c] = sv;
        rq |= 1u << k;
      }
    }
    s -= cv[k];
  }
  const int32_t nrq = __popc(rq);
  int32_t rincl = nrq;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t o = __shfl_up(rincl, d, 64);
    if (lane >= d) rincl += o;
  }
  const int32_t wtot = __shfl(rincl, 63, 64);
  if (wtot > 0) {
    int32_t q0 = 0;
    if (lane == 63) q0 = atomicAdd(n_todo, wtot);
    q0 = __shfl(q0, 63, 64) + rincl - nrq;
#pragma unroll
    for (int k = 0; k < DR_PER; k++)
      if (rq & (1u << k)) todo[q0++] = c0 + k;
  }
  // the unit's last tile: draws left after its last chunk
  if (t == DR_THREADS - 1 && (blockIdx.x + 1 == gridDim.x || tiles[blockIdx.x + 1].unit != tl.unit)) {
    const int64_t left = carry - (pre + incl);
    rem[tl.unit] = left < 1 ? 0 : left;
  }
}

// ---- the tail: a unit's last draws (small i) ----------------------------------------------------------------------
// Below a few ten thousand draws a chunk's margin is a handful of draws, so every correction upstream requeues it and
// the count passes would keep running for the tail alone.  Instead the tail is excluded from the passes and decoded
// here once the bulk has converged: one wave per unit walks the words 256 at a time (4 per lane) from the exact start.
// Within a step, lane k's words start at draw index i - A_k with A_k = accepts of lanes < k; A is iterated to its fixed
// point, which is the sequential solution (lane k is exact after k + 1 iterations, so at most 65 iterations).
struct TailJob {
  const uint32_t *words;
  int64_t n_words;
  int64_t base;           // first word of the tail
  const int64_t *start;   // exact draw index at `base` (s1 of the unit's first tail chunk)
  uint32_t *j;
  int64_t *status;        // draws left undecoded (0 = complete)
};

constexpr int DT_PER = 4;                 // words per lane per step
constexpr int DT_STEP = 64 * DT_PER;

__device__ __forceinline__ void tail_load(const TailJob &job, int64_t at, uint32_t (&w)[DT_PER]) {
  if (at + DT_PER <= job.n_words) {
    const uint4 q = *(const uint4 *)(job.words + at);   // stream and tail bases are 16-byte aligned
    w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < DT_PER; e++) w[e] = at + e < job.n_words ? job.words[at + e] : 0u;
  }
}

// One 256-word step from draw index i at word pos; false if the fixed point was not reached (cannot happen).
// Lane counts are 0..4, so their exclusive prefix is three ballots' bit-plane popcounts.
__device__ __forceinline__ bool tail_step(const TailJob &job, int64_t &i, int64_t pos, const uint32_t (&w)[DT_PER],
                                          int lane, uint64_t below) {
  const int64_t at = pos + DT_PER * lane;
  const uint32_t m0 = interval_mask((uint32_t)min(i, (int64_t)0xFFFFFFFF));
  int32_t A = (int32_t)((float)(i + 1) / ((float)m0 + 1.0f) * (float)(DT_PER * lane));
  uint32_t v[DT_PER];
  bool acc[DT_PER];
  for (int it = 0; it < 66; it++) {
    int32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < DT_PER; e++) {
      const int64_t ii = i - A - cnt;
      v[e] = ii >= 1 ? (w[e] & interval_mask((uint32_t)ii)) : 0u;
      acc[e] = at + e < job.n_words && ii >= 1 && v[e] <= (uint32_t)ii;
      cnt += acc[e];
    }
    const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
    const int32_t A2 = (int32_t)(__popcll(b0 & below) + 2 * __popcll(b1 & below) + 4 * __popcll(b2 & below));
    if (__ballot(A2 != A) == 0) {
      int32_t a = 0;
#pragma unroll
      for (int e = 0; e < DT_PER; e++) {
        if (acc[e]) job.j[i - A - a] = v[e];
        a += acc[e];
      }
      i -= (int64_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
      return true;
    }
    A = A2;
  }
  return false;
}

// Words are prefetched DT_RING steps ahead (a register ring, unrolled so every index is static).
constexpr int DT_RING = 4;

__global__ void __launch_bounds__(64) k_decode_tail(const TailJob *jobs) {
  const TailJob job = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int64_t i = *job.start;
  int64_t pos = job.base;
  uint32_t w[DT_RING][DT_PER];
#pragma unroll
  for (int r = 0; r < DT_RING; r++) tail_load(job, pos + (int64_t)r * DT_STEP + DT_PER * lane, w[r]);
  bool ok = true;
  while (ok && i >= 1 && pos < job.n_words) {
#pragma unroll
    for (int r = 0; r < DT_RING; r++) {
      if (!(ok && i >= 1 && pos < job.n_words)) break;
      ok = tail_step(job, i, pos, w[r], lane, below);
      tail_load(job, pos + (int64_t)DT_RING * DT_STEP + DT_PER * lane, w[r]);
      pos += DT_STEP;
    }
  }
  // !ok cannot happen; i != 0 then sends the unit to the exact sequential decode
  if (lane == 0) *job.status = i < 1 ? 0 : i;
}

// Sequential-stream variant (exact fallback): MT19937 in LDS fused with the decode, one 640-thread workgroup.
constexpr int SD_THREADS = 640;
constexpr int SD_WAVES = SD_THREADS / 64;

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
    const bool have = t < 624;
    const uint32_t w = have ? words[t] : 0u;
    int32_t A = t;
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
// Fisher-Yates (for i = n-1..1: swap(x[i], x[j_i]), j_i <= i) composes to a_final[p] = x[sigma(p)], sigma =
// tau_{n-1} o ... o tau_1 with tau_i = (i j_i).  Following p through tau_1, tau_2, ...: nothing moves it before
// step p; step p sends it to slot j_p; afterwards it moves only when a later step i targets its current slot c,
// landing on slot i.  With the steps sorted by (target, step) — one radix sort of j with the step index as value —
// the first move after step p is the next entry of p's bucket, and every move after that is
// next(c) = the smallest step > c targeting c = the head of bucket c (or the one after it when step c targeted
// itself).  So sigma(p) = the end of the chain first(p), next(.), next(.), ... or j_p when p's bucket has no later
// step.  (j_0 = 0: step 0 is a self-swap, which the sort places first in bucket 0.)
__global__ void __launch_bounds__(256) k_perm_heads(int64_t n, const uint32_t *K, const uint32_t *V, int32_t *nxt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t b = K[k];
  if (k > 0 && K[k - 1] == b) return;
  int32_t s = (int32_t)V[k];
  if ((uint32_t)s == b) s = (k + 1 < n && K[k + 1] == b) ? (int32_t)V[k + 1] : -1;   // step b: not later than b
  nxt[b] = s;   // buckets without a head keep the -1 of the memset
}

// sorted entries [k0, n): one unit's range of the batch sort (its keys are its own: K[n] starts another unit) or all
__global__ void __launch_bounds__(256) k_perm_chase(int64_t k0, int64_t n, const uint32_t *K, const uint32_t *V,
                                                    const int32_t *nxt, const int64_t *ts, int64_t *out) {
  const int64_t k = k0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t b = K[k], p = V[k];
  int64_t q = b;
  if (k + 1 < n && K[k + 1] == b) {
    int32_t c = (int32_t)V[k + 1], d;
    while ((d = nxt[c]) >= 0) c = d;
    q = c;
  }
  out[p] = ts[q];
}

// The batch-wide permutation: every unit of a batch in one sort.  Unit u's step k sits at global index
// j_off(u) + k and targets j_off(u) + j_k, so the units' buckets stay apart and one sort, one heads pass and one
// chase serve them all (per-unit sorts of a whole-genome job were ~100 small sorts, each a handful of launches).
// Padding entries between units target themselves (an empty chain).  Also sets every head to -1 (k_perm_heads
// then writes the buckets that have one).
constexpr int PK_UNITS = 512;   // units per batch staged in LDS
__global__ void __launch_bounds__(256) k_perm_keys(int64_t total, const uint32_t *jall, const int64_t *u_off,
                                                   const int64_t *u_n, int32_t n_units, uint32_t *keys,
                                                   int32_t *nxt) {
  __shared__ int64_t s_off[PK_UNITS], s_n[PK_UNITS];
  for (int i = threadIdx.x; i < n_units; i += 256) {
    s_off[i] = u_off[i];
    s_n[i] = u_n[i];
  }
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  int lo = 0, hi = n_units - 1;   // the last unit whose offset is <= g
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_off[mid] <= g) lo = mid; else hi = mid - 1;
  }
  const int64_t k = g - s_off[lo];
  keys[g] = k < s_n[lo] ? (uint32_t)(s_off[lo] + jall[g]) : (uint32_t)g;
  nxt[g] = -1;
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
  if (fabs(qv - r) <= 1e-12 * fmax(1.0, fabs(qv))) {  // ceil() could differ from the host libm: flag
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
struct StoreTs {   // ts = cumsum + p_min + 1, with its start node packed in (NodeIdx, mh_internal.h) when known
  int64_t *ts; int64_t add; NodeIdx ni;
  __device__ void operator()(int64_t k, int64_t incl, int64_t) const { ts[k] = ts_pack(ni, incl + add); }
};

// ---- template length, compaction, file order ----------------------------------------------------------------
constexpr int TLEN_PER = 8;
__global__ void __launch_bounds__(256) k_tlen(int64_t n, const uint32_t *w, const double *cum_tlen, int32_t n_tlen,
                                              int64_t rlen, int64_t p_max, const int64_t *ts, int64_t *te,
                                              uint8_t *keep) {
  extern __shared__ __attribute__((aligned(16))) double s_cum[];
  for (int i = threadIdx.x; i < n_tlen; i += blockDim.x) s_cum[i] = cum_tlen[i];
  __syncthreads();
  // TLEN_PER draws per thread (lane-strided): the table is staged once per TLEN_PER * 256 draws
  for (int q = 0; q < TLEN_PER; q++) {
    const int64_t k = ((int64_t)blockIdx.x * TLEN_PER + q) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double u = mt_double(w, k);
    int32_t lo = 0, hi = n_tlen;                        // searchsorted(side='left')
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (s_cum[mid] < u) lo = mid + 1; else hi = mid;
    }
    const int64_t tl = lo < rlen ? rlen : lo;           // tl.clip(rlen)
    const int64_t e = (ts[k] & TS_POS_MASK) + tl;
    te[k] = e;
    keep[k] = e < p_max;
  }
}
struct LoadKeep {
  const uint8_t *keep;
  __device__ int64_t operator()(int64_t k) const { return keep[k]; }
};
// the kept template's place excl: its positions, and its file-order bit (fo0[k] = byte (k & 3) of word k >> 2, & 1:
// randint(2, dtype=int8) buffering, illumina.py:80 — the k-th kept template takes the k-th draw)
struct StoreCompact {
  const uint8_t *keep; const int64_t *ts, *te; int64_t *pos0, *pos1; int64_t rlen;
  const uint32_t *wfo; int8_t *fo0;
  int32_t *n0;   // mate 0's start node, unpacked from ts (null: the set keeps none)
  __device__ void operator()(int64_t k, int64_t, int64_t excl) const {
    if (!keep[k]) return;
    const int64_t v = ts[k];
    pos0[excl] = v & TS_POS_MASK;
    if (n0) n0[excl] = (int32_t)(v >> TS_NODE_SHIFT) - 1;
    pos1[excl] = te[k] - rlen;
    fo0[excl] = (int8_t)((wfo[excl >> 2] >> (8 * (excl & 3))) & 1u);
  }
};

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

// ---- host-side planning ---------------------------------------------------------------------------------------
// Expected MT words consumed by the shuffle's n-1 random_interval draws, plus a wide margin.
int64_t shuffle_words_alloc(int64_t n) {
  if (n <= 1) return DC_CHUNK;
  double E = 0.0;
  // draws i in [a, b] share mask M (i in [2^(k-1), 2^k - 1], M = 2^k): sum M/(i+1) = M (H(b+1) - H(a))
  auto H = [](double x) { return x < 20 ? 0.0 : std::log(x) + 0.5772156649015329 + 1.0 / (2 * x) - 1.0 / (12 * x * x); };
  for (int64_t a = 1; a <= n - 1; a *= 2) {
    int64_t b = std::min(2 * a - 1, n - 1);
    double M = (double)(2 * a);
    if (b < 64) {
      for (int64_t i = a; i <= b; i++) E += M / (double)(i + 1);
    } else {
      E += M * (H((double)(b + 1)) - H((double)a));
    }
  }
  double sd = 2.0 * std::sqrt((double)n);
  int64_t w = (int64_t)(E + 12.0 * sd) + 2 * DC_CHUNK;
  return ((w + DC_CHUNK - 1) / DC_CHUNK) * DC_CHUNK;
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

namespace {

// jump polynomials x^(k * seg) mod P, k = 0..kmax (cached on host and device)
int32_t ensure_polys(mh_ctx *ctx, hipStream_t st, int64_t kmax, int64_t seg) {
  if (ctx->jump_k >= kmax + 1 && ctx->jump_seg == seg) return MH_OK;
  std::vector<uint32_t> polys((size_t)(kmax + 1) * 624);
  for (int64_t k = 0; k <= kmax; k++) jump::jump_poly_words((uint64_t)seg, k, polys.data() + k * 624);
  MH_TRY(ensure(ctx, ctx->jump_polys, 4 * polys.size()));
  HIPCHK(ctx, hipMemcpyAsync(ctx->jump_polys.p, polys.data(), 4 * polys.size(), hipMemcpyHostToDevice, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  ctx->jump_k = kmax + 1;
  ctx->jump_seg = seg;
  return MH_OK;
}

// The stream continued from an explicit state (numpy's get_state(): raw key, pos): one workgroup, twist by twist.
__global__ void __launch_bounds__(256) k_mt_state(const uint32_t *key, int32_t pos, int64_t count, uint32_t *out) {
  __shared__ uint32_t st[2][624];
  for (int i = threadIdx.x; i < 624; i += 256) st[0][i] = key[i];
  lds_barrier();
  const int64_t lead = 624 - pos;   // outputs left in the current state
  for (int64_t i = threadIdx.x; i < lead && i < count; i += 256) out[i] = mt_temper(st[0][pos + i]);
  uint32_t *o = st[0], *nw = st[1];
  for (int64_t base = lead; base < count; base += 624) {
    mt_twist_block(o, nw, [&](int k, uint32_t w) {
      if (base + k < count) out[base + k] = w;
    });
    uint32_t *tmp = o; o = nw; nw = tmp;
  }
}

}  // namespace

int32_t mt_stream_words(mh_ctx *ctx, hipStream_t st, uint32_t seed, int64_t first, int64_t count, DevBuf &out,
                        DevBuf &jobs_buf, int64_t *lead) {
  const int64_t SEG = seg_words();
  const int64_t k0 = first / SEG, k1 = (first + std::max<int64_t>(count, 1) - 1) / SEG;
  *lead = first - k0 * SEG;
  MH_TRY(ensure(ctx, out, 4 * (size_t)((k1 - k0 + 1) * SEG) + 64));
  std::vector<SegJob> jobs;
  for (int64_t k = k0; k <= k1; k++)
    jobs.push_back(SegJob{(uint32_t *)out.p, (k - k0) * SEG, std::min(SEG, first + count - k * SEG), seed, (int32_t)k});
  MH_TRY(ensure_polys(ctx, st, k1, SEG));
  MH_TRY(ensure(ctx, jobs_buf, sizeof(SegJob) * jobs.size() + 64));
  HIPCHK(ctx, hipMemcpyAsync(jobs_buf.p, jobs.data(), sizeof(SegJob) * jobs.size(), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_mt_segments, dim3((unsigned)jobs.size()), dim3(256), 0, st, (const SegJob *)jobs_buf.p,
                     (const uint32_t *)ctx->jump_polys.p);
  HIPCHK(ctx, hipGetLastError());
  SYNCCHK(ctx, hipStreamSynchronize(st));   // the host job table goes out of scope
  return MH_OK;
}

int32_t mt_state_words(mh_ctx *ctx, hipStream_t st, const uint32_t *key624, int32_t pos, int64_t count, DevBuf &out,
                       DevBuf &key_buf) {
  if (pos < 0 || pos > 624) return arg_fail(ctx, MH_E_ARG, "MT19937 state position outside 0..624");
  MH_TRY(ensure(ctx, out, 4 * (size_t)count + 64));
  MH_TRY(ensure(ctx, key_buf, 4 * 624));
  HIPCHK(ctx, hipMemcpyAsync(key_buf.p, key624, 4 * 624, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_mt_state, dim3(1), dim3(256), 0, st, (const uint32_t *)key_buf.p, pos, count,
                     (uint32_t *)out.p);
  HIPCHK(ctx, hipGetLastError());
  SYNCCHK(ctx, hipStreamSynchronize(st));   // key624 is the caller's host memory
  return MH_OK;
}

namespace {

struct UnitPlan {
  NodeIdx ni;   // the unit's haplotype nodes (start nodes packed into ts), or none
  int64_t p_min, p_max, n, n_fo_words, n_shuf_words;
  uint32_t s_tloc, s_tlen, s_shuf, s_fo;
  int64_t w_tloc, w_tlen, w_fo, w_shuf;   // word offsets in the batch word buffer
  int64_t j_off;                          // offset in the batch j buffer
  TplSet *out;
};

// Chunk-parallel Fisher-Yates decode of every unit in `dec` (see k_decode_chunks).  On success the swap indices are
// written and d_status[u] = draws left undecoded (0 unless the unit ran out of pre-generated words); *done = false
// when the starts did not reach their fixed point within the pass budget (the caller then runs k_shuffle_decode2).
int32_t decode_parallel(mh_ctx *ctx, const std::vector<DecJob> &dec, int64_t *d_status, bool *done) {
  hipStream_t st = ctx->stream;
  *done = false;
  // Chunks shrink with the draw index: a chunk's margin (in draws) is about mask(i) / its words, so sizing chunks as
  // i / 128 words (a power of two, 64 .. DC_CHUNK) keeps margins from collapsing as i falls.
  // Starts: the exact one for each unit's first chunk, then the expected accepts (rate (i+1)/(mask+1)).
  const int64_t div = 128;
  const int64_t minw = 64;
  std::vector<ChunkJob> cj;
  std::vector<int64_t> s0;
  std::vector<int32_t> first(dec.size() + 1, 0);
  for (size_t u = 0; u < dec.size(); u++) {
    first[u] = (int32_t)cj.size();
    double i = (double)(dec[u].n - 1);
    for (int64_t b = 0; b < dec[u].n_words;) {
      int64_t size = DC_CHUNK;
      while (size > minw && (double)size * (double)div > i) size >>= 1;
      cj.push_back(ChunkJob{dec[u].words, dec[u].n_words, b, dec[u].j, 0, (int32_t)size});
      s0.push_back(b == 0 ? dec[u].n - 1 : (i >= 1.0 ? (int64_t)llround(i) : 0));
      double rem = (double)size;
      while (rem > 0 && i >= 1.0) {   // integrate the acceptance rate piecewise over mask epochs
        uint32_t ii = (uint32_t)i, m = ii;
        m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
        const double rate = (i + 1.0) / ((double)m + 1.0);
        const double lo = (double)((m >> 1) + 1);              // i stays in this epoch while i >= lo
        const double need = (i - lo + 1.0) / rate;             // words to leave the epoch
        if (need >= rem) { i -= rem * rate; rem = 0; }
        else { i = lo - 1.0; rem -= need; }
      }
      b += size;
    }
  }
  first[dec.size()] = (int32_t)cj.size();
  const int64_t C = (int64_t)cj.size();
  if (C == 0) {
    *done = true;
    return MH_OK;
  }
  const int32_t U = (int32_t)dec.size();
  // the tail of each unit: its chunks from the first one expected to start below 2^15 draws
  const int64_t tail_at = (int64_t)1 << 15;
  std::vector<int32_t> tail_c(U, -1);
  for (int32_t u = 0; u < U; u++)
    for (int32_t c = first[u]; c < first[u + 1] && tail_at > 0; c++)
      if (s0[c] < tail_at) {
        tail_c[u] = c;
        for (int32_t k = c; k < first[u + 1]; k++) cj[k].tail = 1;
        break;
      }
  const int32_t tile_sz = DR_TILE;
  std::vector<DecTile> tiles;
  for (int32_t u = 0; u < U; u++) {
    const int32_t ft = (int32_t)tiles.size();
    for (int32_t b = first[u]; b < first[u + 1]; b += tile_sz)
      tiles.push_back(DecTile{u, b, std::min(b + tile_sz, first[u + 1]), ft});
  }
  const int32_t T = (int32_t)tiles.size();
  const size_t bytes = ((sizeof(ChunkJob) * C + 15) / 16) * 16 + 8 * C * 2 + 8 * U * 2 + sizeof(TailJob) * U +
                       sizeof(DecTile) * (T + 1) + 4 * C * 2 + 8 * C + 512;
  MH_TRY(ensure(ctx, ctx->dec_buf, bytes));
  char *p = (char *)ctx->dec_buf.p;
  ChunkJob *d_jobs = (ChunkJob *)p;
  int64_t *d_s0 = (int64_t *)(p + ((sizeof(ChunkJob) * C + 15) / 16) * 16);
  int64_t *d_s1 = d_s0 + C;
  int64_t *d_ndraw = d_s1 + C;
  int64_t *d_rem = d_ndraw + U;
  TailJob *d_tail = (TailJob *)(d_rem + U);
  DecTile *d_tiles = (DecTile *)(d_tail + U);
  int32_t *d_count = (int32_t *)(d_tiles + T + 1);
  int32_t *d_todo = d_count + C;
  int32_t *d_margin = d_todo + C;
  int32_t *d_ntodo = d_margin + 2 * C;   // two queue counters, alternating by pass
  std::vector<int64_t> ndraw(U);
  for (int32_t u = 0; u < U; u++) ndraw[u] = dec[u].n;
  std::vector<TailJob> tj;
  for (int32_t u = 0; u < U; u++)
    if (tail_c[u] >= 0 && dec[u].n > 0)
      tj.push_back(TailJob{dec[u].words, dec[u].n_words, cj[tail_c[u]].base, d_s1 + tail_c[u], dec[u].j, dec[u].status});
  HIPCHK(ctx, hipMemcpyAsync(d_jobs, cj.data(), sizeof(ChunkJob) * C, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_s0, s0.data(), 8 * C, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_tiles, tiles.data(), sizeof(DecTile) * T, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_ndraw, ndraw.data(), 8 * U, hipMemcpyHostToDevice, st));
  if (!tj.empty()) HIPCHK(ctx, hipMemcpyAsync(d_tail, tj.data(), sizeof(TailJob) * tj.size(), hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemsetAsync(d_ntodo, 0, 8, st));
  const unsigned grid = (unsigned)std::min<int64_t>(C, 4096);
  // pass 1 over every chunk, then passes over the queued chunks (resolve + recount), PASS_BATCH per host check
  constexpr int MAX_PASSES = 64;
  // one host check per 24 passes (the decode converges in ~22): a host round trip per 8 passes had cost 0.9 % of the
  // WGS step (round 5's A/B); the passes after convergence find an empty queue
  const int PASS_BATCH = 24;
  hipLaunchKernelGGL(k_decode_chunks<false>, dim3(grid), dim3(DC_THREADS), 0, st, (const ChunkJob *)d_jobs,
                     (const int32_t *)nullptr, (const int32_t *)nullptr, (int32_t)C, (const int64_t *)d_s0, d_count,
                     d_margin);
  HIPCHK(ctx, hipGetLastError());
  bool conv = false;
  int passes = 1;
  while (passes < MAX_PASSES) {
    int32_t *cur = d_ntodo;
    for (int k = 0; k < PASS_BATCH; k++, passes++) {
      cur = d_ntodo + (passes & 1);
      int32_t *nxt = d_ntodo + ((passes + 1) & 1);
      // the queue shrinks fast: a smaller grid once the first passes are done
      const unsigned g = passes < 4 ? grid : std::min(grid, 1024u);
      hipLaunchKernelGGL(k_decode_resolve, dim3(T), dim3(DR_THREADS), 0, st, (const DecTile *)d_tiles,
                         (const int64_t *)d_ndraw, (const int32_t *)d_count, (const int32_t *)d_margin, d_s0, d_s1,
                         d_todo, cur, nxt, d_rem);
      hipLaunchKernelGGL(k_decode_chunks<false>, dim3(g), dim3(DC_THREADS), 0, st, (const ChunkJob *)d_jobs,
                         (const int32_t *)d_todo, (const int32_t *)cur, (int32_t)C, (const int64_t *)d_s0, d_count,
                         d_margin);
    }
    HIPCHK(ctx, hipGetLastError());
    int64_t *hs = pinned_small(ctx);
    if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
    HIPCHK(ctx, hipMemcpyAsync(hs + 32, cur, 4, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    const int32_t h_ntodo = (int32_t)(hs[32] & 0xffffffff);
    if (h_ntodo == 0) {   // the last pass counted nothing: the starts in s1 are the sequential ones
      conv = true;
      break;
    }
  }
  ctx->dec_passes = passes;
  if (!conv) return MH_OK;
  // every bulk start exact now: the write pass, the tails from their exact starts, and draws left per unit (0 unless
  // a unit ran out of words; a unit with a tail gets it from k_decode_tail)
  hipLaunchKernelGGL(k_decode_chunks<true>, dim3(grid), dim3(DC_THREADS), 0, st, (const ChunkJob *)d_jobs,
                     (const int32_t *)nullptr, (const int32_t *)nullptr, (int32_t)C, (const int64_t *)d_s1, d_count,
                     d_margin);
  HIPCHK(ctx, hipGetLastError());
  for (int32_t u = 0; u < U; u++)
    if (dec[u].n > 0 && tail_c[u] < 0) HIPCHK(ctx, hipMemcpyAsync(dec[u].status, d_rem + u, 8, hipMemcpyDeviceToDevice, st));
  if (!tj.empty()) {
    hipLaunchKernelGGL(k_decode_tail, dim3((unsigned)tj.size()), dim3(64), 0, st, (const TailJob *)d_tail);
    HIPCHK(ctx, hipGetLastError());
  }
  // j[0] = 0 (the shuffle's unused slot), as k_shuffle_decode2 sets it
  for (size_t u = 0; u < dec.size(); u++)
    if (dec[u].n > 0) HIPCHK(ctx, hipMemsetAsync(dec[u].j, 0, 4, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  *done = true;
  return MH_OK;
}

// Everything after the word streams for one unit: ts (geometric scan), shuffle, tlen + keep + compaction into
// `out`, file order.  `exact`: materialise the draws and recompute flagged ones on the host (rare path).
// `lane` 1 runs on the second sampling stream with its own scratch (the units' stages are latency-bound, so two
// units side by side fill the chip better than one after the other).
// phase: 0 = everything; 1 = the geometric scan (and a per-unit sort); 2 = the rest.
// bp (the batch-wide permutation): phase 1 writes the unit's ts into bp_ts + j_off, phase 2 takes its shuffled ts
// from bp_tsh + j_off; the unit's own sort and chase are skipped
// The permutation's (target, step) sort: the hand-written LSD radix sort of mh_sort.h (9-bit digits with the tile
// counts folded into the scatter: a 64 M-draw batch's 27-bit keys in 3 passes, 512-thread workgroups that fit beside
// the FASTQ writers; round 5's A/B against rocprim's onesweep: within noise).
template <class KIn>
static hipError_t perm_sort(void *tmp, size_t &tmp_bytes, KIn keys_in, uint32_t *keys_out, uint32_t *vals_out,
                            size_t n, unsigned end_bit, hipStream_t st) {
  return lsd_sort_pairs_iota(tmp, tmp_bytes, keys_in, keys_out, vals_out, (int64_t)n, end_bit, st);
}

struct BatchPerm {
  int64_t *ts, *tsh;
};

int32_t finish_unit(mh_ctx *ctx, UnitPlan &u, const uint32_t *words, const uint32_t *jarr, double p, int32_t rlen,
                    const double *d_cum, int32_t n_tlen, int32_t rng_mode, bool exact, int64_t *d_m,
                    uint32_t *d_flag, int lane = 0, int phase = 0, const BatchPerm *bp = nullptr) {
  hipStream_t st = lane == 0 ? ctx->stream : lane == 1 ? ctx->stream2 : ctx->xstream[lane - 2];
  ctx->stage_stream = lane ? st : nullptr;
  struct Restore {
    mh_ctx *c;
    ~Restore() { c->stage_stream = nullptr; }
  } restore{ctx};
  mh::DevBuf *S4 = lane == 0 ? ctx->s + 4 : lane == 1 ? ctx->lane2 : ctx->xlane[lane - 2];   // the lane's s[4..10]
  mh::DevBuf &perm_tmp = lane == 0 ? ctx->perm_tmp : S4[7];
  void *scan_partials = lane == 0 ? ctx->scan_partials.p : lane == 1 ? ctx->scan_partials2.p : ctx->xscan[lane - 2].p;
  const int64_t n = u.n;
  const uint32_t *w_tloc = words + u.w_tloc, *w_tlen = words + u.w_tlen, *w_fo = words + u.w_fo;
  int64_t *ts = bp ? bp->ts + u.j_off : (int64_t *)S4[0].p;
  int64_t *ts_shuf = (int64_t *)S4[1].p, *te = (int64_t *)S4[2].p;
  uint32_t *sk = (uint32_t *)S4[4].p, *sv = (uint32_t *)S4[5].p;
  int32_t *nxt = (int32_t *)S4[6].p;
  const bool permute = rng_mode == MH_RNG_MITTY && n > 1 && !bp;
  uint8_t *keep = (uint8_t *)S4[3].p;
  int64_t *flag_idx = (int64_t *)ctx->s[11].p;
  int64_t *tot = (int64_t *)((char *)ctx->d_small.p + 128 + 64 * lane);
  const double log_q = std::log(1.0 - p);
  GeoFlags fl{flag_idx, d_flag, 1024};

  if (phase != 2) {
    stage_begin(ctx, "sample_geometric_scan");
    if (!exact) {
      HIPCHK(ctx, device_scan_sum<int64_t>(st, n, LoadGeo{w_tloc, p, log_q, fl}, StoreTs{ts, u.p_min + 1, u.ni},
                                           scan_partials, tot));
    } else {
      int64_t *g = (int64_t *)ctx->s[12].p;
      uint32_t nflag = 0;
      HIPCHK(ctx, hipMemsetAsync(d_flag, 0, 4, st));
      hipLaunchKernelGGL(k_geo_array, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, w_tloc, p, log_q, fl, g);
      HIPCHK(ctx, hipMemcpyAsync(&nflag, d_flag, 4, hipMemcpyDeviceToHost, st));
      SYNCCHK(ctx, hipStreamSynchronize(st));
      auto host_geo = [&](const uint32_t *ww) {   // numpy legacy_random_geometric_inversion on the host libm
        double U = (((int32_t)(ww[0] >> 5)) * 67108864.0 + ((int32_t)(ww[1] >> 6))) / 9007199254740992.0;
        return (int64_t)std::ceil(std::log1p(-U) / std::log(1.0 - p));
      };
      if (ctx->force_geo && p < 0.333333333333333333333333) {
        // MH_DEC_FORCE_GEO (tests): every draw of the unit from the host libm, so this path is pinned against the
        // oracle on whole units, not only on the rare draws the device flags
        std::vector<uint32_t> hw(2 * (size_t)n);
        std::vector<int64_t> hg((size_t)n);
        HIPCHK(ctx, hipMemcpy(hw.data(), w_tloc, 8 * (size_t)n, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < n; k++) hg[k] = host_geo(hw.data() + 2 * k);
        HIPCHK(ctx, hipMemcpy(g, hg.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
      } else {
        if (nflag > 1024) return arg_fail(ctx, MH_E_ARG, "too many near-integer geometric quotients");
        std::vector<int64_t> idx(nflag);
        if (nflag) HIPCHK(ctx, hipMemcpy(idx.data(), flag_idx, 8 * nflag, hipMemcpyDeviceToHost));
        for (int64_t k : idx) {
          uint32_t ww[2];
          HIPCHK(ctx, hipMemcpy(ww, w_tloc + 2 * k, 8, hipMemcpyDeviceToHost));
          int64_t gv = host_geo(ww);   // the reference's libm
          HIPCHK(ctx, hipMemcpy(g + k, &gv, 8, hipMemcpyHostToDevice));
        }
      }
      HIPCHK(ctx, hipMemsetAsync(d_flag, 0, 4, st));
      HIPCHK(ctx, device_scan<int64_t>(st, n, LoadArr{g}, StoreTs{ts, u.p_min + 1, u.ni}, OpSum{}, (int64_t)0,
                                       (int64_t *)scan_partials, tot));
    }
    stage_end(ctx);

    if (permute) {
      stage_begin(ctx, "sample_permutation");
      // steps sorted by (target, step): keys j, values the step index (stable LSD radix sort over the target's bits)
      unsigned end_bit = 1;
      while (end_bit < 32 && ((int64_t)1 << end_bit) < n) end_bit++;
      size_t tmp = 0;
      HIPCHK(ctx, perm_sort(nullptr, tmp, jarr, sk, sv, (size_t)n, end_bit, st));
      MH_TRY(ensure(ctx, perm_tmp, tmp + 256));
      HIPCHK(ctx, perm_sort(perm_tmp.p, tmp, jarr, sk, sv, (size_t)n, end_bit, st));
      HIPCHK(ctx, hipMemsetAsync(nxt, 0xff, 4 * (size_t)n, st));
      hipLaunchKernelGGL(k_perm_heads, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, n, (const uint32_t *)sk,
                         (const uint32_t *)sv, nxt);
      HIPCHK(ctx, hipGetLastError());
      stage_end(ctx);
    }
  }
  if (phase == 1) return MH_OK;

  const int64_t *ts_use = bp && rng_mode == MH_RNG_MITTY && n > 1 ? bp->tsh + u.j_off : ts;
  if (permute) {
    stage_begin(ctx, "sample_permutation");
    hipLaunchKernelGGL(k_perm_chase, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (int64_t)0, n,
                       (const uint32_t *)sk, (const uint32_t *)sv, (const int32_t *)nxt, (const int64_t *)ts, ts_shuf);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    ts_use = ts_shuf;
  }

  stage_begin(ctx, "sample_tlen_compact");
  hipLaunchKernelGGL(k_tlen, dim3(grid_for((n + TLEN_PER - 1) / TLEN_PER, 256, INT32_MAX)), dim3(256), 8 * n_tlen, st,
                     n, w_tlen, d_cum, n_tlen,
                     (int64_t)rlen, u.p_max, ts_use, te, keep);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, device_scan_sum<int64_t>(st, n, LoadKeep{keep},
                                       StoreCompact{keep, ts_use, te, (int64_t *)u.out->pos0.p,
                                                    (int64_t *)u.out->pos1.p, (int64_t)rlen, w_fo,
                                                    (int8_t *)u.out->fo0.p,
                                                    u.out->has_n0 ? (int32_t *)u.out->n0.p : nullptr},
                                       scan_partials, d_m));
  stage_end(ctx);
  return MH_OK;
}

}  // namespace

// A batch's sampling state between its two halves (sample_head / sample_tail): the plan, the batch buffers and the
// lanes.  The batch buffers are shared by every batch.
struct SampleState {
  std::vector<UnitPlan> plan;
  int32_t n_units = 0, rng_mode = 0, rlen = 0, n_tlen = 0, n_lanes = 1;
  bool two_lanes = false, batch = false;
  double p = 0;
  int64_t j_total = 0, nn = 0;
  uint32_t *words = nullptr, *jall = nullptr;
  double *d_cum = nullptr;
  int64_t *d_m = nullptr, *d_status = nullptr;
  uint32_t *d_flags = nullptr;
  BatchPerm bp{nullptr, nullptr};
  // the asynchronous tail (sample_units_async): per unit, its tail's end on stream2; units not yet resolved
  std::vector<hipEvent_t> ev;
  int32_t n_pending = 0;
  ~SampleState() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

// One unit's draws and its four word streams' seeds and offsets in the batch word buffer (readgenerate's
// illumina.generate_reads: int((p_max - p_min) * p * 1.2) draws; the seeds from the unit's RandomState)
static void plan_unit_words(UnitPlan &q, int64_t p_min, int64_t p_max, uint64_t seed, double p, int32_t rng_mode,
                            int64_t &words_total) {
  q.p_min = p_min;
  q.p_max = p_max;
  q.n = (int64_t)((double)(q.p_max - q.p_min) * p * 1.2);   // int((p_max - p_min) * p * 1.2)
  if (q.n < 0) q.n = 0;
  HostMT sr;
  sr.seed((uint32_t)seed);
  q.s_tloc = (uint32_t)sr.interval(0xfffffffeull);
  q.s_tlen = (uint32_t)sr.interval(0xfffffffeull);
  q.s_shuf = (uint32_t)sr.interval(0xfffffffeull);
  q.s_fo = (uint32_t)sr.interval(0xfffffffeull);
  q.n_fo_words = (q.n + 3) / 4 + 1;
  q.n_shuf_words = rng_mode == MH_RNG_MITTY ? shuffle_words_alloc(q.n) : 0;
  auto take = [&](int64_t cnt) {   // 16-byte aligned stream offsets (vector loads in the decode)
    int64_t at = words_total;
    words_total = (words_total + cnt + 4 + 3) & ~(int64_t)3;
    return at;
  };
  q.w_tloc = take(2 * q.n);
  q.w_tlen = take(2 * q.n);
  q.w_fo = take(q.n_fo_words);
  q.w_shuf = take(q.n_shuf_words);
}

// The unit's four MT19937 streams as jump-ahead segments into `words`
static void unit_seg_jobs(uint32_t *words, const UnitPlan &q, std::vector<SegJob> &jobs, int64_t &kmax) {
  const int64_t SEG_WORDS = seg_words();
  auto add_stream = [&](uint32_t *out, int64_t count, uint32_t seed) {
    for (int64_t k = 0; k * SEG_WORDS < count; k++) {
      int64_t s0 = k * SEG_WORDS;
      jobs.push_back(SegJob{out, s0, std::min(SEG_WORDS, count - s0), seed, (int32_t)k});
      kmax = std::max(kmax, k);
    }
  };
  add_stream(words + q.w_tloc, 2 * q.n, q.s_tloc);
  add_stream(words + q.w_tlen, 2 * q.n, q.s_tlen);
  add_stream(words + q.w_fo, q.n_fo_words, q.s_fo);
  add_stream(words + q.w_shuf, q.n_shuf_words, q.s_shuf);
}

// First half: plan, word streams, shuffle decode, geometric scans and — batch path — the permutation's sort and
// heads; the per-unit path runs its units whole here.
static int32_t sample_head(mh_ctx *ctx, SampleState &S, int32_t n_units, const int32_t *tpl_ids, const int64_t *p_min,
                           const int64_t *p_max, const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen,
                           int32_t n_tlen, int32_t rng_mode, const NodeIdx *nidx) {
  for (int32_t u = 0; u < n_units; u++)
    if (seeds[u] > 0xffffffffull)
      return arg_fail(ctx, MH_E_SEED, "Seed value " + std::to_string(seeds[u]) + " is out of range 0 - 4294967295");
  if (n_tlen <= 0 || n_tlen > 8192) return arg_fail(ctx, MH_E_ARG, "cum_tlen must have 1..8192 entries");
  if (rng_mode != MH_RNG_MITTY && rng_mode != MH_RNG_PHILOX) return arg_fail(ctx, MH_E_ARG, "unknown rng_mode");
  MH_TRY(tpl_resolve_all(ctx));   // the previous batch's asynchronous tail reads the batch buffers this one refills
  hipStream_t st = ctx->stream;

  // ---- plan ---------------------------------------------------------------------------------------------------
  std::vector<UnitPlan> plan(n_units);
  int64_t words_total = 0, j_total = 0, n_max = 1;
  for (int32_t u = 0; u < n_units; u++) {
    UnitPlan &q = plan[u];
    plan_unit_words(q, p_min[u], p_max[u], seeds[u], p, rng_mode, words_total);
    // (< 2^30 draws: the permutation sort's look-back counts are 30-bit; a 2x150 30x unit of 2^30 draws is a
    // 36 Gbp region)
    if (q.n > ((int64_t)1 << 30) - 8) return arg_fail(ctx, MH_E_ARG, "region too large for one work unit");
    q.j_off = j_total; j_total += q.n + 4;
    n_max = std::max(n_max, q.n);
    TplSet &ts = ctx->tsets[tpl_ids[u]];
    MH_TRY(wait_unused(ctx, ts.used, ts.used_set));   // a queued FASTQ writer may still read the old templates
    MH_TRY(ensure(ctx, ts.fo0, q.n + 16));
    MH_TRY(ensure(ctx, ts.pos0, 8 * (q.n + 16)));
    MH_TRY(ensure(ctx, ts.pos1, 8 * (q.n + 16)));
    q.ni = nidx ? nidx[u] : NodeIdx{};
    ts.n_draws = q.n;
    ts.has_n0 = q.ni.nd != nullptr;
    if (ts.has_n0) MH_TRY(ensure(ctx, ts.n0, 4 * (q.n + 16)));
    ts.valid = false;
    q.out = &ts;
  }
  const int64_t nn = n_max + 1;
  ctx->batch_left = 0;
  for (const UnitPlan &q : plan) ctx->batch_left += q.n;
  // this batch's word streams generated ahead by the prefetch thread (prefetch_words, same plan): its buffer becomes
  // the batch's (the previous batch's tails, which read the old one, were resolved above)
  PrefetchedWords &pw = ctx->pf_words;
  const bool have_words = rng_mode == MH_RNG_MITTY && pw.valid && pw.p == p && pw.seeds.size() == (size_t)n_units &&
                          std::equal(pw.seeds.begin(), pw.seeds.end(), seeds) &&
                          std::equal(pw.p_min.begin(), pw.p_min.end(), p_min) &&
                          std::equal(pw.p_max.begin(), pw.p_max.end(), p_max) && pw.words_total == words_total;
  pw.valid = false;
  if (have_words) std::swap(ctx->s[0], pw.buf);
  MH_TRY(ensure(ctx, ctx->s[0], 4 * (size_t)words_total + 64));
  MH_TRY(ensure(ctx, ctx->s[3], 4 * (size_t)j_total + 64));
  MH_TRY(ensure(ctx, ctx->s[4], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[5], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[6], 8 * nn));
  MH_TRY(ensure(ctx, ctx->s[7], nn));
  MH_TRY(ensure(ctx, ctx->s[8], 4 * (nn + 1)));
  MH_TRY(ensure(ctx, ctx->s[9], 4 * (nn + 1)));
  MH_TRY(ensure(ctx, ctx->s[10], 4 * nn));
  MH_TRY(ensure(ctx, ctx->s[11], 8 * 1024));
  // sampling lanes for the per-unit stages: two (four let more of the sampling run beside the FASTQ writers, which
  // then take longer: 3.45 against 2.73 ms per launch), at most one per unit
  int n_lanes = std::max(1, std::min(2, (int)n_units));
  const bool two_lanes = n_lanes > 1;
  // lanes 2 and 3 get their streams on first use only: the box runs with 4 hardware queues per process
  // (GPU_MAX_HW_QUEUES), and streams beyond that share queues — a sampling lane sharing the writer's queue would
  // serialize behind it
  for (int l = 2; l < n_lanes; l++)
    if (!ctx->xstream[l - 2]) {
      int lo = 0, hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
      HIPCHK(ctx, hipStreamCreateWithPriority(&ctx->xstream[l - 2], hipStreamNonBlocking, hi));
      HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_xjoin[l - 2], hipEventDisableTiming));
    }
  for (int l = 1; l < n_lanes; l++) {
    mh::DevBuf *L = l == 1 ? ctx->lane2 : ctx->xlane[l - 2];
    MH_TRY(ensure(ctx, L[0], 8 * nn));
    MH_TRY(ensure(ctx, L[1], 8 * nn));
    MH_TRY(ensure(ctx, L[2], 8 * nn));
    MH_TRY(ensure(ctx, L[3], nn));
    MH_TRY(ensure(ctx, L[4], 4 * (nn + 1)));
    MH_TRY(ensure(ctx, L[5], 4 * (nn + 1)));
    MH_TRY(ensure(ctx, L[6], 4 * nn));
    MH_TRY(ensure(ctx, l == 1 ? ctx->scan_partials2 : ctx->xscan[l - 2],
                  std::max<size_t>(16 * scan_partials_count(nn + 1) + 64, scan_lb_scratch_bytes<int64_t>(nn + 1))));
  }
  MH_TRY(ensure(ctx, ctx->s[13], 8 * (size_t)n_tlen + 64));
  MH_TRY(ensure(ctx, ctx->s[1], 64 * (size_t)n_units + 64));          // per-unit m, flags, decode status
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  MH_TRY(ensure(ctx, ctx->scan_partials, std::max<size_t>(16 * scan_partials_count(nn + 1) + 64,
                                                           scan_lb_scratch_bytes<int64_t>(nn + 1))));
  uint32_t *words = (uint32_t *)ctx->s[0].p, *jall = (uint32_t *)ctx->s[3].p;
  double *d_cum = (double *)ctx->s[13].p;
  int64_t *d_m = (int64_t *)ctx->s[1].p;                                // [n_units]
  int64_t *d_status = d_m + n_units;                                    // [n_units]
  uint32_t *d_flags = (uint32_t *)(d_status + n_units);                 // [n_units]
  HIPCHK(ctx, hipMemsetAsync(ctx->s[1].p, 0, 64 * (size_t)n_units + 64, st));
  HIPCHK(ctx, hipMemcpyAsync(d_cum, cum_tlen, 8 * n_tlen, hipMemcpyHostToDevice, st));

  stage_begin(ctx, "sample");
  // ---- word streams ------------------------------------------------------------------------------------------
  if (rng_mode == MH_RNG_MITTY) {
    std::vector<SegJob> jobs;
    std::vector<DecJob> dec;
    int64_t kmax = 0;
    const int64_t SEG_WORDS = seg_words();
    for (int32_t u = 0; u < n_units; u++) {
      UnitPlan &q = plan[u];
      if (q.n == 0) continue;
      unit_seg_jobs(words, q, jobs, kmax);
      dec.push_back(DecJob{words + q.w_shuf, q.n_shuf_words, q.n, jall + q.j_off, d_status + u});
    }
    if (!jobs.empty()) {
      MH_TRY(ensure_polys(ctx, st, kmax, SEG_WORDS));
      MH_TRY(ensure(ctx, ctx->s[2], sizeof(SegJob) * jobs.size() + sizeof(DecJob) * dec.size() + 64));
      SegJob *d_jobs = (SegJob *)ctx->s[2].p;
      DecJob *d_dec = (DecJob *)((char *)ctx->s[2].p + ((sizeof(SegJob) * jobs.size() + 15) / 16) * 16);
      HIPCHK(ctx, hipMemcpyAsync(d_jobs, jobs.data(), sizeof(SegJob) * jobs.size(), hipMemcpyHostToDevice, st));
      HIPCHK(ctx, hipMemcpyAsync(d_dec, dec.data(), sizeof(DecJob) * dec.size(), hipMemcpyHostToDevice, st));
      if (!have_words) {
        stage_begin(ctx, "sample_mt_segments");
        hipLaunchKernelGGL(k_mt_segments, dim3((unsigned)jobs.size()), dim3(256), 0, st, (const SegJob *)d_jobs,
                           (const uint32_t *)ctx->jump_polys.p);
        HIPCHK(ctx, hipGetLastError());
        stage_end(ctx);
      }
      stage_begin(ctx, "sample_shuffle_decode");
      bool done = false;
      if (!ctx->decode_sequential) MH_TRY(decode_parallel(ctx, dec, d_status, &done));
      if (!done) {   // no fixed point within the pass budget: the block-sequential decode
        hipLaunchKernelGGL(k_shuffle_decode2, dim3((unsigned)dec.size()), dim3(DC_THREADS), 0, st,
                           (const DecJob *)d_dec);
        HIPCHK(ctx, hipGetLastError());
      }
      stage_end(ctx);
      // keep the job tables alive until the kernels ran
      SYNCCHK(ctx, hipStreamSynchronize(st));
    }
  } else {
    for (int32_t u = 0; u < n_units; u++) {
      UnitPlan &q = plan[u];
      if (q.n == 0) continue;
      uint64_t key = ((uint64_t)q.s_tloc << 32) | q.s_tlen;
      hipLaunchKernelGGL(k_philox_words, dim3(grid_for((2 * q.n + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st,
                         words + q.w_tloc, 2 * q.n, key, 1u);
      hipLaunchKernelGGL(k_philox_words, dim3(grid_for((2 * q.n + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st,
                         words + q.w_tlen, 2 * q.n, key, 2u);
      hipLaunchKernelGGL(k_philox_words, dim3(grid_for((q.n_fo_words + 3) / 4, 256, INT32_MAX)), dim3(256), 0, st,
                         words + q.w_fo, q.n_fo_words, key, 3u);
      HIPCHK(ctx, hipGetLastError());
    }
  }

  // ---- per-unit parallel stages (stream-ordered, shared scratch) ------------------------------------------------
  // units alternate between the two lanes; the second lane forks after the word streams and joins before readback.
  // (They overlap the FASTQ writers queued earlier: the radix sorts and look-back scans run several times slower beside
  // a bandwidth-bound writer than alone, but waiting for the writers to drain left the writer stream idle instead —
  // the same step time, round 2.)
  if (two_lanes) {
    HIPCHK(ctx, hipEventRecord(ctx->ev_fork, st));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
    for (int l = 2; l < n_lanes; l++) HIPCHK(ctx, hipStreamWaitEvent(ctx->xstream[l - 2], ctx->ev_fork, 0));
  }
  // the batch-wide permutation (one sort per unit when the batch's draws exceed 2^30)
  const bool batch = rng_mode == MH_RNG_MITTY && j_total < ((int64_t)1 << 30) && n_units <= PK_UNITS;
  if (batch) {
    MH_TRY(ensure(ctx, ctx->pb[0], 8 * (size_t)j_total + 64));
    MH_TRY(ensure(ctx, ctx->pb[1], 8 * (size_t)j_total + 64));
    for (int b = 2; b < 6; b++) MH_TRY(ensure(ctx, ctx->pb[b], 4 * (size_t)j_total + 64));
    BatchPerm bp{(int64_t *)ctx->pb[0].p, (int64_t *)ctx->pb[1].p};
    // 1. every unit's geometric cumsum into the batch ts (lanes)
    for (int32_t u = 0, k = 0; u < n_units; u++) {
      if (plan[u].n == 0) continue;
      MH_TRY(finish_unit(ctx, plan[u], words, jall + plan[u].j_off, p, rlen, d_cum, n_tlen, rng_mode, false, d_m + u,
                         d_flags + u, k++ % n_lanes, 1, &bp));
    }
    if (two_lanes) {
      HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
      HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_join, 0));
      for (int l = 2; l < n_lanes; l++) {
        HIPCHK(ctx, hipEventRecord(ctx->ev_xjoin[l - 2], ctx->xstream[l - 2]));
        HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_xjoin[l - 2], 0));
      }
    }
    // 2. one sort of every unit's (target, step), heads, chase (main stream)
    stage_begin(ctx, "sample_permutation");
    std::vector<int64_t> uo(n_units), un(n_units);
    for (int32_t u = 0; u < n_units; u++) {
      uo[u] = plan[u].j_off;
      un[u] = plan[u].n;
    }
    int64_t *d_uo = (int64_t *)ctx->s[12].p;
    MH_TRY(ensure(ctx, ctx->s[12], 16 * (size_t)n_units + 64));
    d_uo = (int64_t *)ctx->s[12].p;
    HIPCHK(ctx, hipMemcpyAsync(d_uo, uo.data(), 8 * n_units, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_uo + n_units, un.data(), 8 * n_units, hipMemcpyHostToDevice, st));
    uint32_t *gk = (uint32_t *)ctx->pb[2].p, *sk = (uint32_t *)ctx->pb[3].p, *sv = (uint32_t *)ctx->pb[4].p;
    int32_t *nxt = (int32_t *)ctx->pb[5].p;
    hipLaunchKernelGGL(k_perm_keys, dim3(grid_for(j_total, 256, INT32_MAX)), dim3(256), 0, st, j_total,
                       (const uint32_t *)jall, (const int64_t *)d_uo, (const int64_t *)(d_uo + n_units), n_units, gk,
                       nxt);
    HIPCHK(ctx, hipGetLastError());
    unsigned end_bit = 1;
    while (end_bit < 32 && ((int64_t)1 << end_bit) < j_total) end_bit++;
    size_t tmp = 0;
    HIPCHK(ctx, perm_sort(nullptr, tmp, gk, sk, sv, (size_t)j_total, end_bit, st));
    MH_TRY(ensure(ctx, ctx->pb_tmp, tmp + 256));
    HIPCHK(ctx, perm_sort(ctx->pb_tmp.p, tmp, gk, sk, sv, (size_t)j_total, end_bit, st));
    hipLaunchKernelGGL(k_perm_heads, dim3(grid_for(j_total, 256, INT32_MAX)), dim3(256), 0, st, j_total,
                       (const uint32_t *)sk, (const uint32_t *)sv, nxt);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    S.bp = bp;
  } else {
    for (int32_t u = 0, k = 0; u < n_units; u++) {
      if (plan[u].n == 0) continue;
      MH_TRY(finish_unit(ctx, plan[u], words, jall + plan[u].j_off, p, rlen, d_cum, n_tlen, rng_mode, false, d_m + u,
                         d_flags + u, k++ % n_lanes));
    }
  }
  S.plan = std::move(plan);
  S.n_units = n_units;
  S.rng_mode = rng_mode;
  S.rlen = rlen;
  S.n_tlen = n_tlen;
  S.n_lanes = n_lanes;
  S.two_lanes = two_lanes;
  S.batch = batch;
  S.p = p;
  S.j_total = j_total;
  S.nn = nn;
  S.words = words;
  S.jall = jall;
  S.d_cum = d_cum;
  S.d_m = d_m;
  S.d_status = d_status;
  S.d_flags = d_flags;
  return MH_OK;
}

// Second half: the batch path's chase and per-unit template lengths, compaction and file order; the lanes joined,
// the counts read back, the rare exact fix-ups, the template sets marked valid.
static int32_t sample_tail(mh_ctx *ctx, SampleState &S, int64_t *out_n) {
  hipStream_t st = ctx->stream;
  std::vector<UnitPlan> &plan = S.plan;
  const int32_t n_units = S.n_units, rng_mode = S.rng_mode, rlen = S.rlen, n_tlen = S.n_tlen, n_lanes = S.n_lanes;
  const bool two_lanes = S.two_lanes;
  const double p = S.p;
  const int64_t j_total = S.j_total, nn = S.nn;
  uint32_t *words = S.words, *jall = S.jall;
  double *d_cum = S.d_cum;
  int64_t *d_m = S.d_m, *d_status = S.d_status;
  uint32_t *d_flags = S.d_flags;
  if (S.batch) {
    const BatchPerm &bp = S.bp;
    const uint32_t *sk = (const uint32_t *)ctx->pb[3].p, *sv = (const uint32_t *)ctx->pb[4].p;
    const int32_t *nxt = (const int32_t *)ctx->pb[5].p;
    stage_begin(ctx, "sample_permutation");
    hipLaunchKernelGGL(k_perm_chase, dim3(grid_for(j_total, 256, INT32_MAX)), dim3(256), 0, st, (int64_t)0, j_total,
                       sk, sv, nxt, (const int64_t *)bp.ts, bp.tsh);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    // 3. every unit's template lengths, compaction and file order (lanes)
    if (two_lanes) {
      HIPCHK(ctx, hipEventRecord(ctx->ev_fork, st));
      HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
      for (int l = 2; l < n_lanes; l++) HIPCHK(ctx, hipStreamWaitEvent(ctx->xstream[l - 2], ctx->ev_fork, 0));
    }
    for (int32_t u = 0, k = 0; u < n_units; u++) {
      if (plan[u].n == 0) continue;
      MH_TRY(finish_unit(ctx, plan[u], words, jall + plan[u].j_off, p, rlen, d_cum, n_tlen, rng_mode, false, d_m + u,
                         d_flags + u, k++ % n_lanes, 2, &bp));
    }
  }
  if (two_lanes) {
    HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
    HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_join, 0));
    for (int l = 2; l < n_lanes; l++) {
      HIPCHK(ctx, hipEventRecord(ctx->ev_xjoin[l - 2], ctx->xstream[l - 2]));
      HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_xjoin[l - 2], 0));
    }
  }
  std::vector<int64_t> hm(n_units), hstat(n_units);
  std::vector<uint32_t> hflag(n_units);
  // d_m, d_status, d_flags are consecutive in s[1] (20 bytes per unit): one readback into pinned memory
  int64_t *hs = pinned_small(ctx);
  const size_t rb_bytes = 20 * (size_t)n_units;
  if (hs && rb_bytes <= 3072) {
    HIPCHK(ctx, hipMemcpyAsync(hs + 64, d_m, rb_bytes, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    std::memcpy(hm.data(), hs + 64, 8 * n_units);
    std::memcpy(hstat.data(), hs + 64 + n_units, 8 * n_units);
    std::memcpy(hflag.data(), hs + 64 + 2 * n_units, 4 * n_units);
  } else {
    HIPCHK(ctx, hipMemcpyAsync(hm.data(), d_m, 8 * n_units, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(hstat.data(), d_status, 8 * n_units, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(hflag.data(), d_flags, 4 * n_units, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
  }

  // ---- rare exact fix-ups: decode out of words (sequential stream), near-integer geometric quotients ------------
  for (int32_t u = 0; u < n_units; u++) {
    UnitPlan &q = plan[u];
    if (q.n == 0) continue;
    // MH_DEC_FORCE_FIXUP / _GEO (tests): take the fallback for every unit
    if (ctx->force_fixup) hstat[u] = 1;
    if (ctx->force_geo) hflag[u] = 1;
    if (hstat[u] == 0 && hflag[u] == 0) continue;
    if (rng_mode == MH_RNG_MITTY && hstat[u] != 0) {
      hipLaunchKernelGGL(k_shuffle_decode, dim3(1), dim3(SD_THREADS), 0, st, q.s_shuf, q.n, jall + q.j_off);
      HIPCHK(ctx, hipGetLastError());
    }
    MH_TRY(ensure(ctx, ctx->s[12], 8 * (size_t)nn));
    HIPCHK(ctx, hipMemsetAsync(d_flags + u, 0, 4, st));
    MH_TRY(finish_unit(ctx, q, words, jall + q.j_off, p, rlen, d_cum, n_tlen, rng_mode, hflag[u] != 0, d_m + u,
                       d_flags + u));
    HIPCHK(ctx, hipMemcpyAsync(&hm[u], d_m + u, 8, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    ctx->fixups++;
  }
  stage_end(ctx);
  for (int32_t u = 0; u < n_units; u++) {
    TplSet &ts = *plan[u].out;
    ts.n = plan[u].n == 0 ? 0 : hm[u];
    ts.rlen = rlen;
    ts.valid = true;
    if (out_n) out_n[u] = ts.n;
  }
  return MH_OK;
}

// One unit's tail results into mapped host memory (plain vector stores; the host reads them after the unit's event).
__global__ void k_unit_result(const int64_t *m, const int64_t *status, const uint32_t *flag, int64_t *out) {
  if (threadIdx.x == 0) {
    out[0] = *m;
    out[1] = *status;
    out[2] = (int64_t)*flag;
  }
}

// The batch tail without a host wait: per unit, in unit order on stream2, its range of the batch chase
// ([j_off, j_off + n + 4) of the sorted entries: a unit's keys are its own), its template lengths and compaction, its
// results into mapped host memory and an event.  The writer of unit 0 then waits for unit 0's tail only, not for the
// whole batch's chase and compactions (the writer stream's idle gap at batch boundaries).  Template sets
// stay pending (TplSet.pend) until tpl_resolve.
static int32_t sample_tail_async(mh_ctx *ctx, const std::shared_ptr<SampleState> &Sp) {
  SampleState &S = *Sp;
  std::vector<UnitPlan> &plan = S.plan;
  const int32_t n_units = S.n_units;
  hipStream_t st = ctx->stream, l1 = ctx->stream2;
  const BatchPerm &bp = S.bp;
  const uint32_t *sk = (const uint32_t *)ctx->pb[3].p, *sv = (const uint32_t *)ctx->pb[4].p;
  const int32_t *nxt = (const int32_t *)ctx->pb[5].p;
  HIPCHK(ctx, hipEventRecord(ctx->ev_fork, st));
  HIPCHK(ctx, hipStreamWaitEvent(l1, ctx->ev_fork, 0));
  S.ev.assign(n_units, nullptr);
  for (int32_t u = 0; u < n_units; u++) {
    UnitPlan &q = plan[u];
    TplSet &ts = *q.out;
    if (q.n == 0) {
      ts.n = 0;
      ts.rlen = S.rlen;
      ts.valid = true;
      continue;
    }
    // (the whole batch's chase on the main stream before the fork instead: the same step time, round 4's A/B)
    ctx->stage_stream = l1;
    stage_begin(ctx, "sample_permutation");
    const int64_t k0 = q.j_off, k1 = q.j_off + q.n + 4;
    hipLaunchKernelGGL(k_perm_chase, dim3(grid_for(k1 - k0, 256, INT32_MAX)), dim3(256), 0, l1, k0, k1, sk, sv, nxt,
                       (const int64_t *)bp.ts, bp.tsh);
    stage_end(ctx);
    ctx->stage_stream = nullptr;
    HIPCHK(ctx, hipGetLastError());
    MH_TRY(finish_unit(ctx, q, S.words, S.jall + q.j_off, S.p, S.rlen, S.d_cum, S.n_tlen, S.rng_mode, false,
                       S.d_m + u, S.d_flags + u, 1, 2, &bp));
    hipLaunchKernelGGL(k_unit_result, dim3(1), dim3(64), 0, l1, (const int64_t *)(S.d_m + u),
                       (const int64_t *)(S.d_status + u), (const uint32_t *)(S.d_flags + u), ctx->d_units + 4 * u);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventCreateWithFlags(&S.ev[u], hipEventDisableTiming));
    HIPCHK(ctx, hipEventRecord(S.ev[u], l1));
    ts.pend = u;
    S.n_pending++;
  }
  stage_end(ctx);
  if (S.n_pending) ctx->tail_state = Sp;
  return MH_OK;
}

int32_t tpl_resolve(mh_ctx *ctx, TplSet &ts) {
  if (ts.pend < 0) return MH_OK;
  const int32_t u = ts.pend;
  ts.pend = -1;
  auto Sp = std::static_pointer_cast<SampleState>(ctx->tail_state);
  if (!Sp || u >= Sp->n_units || Sp->plan[u].out != &ts)
    return arg_fail(ctx, MH_E_STATE, "template set of a lost sampling batch");
  SampleState &S = *Sp;
  UnitPlan &q = S.plan[u];
  hipStream_t st = ctx->stream;
  SYNCCHK(ctx, hipEventSynchronize(S.ev[u]));
  const volatile int64_t *r = ctx->h_units + 4 * u;
  int64_t m = r[0];
  const int64_t status = ctx->force_fixup ? 1 : r[1];                // MH_DEC_FORCE_FIXUP (tests)
  const uint32_t flag = ctx->force_geo ? 1u : (uint32_t)r[2];         // MH_DEC_FORCE_GEO (tests)
  HIPCHK(ctx, hipStreamWaitEvent(st, S.ev[u], 0));   // (the main stream's work on this set comes after its tail)
  if (status != 0 || flag != 0) {   // rare exact fix-up, as in sample_tail
    if (S.rng_mode == MH_RNG_MITTY && status != 0) {
      hipLaunchKernelGGL(k_shuffle_decode, dim3(1), dim3(SD_THREADS), 0, st, q.s_shuf, q.n, S.jall + q.j_off);
      HIPCHK(ctx, hipGetLastError());
    }
    MH_TRY(ensure(ctx, ctx->s[12], 8 * (size_t)S.nn));
    HIPCHK(ctx, hipMemsetAsync(S.d_flags + u, 0, 4, st));
    MH_TRY(finish_unit(ctx, q, S.words, S.jall + q.j_off, S.p, S.rlen, S.d_cum, S.n_tlen, S.rng_mode, flag != 0,
                       S.d_m + u, S.d_flags + u));
    HIPCHK(ctx, hipMemcpyAsync(&m, S.d_m + u, 8, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    ctx->fixups++;
  }
  ts.n = m;
  ts.rlen = S.rlen;
  ts.valid = true;
  if (--S.n_pending == 0) ctx->tail_state.reset();
  return MH_OK;
}

int32_t tpl_resolve_all(mh_ctx *ctx) {
  auto Sp = std::static_pointer_cast<SampleState>(ctx->tail_state);
  if (!Sp) return MH_OK;
  for (UnitPlan &q : Sp->plan)
    if (q.out && q.out->pend >= 0) MH_TRY(tpl_resolve(ctx, *q.out));
  return MH_OK;
}

int32_t prefetch_words(mh_ctx *ctx, hipStream_t st, int32_t n_units, const int64_t *p_min, const int64_t *p_max,
                       const uint64_t *seeds, double p) {
  PrefetchedWords &pw = ctx->pf_words;
  pw.valid = false;
  std::vector<UnitPlan> plan(n_units);
  int64_t words_total = 0;
  for (int32_t u = 0; u < n_units; u++) {
    plan_unit_words(plan[u], p_min[u], p_max[u], seeds[u], p, MH_RNG_MITTY, words_total);
    if (plan[u].n > ((int64_t)1 << 30) - 8) return MH_OK;   // (sample_head reports it)
  }
  MH_TRY(ensure(ctx, pw.buf, 4 * (size_t)words_total + 64));
  std::vector<SegJob> jobs;
  int64_t kmax = 0;
  for (const UnitPlan &q : plan)
    if (q.n > 0) unit_seg_jobs((uint32_t *)pw.buf.p, q, jobs, kmax);
  // the jump polynomials are the main thread's (ensure_polys): without them resident the batch is not prefetched
  if (jobs.empty() || ctx->jump_k < kmax + 1 || ctx->jump_seg != seg_words()) return MH_OK;
  MH_TRY(ensure(ctx, pw.jobs, sizeof(SegJob) * jobs.size() + 64));
  HIPCHK(ctx, hipMemcpyAsync(pw.jobs.p, jobs.data(), sizeof(SegJob) * jobs.size(), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_mt_segments, dim3((unsigned)jobs.size()), dim3(256), 0, st, (const SegJob *)pw.jobs.p,
                     (const uint32_t *)ctx->jump_polys.p);
  HIPCHK(ctx, hipGetLastError());
  SYNCCHK(ctx, hipStreamSynchronize(st));   // (the job table's host copy lives until here)
  pw.p = p;
  pw.seeds.assign(seeds, seeds + n_units);
  pw.p_min.assign(p_min, p_min + n_units);
  pw.p_max.assign(p_max, p_max + n_units);
  pw.words_total = words_total;
  pw.valid = true;
  return MH_OK;
}

int32_t sample_units_async(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int64_t *p_min,
                           const int64_t *p_max, const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen,
                           int32_t n_tlen, int32_t rng_mode, const NodeIdx *nidx) {
  if (!ctx->h_units) {
    if (hipHostMalloc((void **)&ctx->h_units, 32 * (size_t)PK_UNITS, hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess) {
      ctx->h_units = nullptr;
      return arg_fail(ctx, MH_E_OOM, "pinned host memory");
    }
    void *d = nullptr;
    HIPCHK(ctx, hipHostGetDevicePointer(&d, ctx->h_units, 0));
    ctx->d_units = (int64_t *)d;
  }
  auto S = std::make_shared<SampleState>();
  MH_TRY(sample_head(ctx, *S, n_units, tpl_ids, p_min, p_max, seeds, p, rlen, cum_tlen, n_tlen, rng_mode, nidx));
  // the per-unit path (Philox, oversized batches) and a one-unit batch (no second lane) end as sample_units does
  if (!S->batch || !S->two_lanes) return sample_tail(ctx, *S, nullptr);
  return sample_tail_async(ctx, S);
}

int32_t sample_units(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int64_t *p_min, const int64_t *p_max,
                     const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                     int32_t rng_mode, int64_t *out_n, const NodeIdx *nidx) {
  SampleState S;
  MH_TRY(sample_head(ctx, S, n_units, tpl_ids, p_min, p_max, seeds, p, rlen, cum_tlen, n_tlen, rng_mode, nidx));
  return sample_tail(ctx, S, out_n);
}

}  // namespace mh
