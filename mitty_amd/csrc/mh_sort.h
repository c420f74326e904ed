// mh_sort.h — the permutation's stable (target, step) sort on gfx950: an LSD radix sort of u32 keys whose values are
// the element indices (the Fisher-Yates steps, illumina.py:70 `shuffle_rng.shuffle(ts)`; DESIGN.md "Kernels").
//
// 9-bit digits, ceil(end_bit / 9) passes (a 64 M-draw batch's 26-27-bit keys: 3), with the tile counts folded into
// the scatter (decoupled look-back per digit), so a pass reads and writes every key and value once:
//   k_rs_hist     every pass's digit histogram in one read of the input keys (LDS per workgroup, then one global
//                 atomic per digit and workgroup); k_rs_starts turns each pass's histogram into digit starts;
//   k_rs_onesweep one 512-thread workgroup per 8192-key tile, tiles taken in launch order from a ticket: each wave
//                 ranks its 16 x 64 keys stably (per item row a match over the digit's 9 bits by ballots, a running
//                 per-wave digit count in LDS); the tile publishes its per-digit counts, looks back over its
//                 predecessors' (thread = digit) until an inclusive prefix, publishes its own; the keys, then the
//                 values, are laid out in LDS in digit order and written out in that order (runs of one digit land
//                 on consecutive addresses: 16 keys per digit and tile on average).
// Round 5 measured the 2048-key tile at ~1 ms per pass of 67 M keys in isolation (~1 TB/s): per key, a quarter of a
// status word to clear, publish and look back over, and 16-byte runs per digit.  The 8192-key tile quarters both.
// 512 threads and ~50 KB of LDS (keys and values staged in turn through one buffer): small enough to take the CU
// slots a retiring FASTQ writer frees (the library sort's 1024-thread workgroups waited for whole CUs).  Stable:
// equal keys keep their input order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mh_device.h"
#include "mh_scan.h"

namespace mh {

constexpr int RS_THREADS = 512;   // (256-thread workgroups / 4096-key tiles: writers 7 % slower beside them, round 5)
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;   // 8192 keys
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_BITS = 9;
constexpr uint32_t RS_BINS = 1u << RS_BITS, RS_MASK = RS_BINS - 1u;
constexpr int RS_DPT = (int)RS_BINS / RS_THREADS;   // digits per thread (1)
static_assert(RS_DPT >= 1 && RS_DPT * RS_THREADS == (int)RS_BINS, "every thread owns whole digits");
constexpr int RS_MAXP = 4;                          // passes (u32 keys: at most 4 x 9 bits)
// look-back status word per (tile, digit): flag in the top two bits, the count (< 2^30) below
constexpr uint32_t RS_AGG = 0x40000000u, RS_INC = 0x80000000u, RS_VAL = 0x3fffffffu;

static __global__ void __launch_bounds__(RS_THREADS) k_rs_hist(const uint32_t *keys, int64_t n, int passes,
                                                              uint32_t *ghist) {
  __shared__ uint32_t h[RS_MAXP * RS_BINS];
  for (int i = threadIdx.x; i < RS_MAXP * (int)RS_BINS; i += RS_THREADS) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * RS_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * RS_THREADS) {
    const uint32_t k = keys[i];
    for (int p = 0; p < passes; p++) atomicAdd(&h[p * RS_BINS + ((k >> (RS_BITS * p)) & RS_MASK)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * (int)RS_BINS; i += RS_THREADS)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// one workgroup per pass: its histogram -> exclusive digit starts, in place
static __global__ void __launch_bounds__(RS_THREADS) k_rs_starts(uint32_t *ghist) {
  __shared__ int32_t wsum[RS_WAVES];
  uint32_t *h = ghist + (size_t)blockIdx.x * RS_BINS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // thread t owns digits RS_DPT t .. RS_DPT t + RS_DPT - 1 (consecutive: the scan runs over the threads)
  uint32_t v[RS_DPT], s = 0;
#pragma unroll
  for (int q = 0; q < RS_DPT; q++) {
    v[q] = h[RS_DPT * tid + q];
    s += v[q];
  }
  int total;
  const int32_t incl = wave_sum_incl((int32_t)s, total);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int32_t pre = 0;
#pragma unroll
  for (int q = 0; q < RS_WAVES; q++) pre += q < w ? wsum[q] : 0;
  uint32_t x = (uint32_t)(pre + incl) - s;
#pragma unroll
  for (int q = 0; q < RS_DPT; q++) {
    h[RS_DPT * tid + q] = x;
    x += v[q];
  }
}

// keys_in / vals_in (null: the element index) -> keys_out / vals_out, stable by digit (key >> shift) & RS_MASK.
// gstart: the pass's digit starts; status: [ticket (64 B)] [tiles x RS_BINS words], zeroed before the launch; fault:
// the look-back scans' host-mapped fault word (a wait that never ends is reported, mh_scan.h).
static __global__ void __launch_bounds__(RS_THREADS) k_rs_onesweep(const uint32_t *keys_in, const uint32_t *vals_in,
                                                                  int64_t n, int shift, const uint32_t *gstart,
                                                                  uint32_t *status, uint32_t *keys_out, uint32_t *vals_out,
                                                                  uint32_t *fault) {
  __shared__ uint32_t wc[RS_WAVES][RS_BINS];   // per wave: running digit counts, then the wave's exclusive prefix
  __shared__ uint32_t ds[RS_BINS];             // the tile's digit starts (exclusive scan over digits)
  __shared__ uint32_t go[RS_BINS];             // the tile's global output offset per digit
  __shared__ uint32_t sb[RS_TILE];             // keys, then values, in digit order
  __shared__ int32_t wsum[RS_WAVES];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t *ticket = status;
  uint32_t *st = status + 16;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  for (int i = tid; i < RS_WAVES * (int)RS_BINS; i += RS_THREADS) (&wc[0][0])[i] = 0;
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t t0 = tile * RS_TILE;
  const int nt = (int)(n - t0 < RS_TILE ? n - t0 : RS_TILE);   // keys in this tile
  const int wb = w * (64 * RS_ITEMS) + lane;                      // item k of this lane: tile key wb + 64 k
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t key[RS_ITEMS], rk[RS_ITEMS];   // (the values are loaded when they are laid out: fewer registers)
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++)   // element order in the wave: item row k, then lane
    key[k] = wb + 64 * k < nt ? keys_in[t0 + wb + 64 * k] : 0xffffffffu;
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const bool ok = wb + 64 * k < nt;
    const uint32_t d = (key[k] >> shift) & RS_MASK;
    uint64_t m = __ballot(ok);   // lanes holding the same digit (invalid lanes match nobody)
#pragma unroll
    for (int b = 0; b < RS_BITS; b++) {
      const uint64_t bal = __ballot(ok && ((d >> b) & 1u));
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const int leader = m ? __builtin_ctzll(m) : lane;
    uint32_t c0 = 0;
    if (ok && lane == leader) c0 = wc[w][d];
    c0 = __shfl(c0, leader, 64);
    rk[k] = c0 + (uint32_t)__popcll(m & below);
    if (ok && lane == leader) wc[w][d] = c0 + (uint32_t)__popcll(m);
  }
  __syncthreads();
  // per digit (thread t: digits RS_DPT t + q): the waves' exclusive prefixes and the tile's count; the count published
  uint32_t t[RS_DPT], s = 0;
#pragma unroll
  for (int q = 0; q < RS_DPT; q++) {
    const int d = RS_DPT * tid + q;
    uint32_t c = 0;
#pragma unroll
    for (int x = 0; x < RS_WAVES; x++) {
      const uint32_t y = wc[x][d];
      wc[x][d] = c;
      c += y;
    }
    t[q] = c;
    s += c;
    __hip_atomic_store(&st[tile * RS_BINS + d], (tile == 0 ? RS_INC : RS_AGG) | c, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  {   // the tile's digit starts: an exclusive scan of the counts over the digits
    int total;
    const int32_t incl = wave_sum_incl((int32_t)s, total);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int32_t pre = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) pre += q < w ? wsum[q] : 0;
    uint32_t x = (uint32_t)(pre + incl) - s;
#pragma unroll
    for (int q = 0; q < RS_DPT; q++) {
      ds[RS_DPT * tid + q] = x;
      x += t[q];
    }
  }
  // look-back per digit: the predecessors' counts until an inclusive prefix
#pragma unroll
  for (int q = 0; q < RS_DPT; q++) {
    const int d = RS_DPT * tid + q;
    uint32_t pre = 0;
    if (tile > 0) {
      int64_t j = tile - 1;
      uint32_t spins = 0;
      for (;;) {
        const uint32_t v = __hip_atomic_load(&st[j * RS_BINS + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v & (RS_INC | RS_AGG)) {
          pre += v & RS_VAL;
          if (v & RS_INC) break;
          j--;
          continue;
        }
        if (++spins > (1u << 24)) {   // never published (a broken ticket or status area): report, do not hang
          if (fault) __hip_atomic_store(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(&st[tile * RS_BINS + d], RS_INC | (pre + t[q]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    go[d] = gstart[d] + pre;
  }
  __syncthreads();
  // each item's place in the tile's digit order (rk becomes it), then the keys through LDS: thread t writes places
  // t, t + RS_THREADS, ... and keeps each one's output index for the values
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    if (wb + 64 * k < nt) {
      const uint32_t d = (key[k] >> shift) & RS_MASK;
      rk[k] = ds[d] + wc[w][d] + rk[k];
      sb[rk[k]] = key[k];
    }
  }
  __syncthreads();
  uint32_t oi[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int p = k * RS_THREADS + tid;
    oi[k] = 0xffffffffu;
    if (p < nt) {
      const uint32_t kk = sb[p], d = (kk >> shift) & RS_MASK;
      const uint32_t o = go[d] + (uint32_t)p - ds[d];
      if ((int64_t)o < n) {   // (always: a guard against a broken offset table, never a stray write)
        keys_out[o] = kk;
        oi[k] = o;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int li = wb + 64 * k;
    if (li < nt) sb[rk[k]] = vals_in ? vals_in[t0 + li] : (uint32_t)(t0 + li);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++)
    if (oi[k] != 0xffffffffu) vals_out[oi[k]] = sb[k * RS_THREADS + tid];
}

// Scratch for lsd_sort_pairs_iota: two key and value buffers, the look-back status words, the histograms.
inline size_t lsd_sort_tmp_bytes(int64_t n) {
  const int64_t tiles = (n + RS_TILE - 1) / RS_TILE;
  return 2 * 4 * (size_t)n + 4 * (size_t)(tiles < 1 ? 1 : tiles) * RS_BINS + 64 + 4 * RS_MAXP * RS_BINS + 2048;
}

// Stable sort of keys_in[0, n) over bits [0, end_bit), values = the element indices: keys_out / vals_out.  tmp null:
// tmp_bytes gets the scratch size (rocprim's two-call convention).
inline hipError_t lsd_sort_pairs_iota(void *tmp, size_t &tmp_bytes, const uint32_t *keys_in, uint32_t *keys_out,
                                      uint32_t *vals_out, int64_t n, unsigned end_bit, hipStream_t st) {
  if (!tmp) {
    tmp_bytes = lsd_sort_tmp_bytes(n);
    return hipSuccess;
  }
  if (tmp_bytes < lsd_sort_tmp_bytes(n) || n < 0 || n >= ((int64_t)1 << 30)) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const int64_t tiles = (n + RS_TILE - 1) / RS_TILE;
  char *p = (char *)tmp;
  auto take = [&](size_t b) {
    char *q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  uint32_t *k2 = (uint32_t *)take(4 * (size_t)n), *v2 = (uint32_t *)take(4 * (size_t)n);
  const size_t st_bytes = 64 + 4 * (size_t)tiles * RS_BINS;
  uint32_t *status = (uint32_t *)take(st_bytes);
  uint32_t *ghist = (uint32_t *)take(4 * RS_MAXP * RS_BINS);
  const int passes = end_bit == 0 ? 1 : (int)((end_bit + RS_BITS - 1) / RS_BITS);
  hipError_t e = hipMemsetAsync(ghist, 0, 4 * (size_t)passes * RS_BINS, st);
  if (e != hipSuccess) return e;
  const int64_t hg = tiles < 2048 ? tiles : 2048;
  hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)hg), dim3(RS_THREADS), 0, st, keys_in, n, passes, ghist);
  hipLaunchKernelGGL(k_rs_starts, dim3((unsigned)passes), dim3(RS_THREADS), 0, st, ghist);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint32_t *ksrc = keys_in, *vsrc = nullptr;
  for (int ps = 0; ps < passes; ps++) {
    // the last pass writes the outputs; the ones before alternate so that it reads the other buffer
    const bool to_out = ((passes - 1 - ps) & 1) == 0;
    uint32_t *kd = to_out ? keys_out : k2, *vd = to_out ? vals_out : v2;
    if ((e = hipMemsetAsync(status, 0, st_bytes, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_rs_onesweep, dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, ksrc, vsrc, n, RS_BITS * ps,
                       (const uint32_t *)(ghist + (size_t)ps * RS_BINS), status, kd, vd, scan_fault_device());
    if ((e = hipGetLastError()) != hipSuccess) return e;
    ksrc = kd;
    vsrc = vd;
  }
  return hipSuccess;
}

}  // namespace mh
