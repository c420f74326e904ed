// mh_sort.h — the permutation's stable (target, step) sort on gfx950: an LSD radix sort of u32 keys whose values are
// the element indices (the Fisher-Yates steps, illumina.py:70 `shuffle_rng.shuffle(ts)`; DESIGN.md "Kernels").
//
// 7-bit digits, ceil(end_bit / 7) passes, each three steps:
//   k_rs_count    one 256-thread workgroup per 2048-key tile: the tile's digit histogram (LDS atomics), written
//                 digit-major (count[d * tiles + tile]), so one exclusive scan of the counts gives every
//                 (digit, tile) its global output offset;
//   scan          device_scan_sum (mh_scan.h's look-back scan) over the 128 x tiles counts;
//   k_rs_scatter  the tile again: each wave ranks its 8 x 64 keys stably (per item row a match over the digit's 7
//                 bits by ballots, a running per-wave digit count in LDS), waves combined per digit, the keys and
//                 values laid out in LDS in digit order, then written out in that order (runs of one digit — 16 keys
//                 on average, 64 bytes — land on consecutive addresses).
// Sized to fit where a FASTQ writer workgroup retires: 256 threads and under 20 KB of LDS (the writer's is ~22 KB), so
// the sort's workgroups take the CU slots the writers free (the library sort's 1024-thread workgroups waited for whole
// CUs, round 3).  Stable: equal keys keep their input order, as rocprim's sort does.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mh_device.h"
#include "mh_scan.h"

namespace mh {

constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;   // 2048 keys
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_BITS = 7;
constexpr uint32_t RS_BINS = 1u << RS_BITS, RS_MASK = RS_BINS - 1u;

__global__ void __launch_bounds__(RS_THREADS) k_rs_count(const uint32_t *keys, int64_t n, int shift,
                                                        uint32_t *count, int64_t tiles) {
  __shared__ uint32_t h[RS_BINS];
  const int tid = threadIdx.x;
  if (tid < (int)RS_BINS) h[tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int64_t i = base + k * RS_THREADS + tid;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & RS_MASK], 1u);
  }
  __syncthreads();
  if (tid < (int)RS_BINS) count[(int64_t)tid * tiles + blockIdx.x] = h[tid];
}

struct RsLoad {
  const uint32_t *c;
  int64_t n;
  __device__ int64_t operator()(int64_t i) const { return i < n ? (int64_t)c[i] : 0; }
};
struct RsStore {
  uint32_t *o;
  __device__ void operator()(int64_t i, int64_t, int64_t ex) const { o[i] = (uint32_t)ex; }
};

// keys_in / vals_in (null: the element index) -> keys_out / vals_out, stable by digit (key >> shift) & RS_MASK
__global__ void __launch_bounds__(RS_THREADS) k_rs_scatter(const uint32_t *keys_in, const uint32_t *vals_in, int64_t n,
                                                          int shift, const uint32_t *offs, int64_t tiles,
                                                          uint32_t *keys_out, uint32_t *vals_out) {
  __shared__ uint32_t wc[RS_WAVES][RS_BINS];   // per wave: running digit counts, then the wave's exclusive prefix
  __shared__ uint32_t ds[RS_BINS];             // the tile's digit starts (exclusive scan over digits)
  __shared__ uint32_t go[RS_BINS];             // the tile's global output offset per digit
  __shared__ uint32_t sk[RS_TILE], sv[RS_TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < (int)RS_BINS) {
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) wc[q][tid] = 0;
    go[tid] = offs[(int64_t)tid * tiles + blockIdx.x];
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE + (int64_t)w * (64 * RS_ITEMS);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t key[RS_ITEMS], val[RS_ITEMS], rk[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {   // element order in the wave: item row k, then lane
    const int64_t i = base + 64 * k + lane;
    const bool ok = i < n;
    key[k] = ok ? keys_in[i] : 0xffffffffu;
    val[k] = ok ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
  }
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int64_t i = base + 64 * k + lane;
    const bool ok = i < n;
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
  // per digit (thread = digit; threads past the bins count 0): the waves' exclusive prefixes and the tile's count,
  // then the digit starts
  uint32_t t = 0;
  if (tid < (int)RS_BINS) {
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) {
      const uint32_t c = wc[q][tid];
      wc[q][tid] = t;
      t += c;
    }
  }
  {
    int total;
    const int32_t incl = wave_sum_incl((int32_t)t, total);   // (within the wave)
    __shared__ int32_t wsum[RS_WAVES];
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int32_t pre = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) pre += q < w ? wsum[q] : 0;
    if (tid < (int)RS_BINS) ds[tid] = (uint32_t)(pre + incl) - t;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int64_t i = base + 64 * k + lane;
    if (i < n) {
      const uint32_t d = (key[k] >> shift) & RS_MASK;
      const uint32_t pos = ds[d] + wc[w][d] + rk[k];
      sk[pos] = key[k];
      sv[pos] = val[k];
    }
  }
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * RS_TILE;
  const int nt = (int)(n - t0 < RS_TILE ? n - t0 : RS_TILE);
#pragma unroll
  for (int k = 0; k < RS_ITEMS; k++) {
    const int p = k * RS_THREADS + tid;
    if (p < nt) {
      const uint32_t kk = sk[p], d = (kk >> shift) & RS_MASK;
      const uint32_t o = go[d] + (uint32_t)p - ds[d];
      if ((int64_t)o < n) {   // (always: a guard against a broken offset table, never a stray write)
        keys_out[o] = kk;
        vals_out[o] = sv[p];
      }
    }
  }
}

// Scratch for lsd_sort_pairs_iota: two key and value buffers, the counts, their offsets, the scan's scratch.
inline size_t lsd_sort_tmp_bytes(int64_t n) {
  const int64_t tiles = (n + RS_TILE - 1) / RS_TILE, nc = RS_BINS * (tiles < 1 ? 1 : tiles);
  return 2 * 4 * (size_t)n + 2 * 4 * (size_t)nc + scan_lb_scratch_bytes<int64_t>(nc) + 2048;
}

// Stable sort of keys_in[0, n) over bits [0, end_bit), values = the element indices: keys_out / vals_out.  tmp null:
// tmp_bytes gets the scratch size (rocprim's two-call convention).
inline hipError_t lsd_sort_pairs_iota(void *tmp, size_t &tmp_bytes, const uint32_t *keys_in, uint32_t *keys_out,
                                      uint32_t *vals_out, int64_t n, unsigned end_bit, hipStream_t st) {
  if (!tmp) {
    tmp_bytes = lsd_sort_tmp_bytes(n);
    return hipSuccess;
  }
  if (tmp_bytes < lsd_sort_tmp_bytes(n) || n < 0 || n >= ((int64_t)1 << 32) - 1) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const int64_t tiles = (n + RS_TILE - 1) / RS_TILE, nc = RS_BINS * tiles;
  char *p = (char *)tmp;
  auto take = [&](size_t b) {
    char *q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  uint32_t *k2 = (uint32_t *)take(4 * (size_t)n), *v2 = (uint32_t *)take(4 * (size_t)n);
  uint32_t *cnt = (uint32_t *)take(4 * (size_t)nc), *off = (uint32_t *)take(4 * (size_t)nc);
  void *scr = take(scan_lb_scratch_bytes<int64_t>(nc));
  int64_t *total = (int64_t *)take(64);
  const int passes = end_bit == 0 ? 1 : (int)((end_bit + RS_BITS - 1) / RS_BITS);
  // the scan scratch sits inside tmp at an offset that moves with n, so the memory under it holds other sorts' keys:
  // its look-back state starts fresh here (zeroed by the first pass's scan) and is dropped after the last pass, so
  // no later scan takes this interior address for zeroed scratch with a running ticket
  lb_forget(scr);
  struct Forget {
    const void *p;
    ~Forget() { lb_forget(p); }
  } forget{scr};
  const uint32_t *ksrc = keys_in, *vsrc = nullptr;
  for (int ps = 0; ps < passes; ps++) {
    // the last pass writes the outputs; the ones before alternate so that it reads the other buffer
    const bool to_out = ((passes - 1 - ps) & 1) == 0;
    uint32_t *kd = to_out ? keys_out : k2, *vd = to_out ? vals_out : v2;
    hipLaunchKernelGGL(k_rs_count, dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, ksrc, n, RS_BITS * ps, cnt, tiles);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = device_scan_sum<int64_t>(st, nc, RsLoad{cnt, nc}, RsStore{off}, scr, total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, ksrc, vsrc, n, RS_BITS * ps,
                       (const uint32_t *)off, tiles, kd, vd);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    ksrc = kd;
    vsrc = vd;
  }
  return hipSuccess;
}

}  // namespace mh
