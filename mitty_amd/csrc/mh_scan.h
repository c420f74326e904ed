// mh_scan.h — generic three-phase device scan (reduce / scan-of-partials / downsweep) with functor load/store.
//
// Every prefix computation on the path goes through this: geometric cumsum (ts), template compaction, node and
// sample-coordinate offsets of the haplotype splice, N-run extraction, and the (kept, bytes1, bytes2) offsets of
// FASTQ emission.  Load(i) produces element i; Store(i, inclusive, exclusive) consumes the prefix, so producers
// and consumers fuse into the scan instead of round-tripping arrays through HBM.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mh {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

template <typename T>
__device__ __forceinline__ T shfl_up_t(const T &v, int d) {
  static_assert(sizeof(T) % 4 == 0, "scan element must be a multiple of 4 bytes");
  union U {
    T t;
    int i[sizeof(T) / 4];
    __device__ U() {}
  } a, b;
  a.t = v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) b.i[k] = __shfl_up(a.i[k], d, 64);
  return b.t;
}

struct OpSum {
  template <typename T>
  __device__ __forceinline__ T operator()(const T &a, const T &b) const { return a + b; }
};
struct OpMax {
  template <typename T>
  __device__ __forceinline__ T operator()(const T &a, const T &b) const { return a > b ? a : b; }
};

// Inclusive scan across the 256-thread block; returns the block total through `total`.
template <typename T, typename Op>
__device__ __forceinline__ T block_inclusive_scan(T v, Op op, T identity, T *lds_waves, T &total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T o = shfl_up_t(v, d);
    if (lane >= d) v = op(o, v);
  }
  if (lane == 63) lds_waves[wave] = v;
  __syncthreads();
  T pre = identity;
  for (int w = 0; w < wave; w++) pre = op(pre, lds_waves[w]);
  total = identity;
  for (int w = 0; w < SCAN_THREADS / 64; w++) total = op(total, lds_waves[w]);
  __syncthreads();
  return op(pre, v);
}

template <typename T, typename Op, typename Load>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(int64_t n, Load load, Op op, T identity, T *partials) {
  __shared__ T lds_w[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  T acc = identity;
#pragma unroll 4
  for (int k = 0; k < SCAN_ITEMS; k++) {
    int64_t i = base + (int64_t)k * SCAN_THREADS + threadIdx.x;
    if (i < n) acc = op(acc, load(i));
  }
  T total;
  block_inclusive_scan(acc, op, identity, lds_w, total);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// Exclusive scan of the per-block partials in place (single block); grand total to *total_out.
template <typename T, typename Op>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_partials(int64_t nb, T *partials, Op op, T identity,
                                                               T *total_out) {
  __shared__ T lds_w[SCAN_THREADS / 64];
  __shared__ T lds_incl[SCAN_THREADS];
  T carry = identity;
  for (int64_t b0 = 0; b0 < nb; b0 += SCAN_THREADS) {
    int64_t i = b0 + threadIdx.x;
    T v = i < nb ? partials[i] : identity;
    T tot;
    T incl = block_inclusive_scan(v, op, identity, lds_w, tot);
    lds_incl[threadIdx.x] = incl;
    __syncthreads();
    T excl = threadIdx.x ? lds_incl[threadIdx.x - 1] : identity;
    if (i < nb) partials[i] = op(carry, excl);
    carry = op(carry, tot);
    __syncthreads();
  }
  if (threadIdx.x == 0) *total_out = carry;
}

template <typename T, typename Op, typename Load, typename Store>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_down(int64_t n, Load load, Store store, Op op, T identity,
                                                           const T *partials) {
  __shared__ T lds_w[SCAN_THREADS / 64];
  __shared__ T lds_incl[SCAN_THREADS];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  T carry = partials[blockIdx.x];
  for (int k = 0; k < SCAN_ITEMS; k++) {
    int64_t i = base + (int64_t)k * SCAN_THREADS + threadIdx.x;
    if (base + (int64_t)k * SCAN_THREADS >= n) break;   // block-uniform
    T v = i < n ? load(i) : identity;
    T tot;
    T incl = block_inclusive_scan(v, op, identity, lds_w, tot);
    lds_incl[threadIdx.x] = incl;
    __syncthreads();
    T excl = threadIdx.x ? lds_incl[threadIdx.x - 1] : identity;
    if (i < n) store(i, op(carry, incl), op(carry, excl));
    carry = op(carry, tot);
    __syncthreads();
  }
}

// Host launcher.  `partials` must hold ceil(n / SCAN_TILE) elements, `total` one element (device memory).
template <typename T, typename Op, typename Load, typename Store>
inline hipError_t device_scan(hipStream_t st, int64_t n, Load load, Store store, Op op, T identity, T *partials,
                              T *total) {
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL((k_scan_reduce<T, Op, Load>), dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, n, load, op,
                     identity, partials);
  hipLaunchKernelGGL((k_scan_partials<T, Op>), dim3(1), dim3(SCAN_THREADS), 0, st, nb, partials, op, identity,
                     total);
  hipLaunchKernelGGL((k_scan_down<T, Op, Load, Store>), dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, n, load,
                     store, op, identity, (const T *)partials);
  return hipGetLastError();
}

// Reduction only (phases 1-2): grand total to *total.
template <typename T, typename Op, typename Load>
inline hipError_t device_reduce(hipStream_t st, int64_t n, Load load, Op op, T identity, T *partials, T *total) {
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL((k_scan_reduce<T, Op, Load>), dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, n, load, op,
                     identity, partials);
  hipLaunchKernelGGL((k_scan_partials<T, Op>), dim3(1), dim3(SCAN_THREADS), 0, st, nb, partials, op, identity,
                     total);
  return hipGetLastError();
}

inline int64_t scan_partials_count(int64_t n) {
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  return nb < 1 ? 1 : nb;
}

}  // namespace mh
