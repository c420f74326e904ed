// mh_scan.h — generic three-phase device scan (reduce / scan-of-partials / downsweep) with functor load/store.
//
// Every prefix computation on the path goes through this: geometric cumsum (ts), template compaction, node and
// sample-coordinate offsets of the haplotype splice, N-run extraction, and the (kept, bytes1, bytes2) offsets of
// FASTQ emission.  Load(i) produces element i; Store(i, inclusive, exclusive) consumes the prefix, so producers
// and consumers fuse into the scan instead of round-tripping arrays through HBM.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <unordered_map>

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

// Host state of every look-back scratch buffer: the bytes zeroed, the ticket counter's value after the launches
// queued so far, the last epoch.  A buffer is used by one stream at a time (launches on it are stream-ordered).
struct LbScratchState {
  size_t zeroed = 0;
  uint32_t ticket = 0;
  uint32_t epoch = 0;
};
inline std::mutex &lb_mu() {
  static std::mutex m;
  return m;
}
inline std::unordered_map<const void *, LbScratchState> &lb_states() {
  static std::unordered_map<const void *, LbScratchState> m;
  return m;
}
// a device buffer about to be freed (or reallocated): whatever lands at its address later starts unzeroed
inline void lb_forget(const void *p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(lb_mu());
  lb_states().erase(p);
}

// Host launcher.  `partials` must hold ceil(n / SCAN_TILE) elements, `total` one element (device memory).
template <typename T, typename Op, typename Load, typename Store>
inline hipError_t device_scan(hipStream_t st, int64_t n, Load load, Store store, Op op, T identity, T *partials,
                              T *total) {
  lb_forget(partials);   // (a buffer shared with look-back scans: their next use starts from zeroed scratch)
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
  lb_forget(partials);
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL((k_scan_reduce<T, Op, Load>), dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, n, load, op,
                     identity, partials);
  hipLaunchKernelGGL((k_scan_partials<T, Op>), dim3(1), dim3(SCAN_THREADS), 0, st, nb, partials, op, identity,
                     total);
  return hipGetLastError();
}

// ---- single-pass scan (decoupled look-back) for sums of non-negative int64 fields ------------------------------
// One kernel reads every element once: tiles are taken in launch order from an atomic ticket (so every tile a tile
// waits for is already running), each publishes its aggregate, then its inclusive prefix once the look-back over
// its predecessors (one wave, 64 tiles per step) finds an inclusive one.  Status words pack the value with a 16-bit
// launch epoch and a 2-bit flag (1 = aggregate, 2 = inclusive) and travel as 64-bit agent-scope atomics, so no
// fences are needed; the epoch makes the previous launches' words stale, so the scratch is zeroed only when it is
// new (not before every launch: a memset per scan was ~6 us of GPU time each, hundreds per whole-genome step), and
// the ticket counter runs on from launch to launch (each launch subtracts its base).
// T must be a struct of int64 fields, each summed, each in [0, 2^46).
constexpr int LB_ITEMS = 8;
constexpr int LB_TILE = SCAN_THREADS * LB_ITEMS;

template <typename T>
struct LbFields {
  static constexpr int K = sizeof(T) / 8;
  static_assert(sizeof(T) % 8 == 0, "look-back scan element must be int64 fields");
  __device__ static int64_t get(const T &v, int k) { return reinterpret_cast<const int64_t *>(&v)[k]; }
  __device__ static void set(T &v, int k, int64_t x) { reinterpret_cast<int64_t *>(&v)[k] = x; }
};

template <typename T>
__device__ __forceinline__ T shfl_xor_t(const T &v, int d) {
  union U {
    T t;
    int i[sizeof(T) / 4];
    __device__ U() {}
  } a, b;
  a.t = v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) b.i[k] = __shfl_xor(a.i[k], d, 64);
  return b.t;
}

template <typename T>
__device__ __forceinline__ T shfl_idx_t(const T &v, int src) {
  union U {
    T t;
    int i[sizeof(T) / 4];
    __device__ U() {}
  } a, b;
  a.t = v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) b.i[k] = __shfl(a.i[k], src, 64);
  return b.t;
}

constexpr int LB_EPOCH_BITS = 16;
constexpr int LB_VAL_SHIFT = 2 + LB_EPOCH_BITS;

__device__ __forceinline__ void lb_put(uint64_t *w, int64_t v, uint64_t flag, uint32_t epoch) {
  __hip_atomic_store(w, ((uint64_t)v << LB_VAL_SHIFT) | ((uint64_t)epoch << 2) | flag, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// the word's flag if it belongs to this launch (epoch), else 0
__device__ __forceinline__ uint32_t lb_flag(uint64_t w, uint32_t epoch) {
  return (uint32_t)((w >> 2) & ((1u << LB_EPOCH_BITS) - 1)) == epoch ? (uint32_t)(w & 3u) : 0u;
}
__device__ __forceinline__ uint64_t lb_get(const uint64_t *w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// scratch: [ticket (64 B)] [aggregate words K x nt] [inclusive words K x nt], zeroed when new; ticket_base: the
// ticket counter's value when this launch starts; epoch: this launch's tag (1 .. 2^16 - 1)
// Host-mapped words a look-back scan reports a timed-out wait to (a broken ticket base or scratch: the scan's sums
// are then wrong), one per context: the host reads its context's word after a synchronisation (scan_fault_take) and
// fails the call with MH_E_STATE instead of returning the wrong offsets as success, and a fault in one context does
// not fail another's calls.  The word a launch reports to is the calling thread's current context's
// (scan_fault_slot, set by every entry point's guard); slot 0 serves launches outside any context.
constexpr int SCAN_FAULT_SLOTS = 256;
inline thread_local int scan_fault_slot = 0;
inline uint32_t *scan_fault_host() {
  static uint32_t *w = [] {
    uint32_t *p = nullptr;
    if (hipHostMalloc((void **)&p, 4 * SCAN_FAULT_SLOTS, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return (uint32_t *)nullptr;
    for (int i = 0; i < SCAN_FAULT_SLOTS; i++) p[i] = 0;
    return p;
  }();
  return w;
}
inline uint32_t *scan_fault_device() {
  static uint32_t *d = [] {
    uint32_t *h = scan_fault_host(), *p = nullptr;
    if (!h || hipHostGetDevicePointer((void **)&p, h, 0) != hipSuccess) return (uint32_t *)nullptr;
    return p;
  }();
  return d ? d + scan_fault_slot : nullptr;
}
// 1 when a look-back scan of this slot timed out since the last call (the word is cleared)
inline uint32_t scan_fault_take(int slot) {
  uint32_t *h = scan_fault_host();
  if (!h) return 0;
  const uint32_t v = __atomic_exchange_n(h + slot, 0u, __ATOMIC_ACQ_REL);
  return v;
}

template <typename T, typename Load, typename Store>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_lb(int64_t n, Load load, Store store, uint64_t *scratch,
                                                         int64_t nt, T *total, uint32_t ticket_base, uint32_t epoch,
                                                         uint32_t *fault) {
  using F = LbFields<T>;
  constexpr int K = F::K;
  __shared__ T lds_w[SCAN_THREADS / 64];
  __shared__ T s_prefix;
  __shared__ int64_t s_tile;
  uint32_t *ticket = (uint32_t *)scratch;
  uint64_t *agg = scratch + 8, *inc = agg + (size_t)K * nt;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = (int64_t)(uint32_t)(atomicAdd(ticket, 1u) - ticket_base);
  __syncthreads();
  const int64_t tile = s_tile;
  // wave w owns elements [tile * LB_TILE + w * 64 * LB_ITEMS, +64 * LB_ITEMS): item k of lane l is element
  // w * 64 * LB_ITEMS + 64 k + l (coalesced loads and stores), scanned with one wave scan per item
  const int64_t base = tile * LB_TILE + (int64_t)wave * 64 * LB_ITEMS + lane;
  T v[LB_ITEMS];
  T carry{};
  // every item loaded before any is scanned: the loads' latencies overlap instead of alternating with the shuffles
#pragma unroll
  for (int k = 0; k < LB_ITEMS; k++) {
    const int64_t i = base + 64 * k;
    v[k] = i < n ? load(i) : T{};
  }
#pragma unroll
  for (int k = 0; k < LB_ITEMS; k++) {
    T x = v[k];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const T o = shfl_up_t(x, d);
      if (lane >= d) x = o + x;
    }
    v[k] = carry + x;                // inclusive prefix within the wave's segment
    carry = shfl_idx_t(v[k], 63);    // running total of the segment
  }
  if (lane == 0) lds_w[wave] = carry;      // the wave segment's total
  __syncthreads();
  T pre{}, tot{};
#pragma unroll
  for (int w = 0; w < SCAN_THREADS / 64; w++) {
    if (w < wave) pre = pre + lds_w[w];
    tot = tot + lds_w[w];
  }
  // publish and look back (wave 0)
  if (wave == 0) {
    T prefix{};
    if (tile == 0) {
      if (lane < K) lb_put(inc + (size_t)lane * nt, F::get(tot, lane), 2u, epoch);
    } else {
      if (lane < K) lb_put(agg + (size_t)lane * nt + tile, F::get(tot, lane), 1u, epoch);
      for (int64_t j = tile - 1;; j -= 64) {
        const int64_t jj = j - lane;   // lane l looks at tile j - l (jj < 0: past tile 0, never needed)
        bool is_inc = jj < 0, ok = jj < 0;
        T val{};
        uint32_t spins = 0;
        while (!ok) {
          bool all_inc = true, all_agg = true;
          int64_t xi[K], xa[K];
#pragma unroll
          for (int k = 0; k < K; k++) {
            const uint64_t wi = lb_get(inc + (size_t)k * nt + jj);
            const uint64_t wa = lb_get(agg + (size_t)k * nt + jj);
            all_inc &= lb_flag(wi, epoch) == 2u;
            all_agg &= lb_flag(wa, epoch) == 1u;
            xi[k] = (int64_t)(wi >> LB_VAL_SHIFT);
            xa[k] = (int64_t)(wa >> LB_VAL_SHIFT);
          }
          if (all_inc || all_agg) {
            ok = true;
            is_inc = all_inc;
#pragma unroll
            for (int k = 0; k < K; k++) F::set(val, k, all_inc ? xi[k] : xa[k]);
          } else if (++spins > (1u << 24)) {   // (a bound on the wait: reported, never a hung GPU)
            ok = is_inc = true;
            if (fault) __hip_atomic_fetch_or(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          } else {
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const uint64_t bal = __ballot(is_inc);
        const int first = bal ? __builtin_ctzll(bal) : 64;   // nearest tile with an inclusive prefix
        if (lane > first || jj < 0) val = T{};
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) val = val + shfl_xor_t(val, d);
        prefix = prefix + val;
        if (first < 64) break;
      }
      const T mine = prefix + tot;
      if (lane < K) lb_put(inc + (size_t)lane * nt + tile, F::get(mine, lane), 2u, epoch);
    }
    if (lane == 0) s_prefix = prefix;
  }
  __syncthreads();
  const T off = s_prefix + pre;
  // element exclusive prefix = the previous lane's inclusive one (lane 0: the previous item's last lane)
  T prev = off;
#pragma unroll
  for (int k = 0; k < LB_ITEMS; k++) {
    const int64_t i = base + 64 * k;
    const T incl = off + v[k];
    T ex = shfl_up_t(incl, 1);
    if (lane == 0) ex = prev;
    prev = shfl_idx_t(incl, 63);
    if (i < n) store(i, incl, ex);
  }
  if (tile == nt - 1 && tid == SCAN_THREADS - 1) *total = off + v[LB_ITEMS - 1];
}

template <typename T>
inline size_t scan_lb_scratch_bytes(int64_t n) {
  const int64_t nt = (n + LB_TILE - 1) / LB_TILE;
  return 64 + 2 * sizeof(T) * (size_t)(nt < 1 ? 1 : nt) + 64;
}

// Host launcher: exclusive/inclusive sums through Store, grand total to *total.  `scratch` holds
// scan_lb_scratch_bytes<T>(n) bytes of device memory.
// skip_tile0 (self-test only, mh_selftest_scan_fault): the ticket base one below the counter and one workgroup
// fewer, so tile 0 never publishes and every other tile's look-back times out (all accesses stay in range)
// A launch's share of a look-back scratch buffer (`need` bytes, `tiles` tickets): the scratch zeroed on `st` when new,
// grown or out of epochs; the ticket counter's value when the launch starts and its epoch.  (device_scan_sum, and
// the single-pass FASTQ writer, mh_emit.hip)
inline hipError_t lb_reserve(hipStream_t st, void *scratch, size_t need, uint32_t tiles, uint32_t *base,
                             uint32_t *epoch) {
  std::lock_guard<std::mutex> lk(lb_mu());
  LbScratchState &S = lb_states()[scratch];
  if (S.zeroed < need || S.epoch >= (1u << LB_EPOCH_BITS) - 1) {   // new (or grown) scratch, or epochs used up
    hipError_t e = hipMemsetAsync(scratch, 0, need, st);
    if (e != hipSuccess) return e;
    S.zeroed = need;
    S.ticket = 0;
    S.epoch = 0;
  }
  *base = S.ticket;
  *epoch = ++S.epoch;
  S.ticket += tiles;
  return hipSuccess;
}

template <typename T, typename Load, typename Store>
inline hipError_t device_scan_sum(hipStream_t st, int64_t n, Load load, Store store, void *scratch, T *total,
                                  bool skip_tile0 = false) {
  int64_t nt = (n + LB_TILE - 1) / LB_TILE;
  if (nt < 1) nt = 1;
  if (skip_tile0 && nt < 2) return hipErrorInvalidValue;
  const size_t need = scan_lb_scratch_bytes<T>(n);
  uint32_t base, epoch;
  {
    hipError_t e = lb_reserve(st, scratch, need, (uint32_t)(skip_tile0 ? nt - 1 : nt), &base, &epoch);
    if (e != hipSuccess) return e;
    if (skip_tile0) base -= 1u;
  }
  hipLaunchKernelGGL((k_scan_lb<T, Load, Store>), dim3((unsigned)(skip_tile0 ? nt - 1 : nt)), dim3(SCAN_THREADS), 0,
                     st, n, load, store, (uint64_t *)scratch, nt, total, base, epoch, scan_fault_device());
  return hipGetLastError();
}

inline int64_t scan_partials_count(int64_t n) {
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  return nb < 1 ? 1 : nb;
}

}  // namespace mh
