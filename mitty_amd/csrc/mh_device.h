// mh_device.h — small device-side helpers shared by the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <rocprim/warp/warp_scan.hpp>

namespace mh {

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations, not for its global
// stores.  __syncthreads() also waits for every outstanding global store of the wave (vmcnt(0)), which puts a full
// memory round trip on every barrier of a kernel that streams results out between barriers.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 0xff in every byte of x equal to the byte replicated in c
__device__ __forceinline__ uint32_t byte_eq(uint32_t x, uint32_t c) {
  const uint32_t y = x ^ c;
  const uint32_t t = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
  return (t >> 7) * 0xffu;
}

// str.maketrans('ATCGN', 'TAGCN') on four bytes at once ('A'^'T' = 0x15, 'C'^'G' = 0x04; others unchanged)
__device__ __forceinline__ uint32_t comp4(uint32_t x) {
  const uint32_t at = byte_eq(x, 0x41414141u) | byte_eq(x, 0x54545454u);
  const uint32_t cg = byte_eq(x, 0x43434343u) | byte_eq(x, 0x47474747u);
  return x ^ (at & 0x15151515u) ^ (cg & 0x04040404u);
}

// 16 bytes from an arbitrarily aligned global address: five dword loads from the dword below it + v_alignbyte.
// Reads up to 3 bytes before and 4 bytes after the range (callers' buffers are padded).
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t *a) {
  const uint32_t *q = (const uint32_t *)((uintptr_t)a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)((uintptr_t)a & 3u);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                    __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// Inclusive sum across the 64 lanes of a wave (DPP row shifts and broadcasts: rocprim's cross-lane warp scan; the
// __shfl_up loop it replaces is six ds_bpermute round trips); `total` = the wave's sum, in every lane.
__device__ __forceinline__ int wave_sum_incl(int v, int &total) {
  using WS = rocprim::warp_scan<int, 64>;
  typename WS::storage_type none;
  int out;
  WS().inclusive_scan(v, out, total, none);
  return out;
}

}  // namespace mh
