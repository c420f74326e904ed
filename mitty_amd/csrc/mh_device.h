// mh_device.h — small device-side helpers shared by the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

namespace mh {

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations, not for its global
// stores.  __syncthreads() also waits for every outstanding global store of the wave (vmcnt(0)), which puts a full
// memory round trip on every barrier of a kernel that streams results out between barriers.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace mh
