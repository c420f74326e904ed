// FETCH_SIZE calibration for the access widths the writer uses (MI355X_MICROARCH.md § HBM says FETCH_SIZE reads
// 1/2 of the bytes of a wide coalesced streaming read and leaves other widths uncalibrated).  Four read kernels over
// an 8 GiB buffer (far past the 256 MiB Infinity Cache), each timed with HIP events; run under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./calib_fetch
// and compare each kernel's FETCH_SIZE with the bytes it must bring from HBM:
//   k_stream   16 B per lane, consecutive: every byte once                          (B bytes)
//   k_line     one 16-byte load per 128-byte line                                   (B bytes if whole lines move)
//   k_half     one 16-byte load per 64-byte half line                               (same lines as k_line)
//   k_window   150-byte windows (ten 16-byte loads, as the writer gathers a read) at random 16-byte-aligned
//              offsets, one window per 4 KiB page, so windows never share a line: 2 or 3 lines each
// build: hipcc -O3 --offload-arch=gfx950 -o calib_fetch calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_stream(const uint4 *a, int64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;   // (never: keeps the loads)
}

__global__ void k_stride(const char *a, int64_t n_loads, int64_t stride, uint32_t *sink) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_loads; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = *(const uint4 *)(a + i * stride);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void k_window(const char *a, int64_t n_win, uint32_t *sink, int64_t *lines) {
  uint32_t acc = 0;
  int64_t nl = 0;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_win; w += (int64_t)gridDim.x * blockDim.x) {
    // window w in page w (4 KiB), at a hashed 16-byte-aligned offset that leaves room for 160 bytes
    uint32_t h = (uint32_t)w * 2654435761u;
    h ^= h >> 15;
    const int64_t off = w * 4096 + (int64_t)(h % 246u) * 16;
    const int64_t first = off >> 7, last = (off + 150 - 1) >> 7;
    nl += last - first + 1;
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const uint4 v = *(const uint4 *)(a + off + 16 * k);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
  atomicAdd((unsigned long long *)lines, (unsigned long long)nl);
}

int main() {
  const int64_t B = 8ll << 30;
  char *a = nullptr;
  uint32_t *sink = nullptr;
  int64_t *lines = nullptr;
  CK(hipMalloc(&a, B));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&lines, 64));
  CK(hipMemset(a, 1, B));
  CK(hipMemset(lines, 0, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(256 * 16), block(256);
  float ms[4];
  for (int rep = 0; rep < 2; rep++) {   // (the second round is the one to read)
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stream, grid, block, 0, 0, (const uint4 *)a, B / 16, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[0], e0, e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stride, grid, block, 0, 0, (const char *)a, B / 128, (int64_t)128, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[1], e0, e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stride, grid, block, 0, 0, (const char *)a, B / 64, (int64_t)64, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[2], e0, e1));
    CK(hipMemset(lines, 0, 64));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_window, grid, block, 0, 0, (const char *)a, B / 4096, sink, lines);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[3], e0, e1));
  }
  int64_t nl = 0;
  CK(hipMemcpy(&nl, lines, 8, hipMemcpyDeviceToHost));
  printf("{\"buffer_bytes\": %lld, \"k_stream\": {\"ms\": %.4f, \"bytes\": %lld}, "
         "\"k_line\": {\"ms\": %.4f, \"loads\": %lld, \"line_bytes\": %lld}, "
         "\"k_half\": {\"ms\": %.4f, \"loads\": %lld, \"line_bytes\": %lld}, "
         "\"k_window\": {\"ms\": %.4f, \"windows\": %lld, \"line_bytes\": %lld, \"window_bytes\": %lld}}\n",
         (long long)B, ms[0], (long long)B, ms[1], (long long)(B / 128), (long long)B, ms[2], (long long)(B / 64),
         (long long)B, ms[3], (long long)(B / 4096), (long long)(nl * 128), (long long)(B / 4096 * 150));
  return 0;
}
