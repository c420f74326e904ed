// Throughput of the integer multiplies a Philox round can be built from, on gfx950 (not the product: a measurement
// for the corruption rows' draw cost).  Every wave runs 8 independent chains of one instruction kind; the grid fills
// every SIMD.  Prints cycles per wave64 instruction per SIMD (clock from hipDeviceProp clockRate, a nominal figure:
// the v_add_u32 row calibrates it, 2 cycles on a SIMD-32).
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_mul.hip -o /tmp/ubench_mul && /tmp/ubench_mul
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

#define CHAINS8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_mad64(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c)                                                                              \
  {                                                                                        \
    uint64_t p;                                                                            \
    asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(p) : "v"(v[c]), "s"(s) : "s0", "s1"); \
    v[c] = (uint32_t)p ^ (uint32_t)(p >> 32);                                              \
  }
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_mulhi(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_mullo(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_mul24(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_fma64(uint32_t *out, double s) {
  double v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  double x = 0;
  for (int c = 0; c < 8; c++) x += v[c];
  if (x == 1.2345) out[0] = 1;
}

__global__ void k_cvt64(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  double d[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[c]) : "v"(v[c])); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(((uint32_t *)&d[c])[1]));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

__global__ void k_xor(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITERS; i++) {
#define ST(c) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "s"(s));
    CHAINS8(ST)
#undef ST
  }
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= v[c];
  if (x == 0x12345678u) out[0] = x;
}

template <typename F>
static void run(const char *name, F launch, int per_iter_instrs, double clk_ghz, int n_simd) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const int blocks = 4096, threads = 256;
  const double waves = (double)blocks * threads / 64;
  const double instrs = waves * ITERS * 8.0 * per_iter_instrs;
  const double cyc = ms * 1e-3 * clk_ghz * 1e9 * n_simd / instrs;
  printf("%-8s %8.3f ms  %6.2f cycles per wave64 instruction per SIMD\n", name, ms, cyc);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const double ghz = p.clockRate / 1e6;
  const int n_simd = p.multiProcessorCount * 4;
  printf("%s  CUs %d  clock %.3f GHz (nominal)\n", p.gcnArchName, p.multiProcessorCount, ghz);
  uint32_t *out;
  hipMalloc(&out, 64);
  const dim3 g(4096), b(256);
  run("add", [&] { hipLaunchKernelGGL(k_add, g, b, 0, 0, out, 3u); }, 1, ghz, n_simd);
  run("xor", [&] { hipLaunchKernelGGL(k_xor, g, b, 0, 0, out, 3u); }, 1, ghz, n_simd);
  run("mul24", [&] { hipLaunchKernelGGL(k_mul24, g, b, 0, 0, out, 0x9E3779u); }, 1, ghz, n_simd);
  run("mullo", [&] { hipLaunchKernelGGL(k_mullo, g, b, 0, 0, out, 0xD2511F53u); }, 1, ghz, n_simd);
  run("mulhi", [&] { hipLaunchKernelGGL(k_mulhi, g, b, 0, 0, out, 0xD2511F53u); }, 1, ghz, n_simd);
  // mad64 chain: one mad + one xor per link
  run("mad64+x", [&] { hipLaunchKernelGGL(k_mad64, g, b, 0, 0, out, 0xD2511F53u); }, 1, ghz, n_simd);
  run("fma64", [&] { hipLaunchKernelGGL(k_fma64, g, b, 0, 0, out, 1.0000001); }, 1, ghz, n_simd);
  run("cvt64+x", [&] { hipLaunchKernelGGL(k_cvt64, g, b, 0, 0, out, 3u); }, 1, ghz, n_simd);
  hipFree(out);
  return 0;
}
