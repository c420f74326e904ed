// Writer-pattern calibration (DESIGN.md "The writer's roofline"): the memory traffic of k_emit_tiles with none of its
// formatting — per template two 150-byte haplotype windows gathered at random offsets, two ~369-byte records written
// to two arenas in template order — so the bench's writer time can be set against what the memory system gives for
// this pattern alone.  Variants (each timed with HIP events, best of 5 launches):
//   tile3      the product's shape: 256 threads per 32 templates, waves 1-3 gather (3 threads per window, 7 unrolled
//              16-byte loads) into LDS, one barrier, 4 lanes per record store aligned 16-byte chunks read from LDS
//   tile4      all four waves gather (4 threads per window), then a flat sweep of the tile's contiguous span per file
//   tile4x2    tile4 with 64 templates per 512-thread workgroup
//   stores     tile4's sweep alone (no gathers)
//   gathers    tile4's gathers alone (no stores)
// Sizes: N templates (default 2.93 M, a WGS launch) over a haplotype of H bytes (default 250 MB and 124 MB).
// build: hipcc -O3 --offload-arch=gfx950 -o calib_writer calib_writer.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int RL = 150;
constexpr int WS = 176;   // window stride in LDS (11 chunks)

struct Args {
  const int64_t *pos0, *pos1;   // window starts (haplotype offsets)
  const int32_t *rlen1, *rlen2; // record length per template and file
  const int64_t *tb1, *tb2;     // per tile: arena offset of its first byte per file
  const uint8_t *hap;
  char *out1, *out2;
  int64_t n;
  int mode;                     // 0 full, 1 stores only, 2 gathers only
};

template <int T, int THREADS, int GPW>   // T templates per workgroup, GPW gather threads per window
__global__ void __launch_bounds__(THREADS) k_tile(Args A) {
  __shared__ __attribute__((aligned(16))) char win[T * 2 * WS + 64];
  __shared__ int32_t rel[2][T + 1];
  const int tid = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * T;
  const int nt = (int)(A.n - t0 < T ? A.n - t0 : T);
  // record offsets inside the tile (wave 0; a wave-serial scan is enough for the calibration)
  if (tid < 2) {
    const int32_t *rl = tid ? A.rlen2 : A.rlen1;
    int32_t o = 0;
    for (int j = 0; j < nt; j++) {
      rel[tid][j] = o;
      o += rl[t0 + j];
    }
    rel[tid][nt] = o;
  }
  const int gthreads = T * 2 * GPW;
  const int gbase = THREADS - gthreads;   // gather threads are the last ones
  if (A.mode != 1 && tid >= gbase) {
    const int g = tid - gbase, w = g / GPW, q = g % GPW, j = w >> 1, s = w & 1;
    const int64_t p = j < nt ? (s ? A.pos1[t0 + j] : A.pos0[t0 + j]) : 0;
    const uint8_t *src = A.hap + (p & ~(int64_t)15);
    constexpr int K = (11 + GPW - 1) / GPW;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int c = q + GPW * k;
      v[k] = *(const uint4 *)(src + 16 * (c < 11 ? c : 0));
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int c = q + GPW * k;
      if (c < 11) *(uint4 *)(win + w * WS + 16 * c) = v[k];
    }
  }
  __syncthreads();
  if (A.mode == 2) return;
  // flat sweep of each file's span: chunk c of the span -> 16 bytes from the record's window (unaligned LDS read)
  for (int f = 0; f < 2; f++) {
    char *out = f ? A.out2 : A.out1;
    const int64_t g0 = (f ? A.tb2 : A.tb1)[blockIdx.x];
    const int32_t span = rel[f][nt];
    const int64_t c0 = g0 >> 4, c1 = (g0 + span) >> 4;
    for (int64_t c = c0 + tid; c < c1; c += THREADS) {
      const int32_t x = (int32_t)((c << 4) - g0);
      int lo = 0, hi = nt;   // record holding byte x
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (rel[f][mid] <= (x < 0 ? 0 : x)) lo = mid; else hi = mid;
      }
      const int32_t y = (x < 0 ? 0 : x) - rel[f][lo];
      uint4 v;
      __builtin_memcpy(&v, win + (lo * 2 + f) * WS + (y % 150), 16);
      *(uint4 *)(out + (c << 4)) = v;
    }
  }
}

// the product's sweep shape: 4 lanes per record, 64 records (both files) per pass
__global__ void __launch_bounds__(256) k_tile3(Args A) {
  __shared__ __attribute__((aligned(16))) char win[32 * 2 * WS + 64];
  __shared__ int32_t rel[2][33];
  const int tid = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * 32;
  const int nt = (int)(A.n - t0 < 32 ? A.n - t0 : 32);
  if (tid < 2) {
    const int32_t *rl = tid ? A.rlen2 : A.rlen1;
    int32_t o = 0;
    for (int j = 0; j < nt; j++) {
      rel[tid][j] = o;
      o += rl[t0 + j];
    }
    rel[tid][nt] = o;
  }
  if (tid >= 64) {
    const int g = tid - 64, w = g / 3, q = g % 3, j = w >> 1, s = w & 1;
    const int64_t p = j < nt ? (s ? A.pos1[t0 + j] : A.pos0[t0 + j]) : 0;
    const uint8_t *src = A.hap + (p & ~(int64_t)15);
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int c = q + 3 * k;
      v[k] = *(const uint4 *)(src + 16 * (c < 11 ? c : 0));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int c = q + 3 * k;
      if (c < 11) *(uint4 *)(win + w * WS + 16 * c) = v[k];
    }
  }
  __syncthreads();
  const int r = tid >> 2, q = tid & 3, f = r >> 5, j = r & 31;
  if (j >= nt) return;
  char *out = f ? A.out2 : A.out1;
  const int64_t ga = (f ? A.tb2 : A.tb1)[blockIdx.x] + rel[f][j];
  const int32_t L = rel[f][j + 1] - rel[f][j];
  const int64_t c0 = (ga + 15) >> 4;
  for (int64_t c = c0 + q; (c << 4) + 16 <= ga + L; c += 4) {
    uint4 v;
    __builtin_memcpy(&v, win + (j * 2 + f) * WS + ((int32_t)((c << 4) - ga) % 150), 16);
    *(uint4 *)(out + (c << 4)) = v;
  }
}

// K tiles per 256-thread workgroup, software-pipelined: tile i+1's window gathers (3 x 16 B per thread, registers)
// are issued before tile i's store sweep and land in the other LDS buffer after it
template <int K>
__global__ void __launch_bounds__(256) k_pipe(Args A) {
  __shared__ __attribute__((aligned(16))) char win[2][32 * 2 * WS + 64];
  __shared__ int32_t rel[2][2][33];
  const int tid = threadIdx.x;
  const int64_t nt_all = (A.n + 31) / 32;
  const int64_t tile0 = (int64_t)blockIdx.x * K;
  auto gather = [&](int64_t tile, uint4 *v) {
    const int64_t t0 = tile * 32;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int s = tid + 256 * k;             // slot: window s / 11, chunk s % 11
      const int w = s / 11, c = s - 11 * w, j = w >> 1;
      const bool ok = tile < nt_all && s < 704 && t0 + j < A.n;
      const int64_t p = ok ? ((w & 1) ? A.pos1[t0 + j] : A.pos0[t0 + j]) : 0;
      v[k] = *(const uint4 *)(A.hap + (p & ~(int64_t)15) + 16 * c);
    }
  };
  auto put = [&](int b, const uint4 *v) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int s = tid + 256 * k;
      if (s < 704) *(uint4 *)(win[b] + (s / 11) * WS + 16 * (s % 11)) = v[k];
    }
  };
  auto offsets = [&](int b, int64_t tile) {
    if (tid < 2 && tile < nt_all) {
      const int64_t t0 = tile * 32;
      const int nt = (int)(A.n - t0 < 32 ? A.n - t0 : 32);
      const int32_t *rl = tid ? A.rlen2 : A.rlen1;
      int32_t o = 0;
      for (int j = 0; j < nt; j++) {
        rel[b][tid][j] = o;
        o += rl[t0 + j];
      }
      rel[b][tid][nt] = o;
    }
  };
  uint4 v[3];
  gather(tile0, v);
  offsets(0, tile0);
  put(0, v);
  __syncthreads();
  for (int i = 0; i < K; i++) {
    const int64_t tile = tile0 + i;
    if (tile >= nt_all) break;
    const int b = i & 1;
    if (i + 1 < K) {
      gather(tile + 1, v);
      offsets(b ^ 1, tile + 1);
    }
    const int64_t t0 = tile * 32;
    const int nt = (int)(A.n - t0 < 32 ? A.n - t0 : 32);
    for (int f = 0; f < 2; f++) {
      char *out = f ? A.out2 : A.out1;
      const int64_t g0 = (f ? A.tb2 : A.tb1)[tile];
      const int32_t span = rel[b][f][nt];
      const int64_t c0 = g0 >> 4, c1 = (g0 + span) >> 4;
      for (int64_t c = c0 + tid; c < c1; c += 256) {
        const int32_t x = (int32_t)((c << 4) - g0);
        int lo = 0, hi = nt;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (rel[b][f][mid] <= (x < 0 ? 0 : x)) lo = mid; else hi = mid;
        }
        const int32_t y = (x < 0 ? 0 : x) - rel[b][f][lo];
        uint4 q;
        __builtin_memcpy(&q, win[b] + (lo * 2 + f) * WS + (y % 150), 16);
        *(uint4 *)(out + (c << 4)) = q;
      }
    }
    if (i + 1 < K) put(b ^ 1, v);
    __syncthreads();
  }
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 2926000;
  std::vector<int64_t> Hs = {250000000, 124000000};
  uint64_t s = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  std::vector<int32_t> rl1(n), rl2(n);
  for (int64_t t = 0; t < n; t++) {
    rl1[t] = 360 + (int32_t)(rnd() % 21);
    rl2[t] = 360 + (int32_t)(rnd() % 21);
  }
  int32_t *d_rl1, *d_rl2;
  int64_t *d_p0, *d_p1, *d_tb1, *d_tb2;
  uint8_t *d_hap;
  char *d_o1, *d_o2;
  const int64_t ntile_max = (n + 31) / 32;
  CK(hipMalloc(&d_rl1, 4 * n));
  CK(hipMalloc(&d_rl2, 4 * n));
  CK(hipMalloc(&d_p0, 8 * n));
  CK(hipMalloc(&d_p1, 8 * n));
  CK(hipMalloc(&d_tb1, 8 * (ntile_max + 1)));
  CK(hipMalloc(&d_tb2, 8 * (ntile_max + 1)));
  CK(hipMalloc(&d_hap, Hs[0] + 4096));
  CK(hipMalloc(&d_o1, 400 * n + 4096));
  CK(hipMalloc(&d_o2, 400 * n + 4096));
  CK(hipMemset(d_hap, 'A', Hs[0] + 4096));
  CK(hipMemcpy(d_rl1, rl1.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rl2, rl2.data(), 4 * n, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("{\"n\": %lld, \"results\": [\n", (long long)n);
  bool first = true;
  for (int64_t H : Hs) {
    std::vector<int64_t> p0(n), p1(n);
    for (int64_t t = 0; t < n; t++) {
      const int64_t a = (int64_t)(rnd() % (uint64_t)(H - 800));
      p0[t] = a;
      p1[t] = a + 250 + (int64_t)(rnd() % 300);
    }
    CK(hipMemcpy(d_p0, p0.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_p1, p1.data(), 8 * n, hipMemcpyHostToDevice));
    int64_t bytes_w = 0;
    for (int64_t t = 0; t < n; t++) bytes_w += rl1[t] + rl2[t];
    for (int T : {32, 64}) {
      const int64_t nt = (n + T - 1) / T;
      std::vector<int64_t> tb1(nt + 1), tb2(nt + 1);
      int64_t a1 = 0, a2 = 0;
      for (int64_t b = 0; b < nt; b++) {
        tb1[b] = a1;
        tb2[b] = a2;
        for (int64_t t = b * T; t < std::min(n, (b + 1) * T); t++) {
          a1 += rl1[t];
          a2 += rl2[t];
        }
      }
      CK(hipMemcpy(d_tb1, tb1.data(), 8 * nt, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_tb2, tb2.data(), 8 * nt, hipMemcpyHostToDevice));
      struct V {
        const char *name;
        int mode, T;
      };
      std::vector<V> vs = T == 32 ? std::vector<V>{{"tile3", 0, 32}, {"tile4", 0, 32}, {"stores", 1, 32},
                                                    {"gathers", 2, 32}, {"pipe2", 0, 32}, {"pipe4", 0, 32},
                                                    {"pipe8", 0, 32}}
                                  : std::vector<V>{{"tile4x2", 0, 64}};
      for (const V &v : vs) {
        Args A{d_p0, d_p1, d_rl1, d_rl2, d_tb1, d_tb2, d_hap, d_o1, d_o2, n, v.mode};
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
          CK(hipEventRecord(e0, 0));
          if (!strcmp(v.name, "tile3"))
            hipLaunchKernelGGL(k_tile3, dim3((unsigned)nt), dim3(256), 0, 0, A);
          else if (!strcmp(v.name, "pipe2"))
            hipLaunchKernelGGL(k_pipe<2>, dim3((unsigned)((nt + 1) / 2)), dim3(256), 0, 0, A);
          else if (!strcmp(v.name, "pipe4"))
            hipLaunchKernelGGL(k_pipe<4>, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, 0, A);
          else if (!strcmp(v.name, "pipe8"))
            hipLaunchKernelGGL(k_pipe<8>, dim3((unsigned)((nt + 7) / 8)), dim3(256), 0, 0, A);
          else if (T == 32)
            hipLaunchKernelGGL((k_tile<32, 256, 4>), dim3((unsigned)nt), dim3(256), 0, 0, A);
          else
            hipLaunchKernelGGL((k_tile<64, 512, 4>), dim3((unsigned)nt), dim3(512), 0, 0, A);
          CK(hipGetLastError());
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
        }
        const double alg = (double)bytes_w + 2.0 * RL * n;
        printf("%s{\"variant\": \"%s\", \"hap_bytes\": %lld, \"ms\": %.4f, \"alg_TBps\": %.3f, \"frac\": %.3f}\n",
               first ? "" : ",", v.name, (long long)H, best, alg / (best * 1e-3) / 1e12, alg / (best * 1e-3) / 8e12);
        first = false;
      }
    }
  }
  printf("]}\n");
  return 0;
}
