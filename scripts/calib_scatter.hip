// Write-pattern calibration for a position-ordered FASTQ writer (DESIGN.md "writer traffic"): the same ~370-byte
// records (5.9 M per file, 2 files: one chr1 unit's FASTQ) written
//   seq   in file order: a 256-thread workgroup writes 32 consecutive records (the tile writer's pattern)
//   rnd   in a random order: a workgroup writes 32 records at random places (a writer walking templates by position)
// interior 16-byte chunks as aligned 16-byte stores, a record's ragged first and last chunks as byte stores (its
// neighbours belong to other workgroups), and the reads of a tile writer:
//   gwin  two 150-byte windows per template at random offsets of a 498 MB haplotype pair (the current gathers)
//   swin  the same windows with the templates walked in position order (consecutive windows ~42 bytes apart)
// Each kernel timed with HIP events (last of three rounds).
// build: hipcc -O3 --offload-arch=gfx950 -o calib_scatter calib_scatter.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

// record r of file f: [off[f][r], off[f][r+1]); order[] maps the workgroup's k-th record to a record index
__global__ void __launch_bounds__(256) k_write(const int64_t *off, int64_t nrec, const uint32_t *order, char *out) {
  const int64_t t0 = (int64_t)blockIdx.x * 32;
  const int lane = threadIdx.x & 7, rl = threadIdx.x >> 3;   // 8 lanes per record, 32 records
  const int64_t k = t0 + rl;
  if (k >= nrec) return;
  const int64_t r = order ? order[k] : k;
  const int64_t a = off[r], b = off[r + 1];
  const uint4 v = make_uint4(0x41414141u ^ (uint32_t)r, 0x43434343u, 0x47474747u, 0x54545454u);
  const int64_t c0 = (a + 15) >> 4, c1 = b >> 4;   // whole chunks [c0, c1)
  for (int64_t c = c0 + lane; c < c1; c += 8) *(uint4 *)(out + (c << 4)) = v;
  if (lane == 0)
    for (int64_t x = a; x < (c0 << 4) && x < b; x++) out[x] = '@';
  if (lane == 1 && c1 >= c0)
    for (int64_t x = c1 << 4; x < b; x++) out[x] = '\n';
}

// two 150-byte windows per template from a hap / rc pair; pos[] in template order (random or sorted)
__global__ void __launch_bounds__(256) k_win(const int64_t *pos, int64_t n, const char *hap, const char *rc,
                                             int64_t L, uint32_t *sink) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t t = g / 6;   // 3 threads per window, 2 windows per template
  if (t >= n) return;
  const int w = (int)(g % 6) / 3, q = (int)(g % 3);
  const int64_t p = w ? L - pos[t] - 300 : pos[t];
  const char *src = (w ? rc : hap) + (p & ~(int64_t)15);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int c = q + 3 * k;
    if (c < 10) {
      const uint4 v = *(const uint4 *)(src + 16 * c);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main() {
  const int64_t nrec = 5890000;   // one chr1 unit's templates, one file
  std::vector<int64_t> off(nrec + 1);
  std::vector<uint32_t> ord(nrec);
  uint64_t s = 0x12345678ull;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  off[0] = 0;
  for (int64_t r = 0; r < nrec; r++) off[r + 1] = off[r] + 360 + (int64_t)(rnd() % 21);
  for (int64_t r = 0; r < nrec; r++) ord[r] = (uint32_t)r;
  for (int64_t r = nrec - 1; r > 0; r--) std::swap(ord[r], ord[rnd() % (uint64_t)(r + 1)]);
  const int64_t B = off[nrec];
  const int64_t L = 249250621;
  std::vector<int64_t> pr(nrec), ps(nrec);
  for (int64_t r = 0; r < nrec; r++) ps[r] = (int64_t)((double)r / nrec * (L - 1000));
  for (int64_t r = 0; r < nrec; r++) pr[r] = ps[ord[r]];
  int64_t *d_off, *d_pr, *d_ps;
  uint32_t *d_ord, *sink;
  char *out, *hap, *rc;
  CK(hipMalloc(&d_off, 8 * (nrec + 1)));
  CK(hipMalloc(&d_pr, 8 * nrec));
  CK(hipMalloc(&d_ps, 8 * nrec));
  CK(hipMalloc(&d_ord, 4 * nrec));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&out, 2 * B + 64));
  CK(hipMalloc(&hap, L + 4096));
  CK(hipMalloc(&rc, L + 4096));
  CK(hipMemcpy(d_off, off.data(), 8 * (nrec + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ord, ord.data(), 4 * nrec, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pr, pr.data(), 8 * nrec, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ps, ps.data(), 8 * nrec, hipMemcpyHostToDevice));
  CK(hipMemset(hap, 'A', L + 4096));
  CK(hipMemset(rc, 'T', L + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned gw = (unsigned)((nrec + 31) / 32), gr = (unsigned)((6 * nrec + 255) / 256);
  float ms[4] = {0, 0, 0, 0};
  for (int rep = 0; rep < 3; rep++) {
    for (int m = 0; m < 4; m++) {
      CK(hipEventRecord(e0));
      if (m < 2)
        for (int f = 0; f < 2; f++)   // two files, as a writer launch writes
          hipLaunchKernelGGL(k_write, dim3(gw), dim3(256), 0, 0, d_off, nrec, m ? d_ord : nullptr, out + f * B);
      else
        hipLaunchKernelGGL(k_win, dim3(gr), dim3(256), 0, 0, m == 2 ? d_pr : d_ps, nrec, hap, rc, L, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[m], e0, e1));
    }
  }
  CK(hipGetLastError());
  printf("{\"records_per_file\": %lld, \"bytes_per_file\": %lld, \"seq_write_ms\": %.4f, \"rnd_write_ms\": %.4f, "
         "\"write_TBps_seq\": %.3f, \"write_TBps_rnd\": %.3f, \"gwin_ms\": %.4f, \"swin_ms\": %.4f, "
         "\"window_bytes\": %lld}\n",
         (long long)nrec, (long long)B, ms[0], ms[1], 2.0 * B / ms[0] / 1e9, 2.0 * B / ms[1] / 1e9, ms[2], ms[3],
         (long long)(nrec * 300));
  return 0;
}
