// mh_corrupt.hip — standalone `corrupt-reads` over existing FASTQ (reference readcorrupt.py:18-118, cli.py:144-157;
// SURVEY.md §8(f) rank 2), Philox mode.
//
//   FASTQ chunk(s) -> newline index (mh_bam.hip) -> k_cr_measure (thread per template: file 1's read name, each
//   file's sequence span, output record sizes) -> scan -> k_cr_write (wave per record: '@' name, the corrupted
//   sequence, '+', the BQ string) appended to the context's FASTQ arenas.
//
// The reference sends (file 1's name, seq1[, seq2]) to corrupt_template (readcorrupt.py:53-54, illumina.py:113-127)
// and writes '@{name}\n{seq}\n+\n{bq}\n' per mate (readcorrupt.py:112-114): both output files carry file 1's name,
// the mate index selects the BQ table, the input qualities are dropped.  Each base pair goes through corrupt_pair
// (mh_corrupt.h) counted by (template index in the whole input, file, base).
#include "mh_corrupt.h"
#include "mh_internal.h"
#include "mh_scan.h"

namespace mh {
namespace {

struct CrTpl {
  int64_t name_off;        // file 1, after '@'
  int64_t seq_off[2];
  int32_t name_len;
  int32_t len[2];
  int32_t size[2];         // output record bytes per file
};

enum { CE_FORMAT = 1, CE_LONG = 2 };

__device__ __forceinline__ int64_t ln_start(const int64_t *nl, int64_t line) { return line == 0 ? 0 : nl[line - 1] + 1; }

__global__ void __launch_bounds__(256) k_cr_measure(const uint8_t *b0, const int64_t *nl0, const uint8_t *b1,
                                                    const int64_t *nl1, int32_t nf, int64_t T, int32_t max_bp,
                                                    CrTpl *tpl, int32_t *err) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  CrTpl o;
  int32_t e = 0;
  const int64_t s = ln_start(nl0, 4 * t), q1e = nl0[4 * t];
  if (q1e <= s || b0[s] != '@') e |= CE_FORMAT;
  int64_t q = s + 1;
  while (q < q1e && b0[q] != ' ' && b0[q] != '\t') q++;   // FastxFile .name
  o.name_off = s + 1;
  o.name_len = (int32_t)(q - s - 1);
  for (int f = 0; f < 2; f++) {
    o.seq_off[f] = 0;
    o.len[f] = 0;
    o.size[f] = 0;
    if (f >= nf) continue;
    const int64_t *nl = f ? nl1 : nl0;
    const int64_t a = ln_start(nl, 4 * t + 1), z = nl[4 * t + 1];
    o.seq_off[f] = a;
    o.len[f] = (int32_t)(z - a);
    if (o.len[f] > max_bp) e |= CE_LONG;
    o.size[f] = 1 + o.name_len + 1 + o.len[f] + 3 + o.len[f] + 1;
  }
  tpl[t] = o;
  if (e) atomicOr(err, e);
}

struct Off2 {
  int64_t a, b;
  __device__ Off2 operator+(const Off2 &o) const { return Off2{a + o.a, b + o.b}; }
};
struct LoadCr {
  const CrTpl *tpl;
  int64_t n;
  __device__ Off2 operator()(int64_t t) const { return t < n ? Off2{tpl[t].size[0], tpl[t].size[1]} : Off2{0, 0}; }
};
struct StoreCr {
  Off2 *off;
  __device__ void operator()(int64_t t, Off2, Off2 excl) const { off[t] = excl; }
};

__global__ void __launch_bounds__(256) k_cr_write(const uint8_t *b0, const uint8_t *b1, const CrTpl *tpl, int64_t T,
                                                  int32_t nf, const Off2 *off, char *out0, char *out1,
                                                  CorruptCfg cc) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= T * nf) return;
  const int64_t t = i / nf;
  const int f = (int)(i % nf);
  const CrTpl &c = tpl[t];
  char *d = (f ? out1 + off[t].b : out0 + off[t].a);
  const uint8_t *nm = b0 + c.name_off;
  const uint8_t *sq = (f ? b1 : b0) + c.seq_off[f];
  const int32_t nl = c.name_len, L = c.len[f];
  if (lane == 0) d[0] = '@';
  for (int32_t k = lane; k < nl; k += 64) d[1 + k] = (char)nm[k];
  char *ds = d + 1 + nl + 1;
  char *dq = ds + L + 3;
  if (lane == 0) {
    d[1 + nl] = '\n';
    ds[L] = '\n'; ds[L + 1] = '+'; ds[L + 2] = '\n';
    dq[L] = '\n';
  }
  for (int32_t k = 2 * lane; k < L; k += 128) {   // base pairs: one Philox draw each
    const int cnt = L - k > 1 ? 2 : 1;
    uint8_t b[2] = {sq[k], cnt > 1 ? sq[k + 1] : (uint8_t)0}, qq[2];
    corrupt_pair(cc, t, f, k, cnt, b, qq);
    ds[k] = (char)b[0];
    dq[k] = (char)qq[0];
    if (cnt > 1) {
      ds[k + 1] = (char)b[1];
      dq[k + 1] = (char)qq[1];
    }
  }
}

}  // namespace

int32_t corrupt_fastq(mh_ctx *ctx, const uint8_t *d0, int64_t len0, const uint8_t *d1, int64_t len1, int64_t t_base,
                      int64_t *used0, int64_t *used1, int64_t *templates) {
  hipStream_t st = ctx->stream;
  BamStore &B = ctx->bam;   // staging + newline buffers are shared with the BAM builder
  *used0 = *used1 = *templates = 0;
  if (!ctx->corrupt_on) return arg_fail(ctx, MH_E_STATE, "corruption model not set (mh_set_corruption)");
  const int32_t nf = d1 ? 2 : 1;
  int64_t n0 = 0, n1 = 0;
  stage_begin(ctx, "corrupt_index");
  MH_TRY(newline_index(ctx, d0, len0, B.nl1, &n0));
  if (d1) MH_TRY(newline_index(ctx, d1, len1, B.nl2, &n1));
  stage_end(ctx);
  int64_t T = n0 / 4;
  if (d1 && n1 / 4 < T) T = n1 / 4;
  if (T == 0) return MH_OK;
  MH_TRY(ensure(ctx, B.tpl, sizeof(CrTpl) * T));
  MH_TRY(ensure(ctx, ctx->s[13], sizeof(Off2) * (T + 1)));
  MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(Off2) * scan_partials_count(T + 1) + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int32_t *err = (int32_t *)((char *)ctx->d_small.p + 64);
  HIPCHK(ctx, hipMemsetAsync(err, 0, 4, st));
  CrTpl *tpl = (CrTpl *)B.tpl.p;
  stage_begin(ctx, "corrupt_measure");
  hipLaunchKernelGGL(k_cr_measure, dim3(grid_for(T, 256, INT32_MAX)), dim3(256), 0, st, d0, (const int64_t *)B.nl1.p,
                     d1, d1 ? (const int64_t *)B.nl2.p : nullptr, nf, T, ctx->corrupt_max_bp, tpl, err);
  HIPCHK(ctx, hipGetLastError());
  Off2 *off = (Off2 *)ctx->s[13].p;
  HIPCHK(ctx, device_scan<Off2>(st, T + 1, LoadCr{tpl, T}, StoreCr{off}, OpSum{}, Off2{0, 0},
                                (Off2 *)ctx->scan_partials.p, (Off2 *)ctx->d_small.p));
  stage_end(ctx);
  int32_t herr = 0;
  Off2 tot;
  int64_t last0 = 0, last1 = 0;
  HIPCHK(ctx, hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(&tot, off + T, sizeof(Off2), hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(&last0, (const int64_t *)B.nl1.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  if (d1) HIPCHK(ctx, hipMemcpyAsync(&last1, (const int64_t *)B.nl2.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (herr & CE_LONG) return arg_fail(ctx, MH_E_ARG, "read longer than the BQ model (illumina.corrupt_single_read)");
  if (herr) return arg_fail(ctx, MH_E_ARG, "malformed FASTQ record");
  MH_TRY(ensure_keep(ctx, ctx->out1, ctx->used1 + tot.a + 64, ctx->used1));
  if (d1) MH_TRY(ensure_keep(ctx, ctx->out2, ctx->used2 + tot.b + 64, ctx->used2));
  const uint64_t key = 0x636f7272757074ull;   // fixed unit key of the standalone tool
  CorruptCfg cc{1, (const float *)ctx->corrupt_cum.p, (const double *)ctx->corrupt_phred.p, ctx->corrupt_max_bp,
                ctx->corrupt_n_bq, (uint32_t)ctx->corrupt_seed, (uint32_t)key,
                (uint32_t)(ctx->corrupt_seed >> 32) ^ (uint32_t)(key >> 32) ^ 0x636f7272u, t_base};
  cc.guide = (const uint16_t *)((const char *)ctx->corrupt_cum.p + ctx->corrupt_guide_off);
  stage_begin(ctx, "corrupt_write");
  hipLaunchKernelGGL(k_cr_write, dim3(grid_for(T * nf * 64, 256, INT32_MAX)), dim3(256), 0, st, d0, d1,
                     (const CrTpl *)tpl, T, nf, (const Off2 *)off, (char *)ctx->out1.p + ctx->used1,
                     d1 ? (char *)ctx->out2.p + ctx->used2 : nullptr, cc);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  HIPCHK(ctx, hipStreamSynchronize(st));
  ctx->used1 += tot.a;
  if (d1) ctx->used2 += tot.b;
  *used0 = last0 + 1;
  *used1 = d1 ? last1 + 1 : 0;
  *templates = T;
  return MH_OK;
}

}  // namespace mh
