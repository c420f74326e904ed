// mh_corrupt.hip — standalone `corrupt-reads` over existing FASTQ (reference readcorrupt.py:18-118, cli.py:144-157;
// SURVEY.md §8(f) rank 2).
//
//   FASTQ chunk(s) -> newline index (mh_bam.hip) -> k_cr_measure (thread per template: file 1's read name, each
//   file's sequence span, output record sizes) -> scan -> k_cr_write (wave per record: '@' name, the corrupted
//   sequence, '+', the BQ string) appended to the context's FASTQ arenas.
//
// The reference sends (file 1's name, seq1[, seq2]) to corrupt_template (readcorrupt.py:53-54, illumina.py:113-127)
// and writes '@{name}\n{seq}\n+\n{bq}\n' per mate (readcorrupt.py:112-114): both output files carry file 1's name,
// the mate index selects the BQ table, the input qualities are dropped.
//
// Two word sources (mh_corrupt.h has the per-base arithmetic, identical in both):
//   Philox  counted by (template index in the whole input, file, base): any chunking, any launch geometry
//   exact   the reference's single-worker stream (readcorrupt.py:84, processes=1): one MT19937 stream consumed
//           template by template, mate 0 then mate 1, per mate rand(n), rand(n), randint(0, 3, n) — 4n words for
//           the two uniforms, then n accepted words of random_interval(2) (a word w is accepted when w & 3 != 3).
//           The stream is generated on the device (jump-ahead segments, or twisted on from an explicit state);
//           k_cx_bits marks the accepted words; k_cx_chain walks the mates in order (one wave: each mate's end is
//           the n-th accepted word after its uniforms, found by a popcount scan over the bitmap staged in LDS); then
//           every record is corrupted in parallel from its start offset (k_cr_write<true>).
#include <algorithm>
#include <cmath>

#include "mh_corrupt.h"
#include "mh_device.h"
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

struct Off3 {
  int64_t a, b, m;   // record bytes of file 1, of file 2; bases of both files (exact mode's stream length)
  __device__ Off3 operator+(const Off3 &o) const { return Off3{a + o.a, b + o.b, m + o.m}; }
};
struct LoadCr {
  const CrTpl *tpl;
  int64_t n;
  __device__ Off3 operator()(int64_t t) const {
    return t < n ? Off3{tpl[t].size[0], tpl[t].size[1], (int64_t)tpl[t].len[0] + tpl[t].len[1]} : Off3{0, 0, 0};
  }
};
struct StoreCr {
  Off3 *off;
  __device__ void operator()(int64_t t, Off3, Off3 excl) const { off[t] = excl; }
};

// ---- exact mode ---------------------------------------------------------------------------------------------------
// bits[i] bit j = 1 when stream word 64 i + j is an accepted random_interval(2) draw (w & 3 != 3)
__global__ void __launch_bounds__(256) k_cx_bits(const uint32_t *w, int64_t nw, uint64_t *bits, int64_t n64) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool acc = g < nw && (w[g] & 3u) != 3u;
  const uint64_t m = __ballot(acc);
  if ((threadIdx.x & 63) == 0 && (g >> 6) < n64) bits[g >> 6] = m;
}

// position (0..63) of the r-th set bit (1-based) of v
__device__ __forceinline__ int select_bit(uint64_t v, int r) {
  int p = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(v & ((1ull << w) - 1ull));
    if (r > c) {
      r -= c;
      v >>= w;
      p += w;
    }
  }
  return p;
}

constexpr int CX_WIN = 8192;   // bitmap words per LDS window: 64 KB = 524,288 stream words

// mstart[k] = first stream word of mate k (k = t * nf + f, the reference's consumption order), mstart[K] = words
// consumed.  One workgroup: all waves stage the bitmap window, wave 0 walks the mates; a mate whose scan leaves the
// window saves its state and the window moves to it.  *overflow = 1 when the stream words run out.
__global__ void __launch_bounds__(256) k_cx_chain(const uint64_t *bits, int64_t n64, const CrTpl *tpl, int32_t nf,
                                                  int64_t K, int64_t *mstart, int32_t *overflow) {
  __shared__ uint64_t win[CX_WIN];
  __shared__ int64_t sh[6];   // window base, k, cur, u, rem, flags (1: inside a mate's scan, 2: finished)
  const int t = threadIdx.x, lane = t & 63;
  if (t < 6) sh[t] = 0;
  lds_barrier();
  for (;;) {
    const int64_t base = sh[0];
    for (int i = t; i < CX_WIN; i += 256) win[i] = base + i < n64 ? bits[base + i] : 0ull;
    lds_barrier();
    if (t < 64) {
      int64_t k = sh[1], cur = sh[2], u = sh[3], rem = sh[4];
      bool mid = (sh[5] & 1) != 0, refill = false;
      int64_t lk0 = -64;
      int32_t lreg = 0;   // lane l: length of mate lk0 + l
      while (k < K) {
        if (!mid) {
          if (k >= lk0 + 64) {
            lk0 = k;
            const int64_t kk = k + lane;
            lreg = kk < K ? tpl[kk / nf].len[kk % nf] : 0;
          }
          const int32_t n = __shfl(lreg, (int)(k - lk0), 64);
          if (lane == 0) mstart[k] = cur;
          if (n == 0) {   // rand(0) and randint(0, 3, 0) draw nothing
            k++;
            continue;
          }
          u = cur + 4 * (int64_t)n;
          rem = n;
          mid = true;
        }
        const int64_t wi = u >> 6;
        if (wi >= n64) break;                                    // out of stream words
        if (wi + 64 > base + CX_WIN) {                           // past the window
          refill = true;
          break;
        }
        uint64_t v = win[wi - base + lane];
        if (lane == 0) v &= ~0ull << (u & 63);
        const int c = __popcll(v);
        int incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int o = __shfl_up(incl, d, 64);
          if (lane >= d) incl += o;
        }
        const int tot = __shfl(incl, 63, 64);
        if (tot < rem) {
          rem -= tot;
          u = (wi + 64) << 6;
          continue;
        }
        const int L = __builtin_ctzll(__ballot(incl >= rem));
        long long end = 0;
        if (lane == L) end = ((wi + L) << 6) + select_bit(v, (int)rem - (incl - c)) + 1;
        cur = __shfl(end, L, 64);
        k++;
        mid = false;
      }
      if (lane == 0) {
        sh[1] = k;
        sh[2] = cur;
        sh[3] = u;
        sh[4] = rem;
        if (k >= K) {
          mstart[K] = cur;
          sh[5] = 2;
        } else if (refill) {
          sh[0] = u >> 6;
          sh[5] = mid ? 1 : 0;
        } else {
          *overflow = 1;
          sh[5] = 2;
        }
      }
    }
    lds_barrier();
    if (sh[5] & 2) break;
  }
}

struct CxArgs {
  const uint32_t *w;        // the stream from the chain's word 0
  const int64_t *mstart;    // [T * nf + 1]
  int64_t nw;
  const double *cum, *phred;
  const uint16_t *guide;
  int32_t max_bp, n_bq;
};

template <bool EXACT>
__global__ void __launch_bounds__(256) k_cr_write(const uint8_t *b0, const uint8_t *b1, const CrTpl *tpl, int64_t T,
                                                  int32_t nf, const Off3 *off, char *out0, char *out1,
                                                  CorruptCfg cc, CxArgs xa) {
  extern __shared__ uint8_t cx_choice[];   // exact mode: per wave, the mate's randint(0, 3) draws
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
  if (EXACT) {
    uint8_t *ch = cx_choice + (threadIdx.x >> 6) * xa.max_bp;
    const int64_t s = xa.mstart[i];
    // randint(0, 3, L): the first L accepted words from s + 4L, compacted in stream order
    int64_t pos = s + 4 * (int64_t)L;
    for (int32_t got = 0; got < L; pos += 64) {
      const uint32_t w = pos + lane < xa.nw ? xa.w[pos + lane] : 3u;
      const bool acc = (w & 3u) != 3u;
      const uint64_t m = __ballot(acc);
      const int idx = got + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (acc && idx < L) ch[idx] = (uint8_t)(w & 3u);
      got += __popcll(m);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's choices are in LDS before any lane reads
    for (int32_t k = lane; k < L; k += 64) {
      const double u1 = mt_double(xa.w[s + 2 * k], xa.w[s + 2 * k + 1]);
      const double u2 = mt_double(xa.w[s + 2 * (int64_t)L + 2 * k], xa.w[s + 2 * (int64_t)L + 2 * k + 1]);
      const uint32_t bq = bq_search(xa.cum, xa.guide, xa.max_bp, xa.n_bq, f, k, u1);
      uint8_t b = sq[k];
      if (u2 < xa.phred[bq]) b = rot_base(b, ch[k]);
      ds[k] = (char)b;
      dq[k] = (char)(bq + 33);
    }
    return;
  }
  for (int32_t k = 3 * lane; k < L; k += 192) {   // base triples (one Philox draw each)
    const int cnt = L - k < 3 ? L - k : 3;
    uint8_t b[3], qq[3];
#pragma unroll
    for (int i = 0; i < 3; i++) b[i] = i < cnt ? sq[k + i] : (uint8_t)0;
    corrupt_triple_g(cc, t, f, k, cnt, b, qq);
#pragma unroll
    for (int i = 0; i < 3; i++)
      if (i < cnt) {
        ds[k + i] = (char)b[i];
        dq[k + i] = (char)qq[i];
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
  MH_TRY(ensure(ctx, ctx->s[13], sizeof(Off3) * (T + 1)));
  MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(Off3) * scan_partials_count(T + 1) + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int32_t *err = (int32_t *)((char *)ctx->d_small.p + 64);
  HIPCHK(ctx, hipMemsetAsync(err, 0, 8, st));
  CrTpl *tpl = (CrTpl *)B.tpl.p;
  stage_begin(ctx, "corrupt_measure");
  hipLaunchKernelGGL(k_cr_measure, dim3(grid_for(T, 256, INT32_MAX)), dim3(256), 0, st, d0, (const int64_t *)B.nl1.p,
                     d1, d1 ? (const int64_t *)B.nl2.p : nullptr, nf, T, ctx->corrupt_max_bp, tpl, err);
  HIPCHK(ctx, hipGetLastError());
  Off3 *off = (Off3 *)ctx->s[13].p;
  HIPCHK(ctx, device_scan<Off3>(st, T + 1, LoadCr{tpl, T}, StoreCr{off}, OpSum{}, Off3{0, 0, 0},
                                (Off3 *)ctx->scan_partials.p, (Off3 *)((char *)ctx->d_small.p + 128)));
  stage_end(ctx);
  int32_t herr = 0;
  Off3 tot;
  int64_t last0 = 0, last1 = 0;
  HIPCHK(ctx, hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(&tot, off + T, sizeof(Off3), hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(&last0, (const int64_t *)B.nl1.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  if (d1) HIPCHK(ctx, hipMemcpyAsync(&last1, (const int64_t *)B.nl2.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  if (herr & CE_LONG) return arg_fail(ctx, MH_E_ARG, "read longer than the BQ model (illumina.corrupt_single_read)");
  if (herr) return arg_fail(ctx, MH_E_ARG, "malformed FASTQ record");
  MH_TRY(ensure_keep(ctx, ctx->out1, ctx->used1 + tot.a + 64, ctx->used1));
  if (d1) MH_TRY(ensure_keep(ctx, ctx->out2, ctx->used2 + tot.b + 64, ctx->used2));
  const uint64_t key = 0x636f7272757074ull;   // fixed unit key of the standalone tool
  const CorruptCfg cc = corrupt_cfg(ctx, key, t_base);
  CxArgs xa{nullptr, nullptr, 0, cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq};
  char *o0 = (char *)ctx->out1.p + ctx->used1, *o1 = d1 ? (char *)ctx->out2.p + ctx->used2 : nullptr;
  const unsigned grid = grid_for(T * nf * 64, 256, INT32_MAX);
  if (ctx->cx_mode == 0) {
    stage_begin(ctx, "corrupt_write");
    hipLaunchKernelGGL(k_cr_write<false>, dim3(grid), dim3(256), 0, st, d0, d1, (const CrTpl *)tpl, T, nf,
                       (const Off3 *)off, o0, o1, cc, xa);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  } else {
    // the reference's single-worker stream: 4 words per base for the two uniforms, then one accepted word per base
    // (a word is rejected with probability 1/4); generous for the rejections, doubled if the chain runs out
    const int64_t K = T * nf, M = tot.m;
    int64_t need = 4 * M + (4 * M + 2) / 3 + 16 * (int64_t)std::sqrt((double)M + 1.0) + 4096;
    MH_TRY(ensure(ctx, ctx->cx_start, 8 * (size_t)(K + 1) + 64));
    int64_t *mstart = (int64_t *)ctx->cx_start.p;
    int32_t *ovf = err + 1;
    int64_t consumed = 0;
    for (;;) {
      int64_t lead = 0;
      stage_begin(ctx, "corrupt_exact_words");
      if (ctx->cx_mode == 1)
        MH_TRY(mt_stream_words(ctx, st, ctx->cx_seed, ctx->cx_pos, need, ctx->cx_words, ctx->cx_aux, &lead));
      else
        MH_TRY(mt_state_words(ctx, st, ctx->cx_key, ctx->cx_kpos, need, ctx->cx_words, ctx->cx_aux));
      stage_end(ctx);
      const uint32_t *w = (const uint32_t *)ctx->cx_words.p + lead;
      const int64_t n64 = (need + 63) / 64;
      MH_TRY(ensure(ctx, ctx->cx_bits, 8 * (size_t)n64 + 64));
      HIPCHK(ctx, hipMemsetAsync(ovf, 0, 4, st));
      stage_begin(ctx, "corrupt_exact_chain");
      hipLaunchKernelGGL(k_cx_bits, dim3(grid_for(n64 * 64, 256, INT32_MAX)), dim3(256), 0, st, w, need,
                         (uint64_t *)ctx->cx_bits.p, n64);
      hipLaunchKernelGGL(k_cx_chain, dim3(1), dim3(256), 0, st, (const uint64_t *)ctx->cx_bits.p, n64,
                         (const CrTpl *)tpl, nf, K, mstart, ovf);
      HIPCHK(ctx, hipGetLastError());
      stage_end(ctx);
      int32_t hovf = 0;
      HIPCHK(ctx, hipMemcpyAsync(&hovf, ovf, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipMemcpyAsync(&consumed, mstart + K, 8, hipMemcpyDeviceToHost, st));
      SYNCCHK(ctx, hipStreamSynchronize(st));
      if (hovf) {
        need *= 2;
        continue;
      }
      xa.w = w;
      xa.mstart = mstart;
      xa.nw = need;
      stage_begin(ctx, "corrupt_write");
      hipLaunchKernelGGL(k_cr_write<true>, dim3(grid), dim3(256), 4 * (size_t)ctx->corrupt_max_bp, st, d0, d1,
                         (const CrTpl *)tpl, T, nf, (const Off3 *)off, o0, o1, cc, xa);
      HIPCHK(ctx, hipGetLastError());
      stage_end(ctx);
      break;
    }
    if (ctx->cx_mode == 1) {
      ctx->cx_pos += consumed;
    } else {   // advance the explicit state by the words consumed (twists only)
      HostMT h;
      std::copy(ctx->cx_key, ctx->cx_key + 624, h.key);
      h.pos = ctx->cx_kpos;
      for (int64_t left = consumed; left > 0;) {
        if (h.pos == 624) {
          h.next();
          left--;
          continue;
        }
        const int64_t take = std::min<int64_t>(624 - h.pos, left);
        h.pos += (int)take;
        left -= take;
      }
      std::copy(h.key, h.key + 624, ctx->cx_key);
      ctx->cx_kpos = h.pos;
    }
  }
  SYNCCHK(ctx, hipStreamSynchronize(st));
  ctx->used1 += tot.a;
  if (d1) ctx->used2 += tot.b;
  *used0 = last0 + 1;
  *used1 = d1 ? last1 + 1 : 0;
  *templates = T;
  return MH_OK;
}

}  // namespace mh
