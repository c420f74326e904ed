// mh_bam.hip — the god-aligner's perfect-alignment BAM (reference mitty/benchmarking/god_aligner.py:19-183) on the
// device: SURVEY.md §8(a) A16 / §8(f) rank 1.
//
//   FASTQ bytes (host chunks, or the context's own FASTQ arenas)
//     -> newline positions           (SWAR '\n' count per 64-byte chunk, a look-back scan, positions stored)
//     -> k_bam_parse                 (thread per template: parse_qname of file 1's name (readgenerate.py:259-291),
//                                     the CIGAR, tid from the @SQ names, seq / qual spans; BAM record sizes)
//     -> scan of record sizes        (appends to the resident record store)
//     -> k_bam_write                 (32 lanes per record: core fields, name, CIGAR, 4-bit seq (reverse-complemented
//                                     for strand 1 with the ATCGN-only table), qual - 33 (reversed for strand 1))
//   finish:
//     -> stable radix sort of (tid, pos + 1, is_reverse)  (samtools sort's coordinate order, input order on ties)
//     -> k_bam_gather                (records into sorted order + per-record index info)
//     -> host: BGZF deflate on a thread pool, BAI from the virtual offsets (mh_bgzf.cpp)
//
// Record attributes follow write_perfect_reads (god_aligner.py:153-183): pos = qname pos - 1, CIGAR from the qname
// ('>p:nI' -> 'nI'), MAPQ 60, flag = reverse | paired / proper / read1 / read2 for two files, mate = the other
// read's tid / pos, TLEN 0, no tags, qname = file 1's read name.  bin = reg2bin(pos, bam_endpos) as htslib sets it.
#include <rocprim/device/device_radix_sort.hpp>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "mh_bgzf.h"
#include "mh_internal.h"
#include "mh_scan.h"
#include "mh_sort.h"

namespace mh {
namespace {

constexpr int BAM_MAX_READS = 2;

struct BamRead {
  int64_t seq_off, qual_off;   // into the file's buffer
  int32_t tid, pos, end;       // end = bam_endpos (pos + reference span, at least 1)
  int32_t l_seq, cig_off, cig_len;   // cig_* relative to the qname start
  int32_t size;                // BAM record bytes including block_size
  uint16_t flag, bin, n_cig;
  uint16_t pad;
};

struct BamTpl {
  int64_t qn_off;    // qname start in file 1 (after '@')
  int32_t qn_len;
  int32_t n_reads;
  BamRead r[BAM_MAX_READS];
};

struct RInfo {       // per record, for the BAI
  int32_t tid, beg, end;
  uint32_t bin;
};

// ---- newline index ----------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t nl_mask4(uint32_t v) {   // 0x80 in every byte equal to '\n'
  uint32_t x = v ^ 0x0a0a0a0au;
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}

// element t = the 64 bytes [64 t, 64 t + 64) of the buffer
constexpr int NL_CH = 64;
struct LoadNL {
  const uint8_t *b;
  int64_t len;
  __device__ int64_t operator()(int64_t t) const {
    const int64_t o = t * NL_CH;
    if (o >= len) return 0;
    if (o + NL_CH <= len) {
      int64_t c = 0;
#pragma unroll
      for (int q = 0; q < NL_CH / 16; q++) {
        const uint4 v = *(const uint4 *)(b + o + 16 * q);
        c += __popc(nl_mask4(v.x)) + __popc(nl_mask4(v.y)) + __popc(nl_mask4(v.z)) + __popc(nl_mask4(v.w));
      }
      return c;
    }
    int64_t c = 0;
    for (int64_t i = o; i < len; i++) c += b[i] == '\n';
    return c;
  }
};

struct StoreNL {
  const uint8_t *b;
  int64_t len;
  int64_t *nl;
  __device__ void operator()(int64_t t, int64_t, int64_t excl) const {
    const int64_t o = t * NL_CH;
    if (o >= len) return;
    if (o + NL_CH <= len) {
#pragma unroll
      for (int q = 0; q < NL_CH / 16; q++) {
        const uint4 v = *(const uint4 *)(b + o + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          uint32_t m = nl_mask4(w[k]);
          while (m) {
            const int bit = __ffs(m) - 1;
            nl[excl++] = o + 16 * q + 4 * k + (bit >> 3);
            m &= m - 1;
          }
        }
      }
      return;
    }
    for (int64_t i = o; i < len; i++)
      if (b[i] == '\n') nl[excl++] = i;
  }
};

// ---- parsing ----------------------------------------------------------------------------------------------------
__device__ __forceinline__ int cigar_code(uint8_t c) {   // BAM_CIGAR_STR "MIDNSHP=X"
  switch (c) {
    case 'M': return 0; case 'I': return 1; case 'D': return 2; case 'N': return 3; case 'S': return 4;
    case 'H': return 5; case 'P': return 6; case '=': return 7; case 'X': return 8;
    default: return -1;
  }
}
__device__ __forceinline__ bool cigar_consumes_ref(int op) { return op == 0 || op == 2 || op == 3 || op == 7 || op == 8; }

// hts_reg2bin(beg, end, 14, 5)
__device__ __forceinline__ uint32_t reg2bin(int64_t beg, int64_t end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (uint32_t)(beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (uint32_t)(beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (uint32_t)(beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (uint32_t)(beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (uint32_t)(beg >> 26);
  return 0;
}

// int() of a decimal field; false if empty or not all digits (optional leading '-')
__device__ __forceinline__ bool parse_int(const uint8_t *s, int32_t n, int64_t &v) {
  if (n <= 0) return false;
  int i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') { neg = s[0] == '-'; i = 1; }
  if (i >= n) return false;
  int64_t x = 0;
  for (; i < n; i++) {
    uint32_t d = (uint32_t)s[i] - '0';
    if (d > 9) return false;
    x = x * 10 + d;
  }
  v = neg ? -x : x;
  return true;
}

enum { BE_QNAME = 1, BE_CHROM = 2, BE_FIELDS = 4, BE_CIGAR = 8, BE_QNAME_LEN = 16, BE_SEQ = 32 };

struct ParseArgs {
  const uint8_t *b[BAM_MAX_READS];
  const int64_t *nl[BAM_MAX_READS];
  int32_t n_files;
  const char *names;          // @SQ names, concatenated
  const int32_t *name_off;    // [n_refs + 1]
  int32_t n_refs;
  int64_t len0;               // bytes of file 1's buffer
};

__device__ __forceinline__ int64_t line_start(const int64_t *nl, int64_t line) { return line == 0 ? 0 : nl[line - 1] + 1; }

// The name lines of a workgroup's 256 templates are first staged in LDS (a wave copies its 64 lines with one 16-byte
// load per lane per line, all in flight together), so the per-template parse below reads LDS, not a chain of
// dependent global byte loads.  A line longer than its LDS row is read from memory.
constexpr int BP_ROW = 192;

__global__ void __launch_bounds__(256) k_bam_parse(ParseArgs a, int64_t T, BamTpl *tpl, int32_t *err) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[256 * BP_ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t tw = (int64_t)blockIdx.x * 256 + 64 * wave;   // the wave's first template
  {
    const int64_t tl = tw + lane;
    const int64_t ls0 = tl < T ? line_start(a.nl[0], 4 * tl) : 0, le0 = tl < T ? a.nl[0][4 * tl] : 0;
#pragma unroll 8
    for (int j = 0; j < 64; j++) {
      const int64_t s0 = __shfl(ls0, j, 64), e0 = __shfl(le0, j, 64);
      const int64_t c0 = s0 & ~(int64_t)15;
      const int nch = (int)((e0 - c0 + 15) >> 4);
      if (tw + j < T && nch * 16 <= BP_ROW && c0 + 16 * nch <= a.len0 && lane < nch)
        *(uint4 *)(rows + (64 * wave + j) * BP_ROW + 16 * lane) = *(const uint4 *)(a.b[0] + c0 + 16 * lane);
    }
  }
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  BamTpl o;
  const int64_t s0 = line_start(a.nl[0], 4 * t);
  const int64_t e0 = a.nl[0][4 * t];
  const int64_t c0 = s0 & ~(int64_t)15;
  const int nch = (int)((e0 - c0 + 15) >> 4);
  const bool staged = nch * 16 <= BP_ROW && c0 + 16 * nch <= a.len0;
  // lp: the line's first byte (LDS row or the buffer itself); lp[x - s0] = file byte x
  const uint8_t *lp = staged ? rows + threadIdx.x * BP_ROW + (s0 - c0) : a.b[0] + s0;
  int32_t e = 0;
  if (e0 <= s0 || lp[0] != '@') e |= BE_QNAME;
  int64_t q0 = s0 + 1, q1 = q0;
  while (q1 < e0 && lp[q1 - s0] != ' ' && lp[q1 - s0] != '\t') q1++;   // FastxFile name: up to the first whitespace
  o.qn_off = q0;
  o.qn_len = (int32_t)(q1 - q0);
  if (o.qn_len > 254) e |= BE_QNAME_LEN;
  o.n_reads = a.n_files;
  // split on '|': rid, chrom, cpy, then (strand, pos, rlen, cigar, v_list) per read
  int32_t fs[3 + 5 * BAM_MAX_READS], fe[3 + 5 * BAM_MAX_READS];
  int nf = 0;
  {
    int64_t st = q0;
    for (int64_t i = q0; i <= q1 && nf < 3 + 5 * BAM_MAX_READS; i++) {
      if (i == q1 || lp[i - s0] == '|') {
        fs[nf] = (int32_t)(st - q0);
        fe[nf] = (int32_t)(i - q0);
        nf++;
        st = i + 1;
      }
    }
  }
  if (nf < 3 + 5 * a.n_files - 1) e |= BE_FIELDS;   // the last read's v_list may be the (empty) tail
  const uint8_t *qn = lp + (q0 - s0);
  // chrom -> tid
  int32_t tid = -1;
  if (!(e & BE_FIELDS)) {
    const int32_t cl = fe[1] - fs[1];
    for (int32_t r = 0; r < a.n_refs && tid < 0; r++) {
      const int32_t no = a.name_off[r], nl = a.name_off[r + 1] - no;
      if (nl != cl) continue;
      bool eq = true;
      for (int32_t k = 0; k < cl && eq; k++) eq = a.names[no + k] == (char)qn[fs[1] + k];
      if (eq) tid = r;
    }
    if (tid < 0) e |= BE_CHROM;
  }
  for (int s = 0; s < a.n_files && !e; s++) {
    BamRead &r = o.r[s];
    const int f = 3 + 5 * s;
    int64_t strand, pos;
    if (!parse_int(qn + fs[f], fe[f] - fs[f], strand) || !parse_int(qn + fs[f + 1], fe[f + 1] - fs[f + 1], pos)) {
      e |= BE_FIELDS;
      break;
    }
    int32_t cs = fs[f + 3], ce = fe[f + 3];
    if (ce > cs && qn[cs] == '>') {   // '>p:nI' -> 'nI' (parse_qname: split(':')[-1])
      int32_t k = ce;
      while (k > cs && qn[k - 1] != ':') k--;
      cs = k;
    }
    int32_t n_cig = 0;
    int64_t ref_span = 0, num = 0;
    bool have = false;
    for (int32_t k = cs; k < ce; k++) {
      uint32_t d = (uint32_t)qn[k] - '0';
      if (d <= 9) { num = num * 10 + d; have = true; continue; }
      int op = cigar_code(qn[k]);
      if (op < 0 || !have) { e |= BE_CIGAR; break; }
      if (cigar_consumes_ref(op)) ref_span += num;
      n_cig++;
      num = 0;
      have = false;
    }
    if (have) e |= BE_CIGAR;
    const int64_t ls = line_start(a.nl[s], 4 * t + 1), le = a.nl[s][4 * t + 1];
    const int64_t qs = line_start(a.nl[s], 4 * t + 3), qe = a.nl[s][4 * t + 3];
    r.seq_off = ls;
    r.qual_off = qs;
    r.l_seq = (int32_t)(le - ls);
    if (qe - qs != le - ls) e |= BE_SEQ;
    r.tid = tid;
    r.pos = (int32_t)(pos - 1);
    r.end = (int32_t)(r.pos + (ref_span > 0 ? ref_span : 1));
    r.bin = (uint16_t)reg2bin(r.pos, r.end);
    r.cig_off = cs;
    r.cig_len = ce - cs;
    r.n_cig = (uint16_t)n_cig;
    r.flag = strand ? 0x10 : 0;
    if (a.n_files == 2) r.flag |= 0x1 | 0x2 | (s == 0 ? 0x40 : 0x80);
    r.size = 4 + 32 + (o.qn_len + 1) + 4 * n_cig + (r.l_seq + 1) / 2 + r.l_seq;
  }
  tpl[t] = o;
  if (e) atomicOr(err, e);
}

struct LoadSize {
  const BamTpl *tpl;
  int32_t nr;
  int64_t n;   // records
  __device__ int64_t operator()(int64_t i) const {   // nr is 1 or 2: shifts, not 64-bit divisions
    return i < n ? (nr == 2 ? tpl[i >> 1].r[i & 1] : tpl[i].r[0]).size : 0;
  }
};
struct StoreOff64 {
  int64_t *off;
  int64_t base;
  __device__ void operator()(int64_t i, int64_t, int64_t excl) const { off[i] = base + excl; }
};

__device__ __forceinline__ uint8_t nt16(uint8_t c) {   // htslib seq_nt16_table: letters a..z (either case) from
  // two nibble tables (selects, no branches or table loads), '=' 0, anything else 15
  const uint32_t x = (uint32_t)(c | 0x20) - 'a';
  const uint64_t lo = 0xfff3fcffb4ffd2e1ull, hi = 0xfaf978865full;
  const uint32_t v = (uint32_t)((x < 16 ? lo >> ((4 * x) & 63) : hi >> ((4 * (x - 16)) & 63)) & 15u);
  return (uint8_t)(x < 26 ? v : c == '=' ? 0u : 15u);
}
__device__ __forceinline__ uint8_t comp_atcgn(uint8_t c) {   // str.maketrans('ATCGN', 'TAGCN')
  return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
}

// One wave per record.  Records are byte-packed (BAM has no padding), so stores are bytewise; every input byte the
// wave needs is loaded by the lanes together (restrict pointers let the loads of an unrolled loop issue ahead of the
// stores), and the CIGAR text is walked from registers (shuffles), not from memory.
// slot (direct sorted write, bam_add_output into an empty store): record i goes to sorted place slot[i] — at
// off[slot[i]], its BAI info at info[slot[i]], no sort key (records are read in input order, so the FASTQ reads
// stream); otherwise record i at off[i] with its key.
// G lanes per record (64: a wave; 32: two records per wave side by side, so twice the records in flight per resident
// wave — the kernel is bound by each record's chain of dependent loads, not by bandwidth)
template <int G>
__global__ void __launch_bounds__(256) k_bam_write(ParseArgs a, const BamTpl *tpl, int64_t n_rec, int32_t nr,
                                                   const uint32_t *slot, const int64_t *off, uint8_t *out,
                                                   uint64_t *key, uint32_t *val, RInfo *info, int64_t rec_base,
                                                   int64_t out_cap, int32_t *bad) {
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1), gb = lane & ~(G - 1);   // lane within the record's group, the group's first lane
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  if (i >= n_rec) return;   // (a whole group)
  const int64_t w = slot ? (int64_t)slot[i] : i;
  const int64_t t = nr == 2 ? i >> 1 : i;   // nr is 1 or 2
  const int s = nr == 2 ? (int)(i & 1) : 0;
  const BamTpl &T = tpl[t];
  const BamRead &r = T.r[s];
  const BamRead &m = T.r[nr == 2 ? 1 - s : s];
  // bounds: the record's place (a sorted slot from the sort's values) and its bytes inside the store; a violation is
  // reported (mh_bam_*: MH_E_STATE), never written
  if (w < 0 || w >= n_rec || off[w] < 0 || off[w] + r.size > out_cap) {
    if (gl == 0) atomicOr(bad, 1);
    return;
  }
  uint8_t *__restrict__ d = out + off[w];
  const uint8_t *__restrict__ qn = a.b[0] + T.qn_off;
  const int32_t lq = T.qn_len + 1;
  const int32_t hdr = 36;
  if (gl < 9) {
    int32_t x;
    switch (gl) {
      case 0: x = r.size - 4; break;
      case 1: x = r.tid; break;
      case 2: x = r.pos; break;
      case 3: x = (int32_t)((uint32_t)r.bin << 16 | 60u << 8 | (uint32_t)lq); break;
      case 4: x = (int32_t)((uint32_t)r.flag << 16 | r.n_cig); break;
      case 5: x = r.l_seq; break;
      case 6: x = nr == 2 ? m.tid : -1; break;
      case 7: x = nr == 2 ? m.pos : -1; break;
      default: x = 0; break;   // TLEN
    }
    uint8_t *p = d + 4 * gl;
    p[0] = (uint8_t)x; p[1] = (uint8_t)(x >> 8); p[2] = (uint8_t)(x >> 16); p[3] = (uint8_t)(x >> 24);
  }
  const uint8_t *__restrict__ sq = a.b[s] + r.seq_off, *__restrict__ ql = a.b[s] + r.qual_off;
  const int32_t L = r.l_seq;
  const bool rev = r.flag & 0x10;
  // every load first: qname, CIGAR text, bases, qualities (4 x G bytes each per pass)
  uint8_t qb[4], cb, sb0[4], sb1[4], qv[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int32_t k = gl + G * u;
    qb[u] = k < T.qn_len ? qn[k] : 0;
  }
  cb = gl < r.cig_len ? qn[r.cig_off + gl] : 0;
  uint8_t *dc = d + hdr + lq;
  uint8_t *ds = dc + 4 * r.n_cig;
  uint8_t *dq = ds + (L + 1) / 2;
  // loads in ascending address order across the lanes for both strands (a strand-1 read is reversed by where each
  // lane stores, not by which byte it loads: descending lane addresses do not coalesce)
  const int32_t J = (L + 1) / 2;   // sequence bytes
  for (int32_t k0 = 0; k0 < L; k0 += 4 * G) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int32_t y = k0 + gl + G * u;               // quality byte loaded
      const int32_t jx = k0 / 2 + gl + G * u;          // sequence byte, in load order
      const int32_t j = rev ? J - 1 - jx : jx;         // ... its output index: bases 2j, 2j + 1
      const bool jv = jx < J && jx < k0 / 2 + 2 * G;
      qv[u] = y < L ? ql[y] : 0;
      sb0[u] = jv ? sq[rev ? L - 1 - 2 * j : 2 * j] : 0;
      sb1[u] = jv && 2 * j + 1 < L ? sq[rev ? L - 2 - 2 * j : 2 * j + 1] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int32_t y = k0 + gl + G * u, jx = k0 / 2 + gl + G * u;
      if (y < L) dq[rev ? L - 1 - y : y] = (uint8_t)(qv[u] - 33);
      if (jx < J && jx < k0 / 2 + 2 * G) {
        const int32_t j = rev ? J - 1 - jx : jx;
        const uint8_t c0 = rev ? comp_atcgn(sb0[u]) : sb0[u];
        const uint8_t lo = 2 * j + 1 < L ? nt16(rev ? comp_atcgn(sb1[u]) : sb1[u]) : 0;
        ds[j] = (uint8_t)(nt16(c0) << 4 | lo);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int32_t k = gl + G * u;
    if (k < lq) d[hdr + k] = qb[u];
  }
  for (int32_t k = gl + 4 * G; k < lq; k += G) d[hdr + k] = k < T.qn_len ? qn[k] : 0;   // longer names
  // CIGAR: lane k of the group holds text byte k; every op lane packs its own op from the digits since the previous
  // op (ballot + shuffles, no serial walk).  A text longer than G bytes is walked serially from memory.
  if (r.cig_len <= G) {
    const bool is_op = gl < r.cig_len && (uint32_t)cb - '0' > 9;
    const uint64_t ops = (__ballot(is_op) >> gb) & (G == 64 ? ~0ull : 0xffffffffull);
    const uint64_t below = gl ? ops & ((~0ull) >> (64 - gl)) : 0ull;
    const int prev = below ? 63 - __builtin_clzll(below) : -1;   // the previous op's lane in the group
    uint32_t num = 0;
    const int nd = is_op ? gl - prev - 1 : 0;
    int ndmax = nd;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) ndmax = max(ndmax, __shfl_xor(ndmax, o, 64));
    for (int q = 0; q < ndmax; q++) {   // the digits prev + 1 .. gl - 1, most significant first
      const int src = prev + 1 + q;
      const uint32_t dgt = (uint32_t)__shfl((int)cb, gb + (src < G ? (src > 0 ? src : 0) : G - 1), 64) - '0';
      if (q < nd) num = num * 10 + dgt;
    }
    if (is_op) {
      const int j = __popcll(below);
      const uint32_t x = num << 4 | (uint32_t)cigar_code(cb);
      dc[4 * j] = (uint8_t)x; dc[4 * j + 1] = (uint8_t)(x >> 8); dc[4 * j + 2] = (uint8_t)(x >> 16);
      dc[4 * j + 3] = (uint8_t)(x >> 24);
    }
  } else {
    uint32_t num = 0;
    int j = 0;
    for (int32_t k = 0; k < r.cig_len; k++) {
      const uint8_t c = qn[r.cig_off + k];
      const uint32_t dd = (uint32_t)c - '0';
      if (dd <= 9) { num = num * 10 + dd; continue; }
      if (gl == 0) {
        const uint32_t x = num << 4 | (uint32_t)cigar_code(c);
        dc[4 * j] = (uint8_t)x; dc[4 * j + 1] = (uint8_t)(x >> 8); dc[4 * j + 2] = (uint8_t)(x >> 16);
        dc[4 * j + 3] = (uint8_t)(x >> 24);
      }
      j++;
      num = 0;
    }
  }
  if (gl == 0) {
    if (key) {
      key[i] = (uint64_t)(uint32_t)r.tid << 33 | (uint64_t)(uint32_t)(r.pos + 1) << 1 | (rev ? 1u : 0u);
      val[i] = (uint32_t)(rec_base + i);
    }
    info[w] = RInfo{r.tid, r.pos, r.end, r.bin};
  }
}
constexpr int BW_G = 32;   // lanes per record (16: the same time)

// record -> its sorted place
__global__ void k_bam_slots(const uint32_t *val2, int64_t n, uint32_t *slot) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) slot[val2[k]] = (uint32_t)k;
}

// samtools sort's key of every record (the direct sorted write sorts before it writes)
__global__ void k_bam_keys(const BamTpl *tpl, int64_t n_rec, int32_t nr, uint64_t *key, uint32_t *val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rec) return;
  const BamRead &r = tpl[nr == 2 ? i >> 1 : i].r[nr == 2 ? (int)(i & 1) : 0];
  key[i] = (uint64_t)(uint32_t)r.tid << 33 | (uint64_t)(uint32_t)(r.pos + 1) << 1 | ((r.flag & 0x10) ? 1u : 0u);
  val[i] = (uint32_t)i;
}

__global__ void k_gather_key(const uint64_t *key, const uint32_t *val, int64_t n, uint64_t *out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = key[val[k]];
}

// sorted position k <- record val[k]
struct LoadSortedSize {
  const uint32_t *val;
  const int64_t *roff;   // [n + 1] unsorted offsets (roff[n] = total)
  int64_t n;
  __device__ int64_t operator()(int64_t k) const {
    if (k >= n) return 0;
    const uint32_t r = val[k];
    return roff[r + 1] - roff[r];
  }
};

// 32 lanes per record, two records per wave (as k_bam_write: each record is a short chain of dependent loads)
__global__ void __launch_bounds__(256) k_bam_gather(const uint8_t *src, const int64_t *roff, const uint32_t *val,
                                                    const int64_t *soff, int64_t n, uint8_t *dst, const RInfo *info,
                                                    RInfo *sinfo, int64_t src_bytes, int64_t dst_cap, int32_t *bad) {
  constexpr int G = 32;
  const int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int gl = threadIdx.x & (G - 1);
  if (k >= n) return;   // (a whole group)
  const uint32_t r = val[k];
  // bounds: r must be a record of the store (the sort's values are a permutation of [0, n)), its bytes inside the
  // input-order store and its sorted place inside the output; a violation is reported, never followed
  if (r >= (uint64_t)n) {
    if (gl == 0) atomicOr(bad, 2);
    return;
  }
  const int64_t a = roff[r], len = roff[r + 1] - a;
  if (a < 0 || len < 0 || a + len > src_bytes || soff[k] < 0 || soff[k] + len > dst_cap) {
    if (gl == 0) atomicOr(bad, 4);
    return;
  }
  const uint8_t *__restrict__ s = src + a;
  uint8_t *__restrict__ d = dst + soff[k];
  for (int64_t j0 = 0; j0 < len; j0 += 8 * G) {   // eight loads in flight per lane, then the stores
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t j = j0 + gl + G * u;
      v[u] = j < len ? s[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t j = j0 + gl + G * u;
      if (j < len) d[j] = v[u];
    }
  }
  if (gl == 0) sinfo[k] = info[r];
}

// a spilled store: only the BAI info is gathered in sorted order on the device (the bytes are assembled on the host)
__global__ void k_bam_sinfo(const uint32_t *val, int64_t n, const RInfo *info, RInfo *sinfo, int32_t *bad) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t r = val[k];
  if (r >= (uint64_t)n) {
    atomicOr(bad, 2);
    return;
  }
  sinfo[k] = info[r];
}

}  // namespace

// the record kernels' bounds flag (1: k_bam_write place / bytes, 2: a sort value outside [0, n), 4: k_bam_gather bytes)
static int32_t bam_check_bounds(mh_ctx *ctx, const int32_t *bad, const char *who) {
  int64_t *hs = pinned_small(ctx);
  if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  HIPCHK(ctx, hipMemcpyAsync(hs + 26, bad, 4, hipMemcpyDeviceToHost, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  const int32_t f = (int32_t)(hs[26] & 0xffffffff);
  if (f) return arg_fail(ctx, MH_E_STATE, std::string("BAM store: ") + who + " index or bytes out of bounds (flag " +
                                            std::to_string(f) + ", internal)");
  return MH_OK;
}

int32_t bam_set_refs(mh_ctx *ctx, int32_t n_refs, const char *names, const int64_t *lengths) {
  BamStore &B = ctx->bam;
  B.ref_names.clear();
  B.ref_len.assign(lengths, lengths + n_refs);
  std::vector<int32_t> off(1, 0);
  std::string cat;
  const char *p = names;
  for (int32_t i = 0; i < n_refs; i++) {
    std::string nm(p);
    p += nm.size() + 1;
    B.ref_names.push_back(nm);
    cat += nm;
    off.push_back((int32_t)cat.size());
  }
  MH_TRY(ensure(ctx, B.names, cat.size() + 16));
  MH_TRY(ensure(ctx, B.name_off, sizeof(int32_t) * off.size()));
  if (!cat.empty()) HIPCHK(ctx, hipMemcpyAsync(B.names.p, cat.data(), cat.size(), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(B.name_off.p, off.data(), sizeof(int32_t) * off.size(), hipMemcpyHostToDevice,
                             ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  B.n_rec = 0;
  B.bytes = 0;
  B.n_files = 0;
  B.sorted = false;
  B.direct = false;
  B.use_tie = false;
  bam_free_spill(B);
  B.refs_set = true;
  return MH_OK;
}

// Newline index of a device buffer into `nl` (grown as needed); returns the count.
int32_t newline_index(mh_ctx *ctx, const uint8_t *b, int64_t len, DevBuf &nl, int64_t *count) {
  hipStream_t st = ctx->stream;
  const int64_t chunks = (len + NL_CH - 1) / NL_CH;
  *count = 0;
  if (len == 0) return MH_OK;
  MH_TRY(ensure(ctx, ctx->scan_partials, std::max<size_t>(sizeof(int64_t) * scan_partials_count(chunks) + 64,
                                                          scan_lb_scratch_bytes<int64_t>(chunks))));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int64_t *tot = (int64_t *)ctx->d_small.p;
  HIPCHK(ctx, device_reduce<int64_t>(st, chunks, LoadNL{b, len}, OpSum{}, (int64_t)0,
                                     (int64_t *)ctx->scan_partials.p, tot));
  int64_t n = 0;
  HIPCHK(ctx, hipMemcpyAsync(&n, tot, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  MH_TRY(ensure(ctx, nl, sizeof(int64_t) * (n + 1)));
  // single pass (decoupled look-back): each element's bytes are re-read by the thread that counted them
  HIPCHK(ctx, device_scan_sum<int64_t>(st, chunks, LoadNL{b, len}, StoreNL{b, len, (int64_t *)nl.p},
                                       ctx->scan_partials.p, tot + 1));
  *count = n;
  return MH_OK;
}

int32_t bam_add(mh_ctx *ctx, const uint8_t *d1, int64_t len1, const uint8_t *d2, int64_t len2, int64_t max_templates,
                int64_t *used1, int64_t *used2, int64_t *templates, bool sorted_direct) {
  BamStore &B = ctx->bam;
  if (B.direct) MH_TRY(bam_undirect(ctx));   // more records after a direct sorted write: back to input order
  hipStream_t st = ctx->stream;
  *used1 = *used2 = *templates = 0;
  if (!B.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  const int32_t nf = d2 ? 2 : 1;
  if (B.n_files && B.n_files != nf) return arg_fail(ctx, MH_E_ARG, "single-end and paired input mixed in one BAM");
  int64_t nnl1 = 0, nnl2 = 0;
  stage_begin(ctx, "bam_index");
  MH_TRY(newline_index(ctx, d1, len1, B.nl1, &nnl1));
  if (d2) MH_TRY(newline_index(ctx, d2, len2, B.nl2, &nnl2));
  stage_end(ctx);
  int64_t T = nnl1 / 4;
  if (d2 && nnl2 / 4 < T) T = nnl2 / 4;
  if (max_templates >= 0 && T > max_templates) T = max_templates;
  if (T == 0) return MH_OK;
  B.n_files = nf;

  MH_TRY(ensure(ctx, B.tpl, sizeof(BamTpl) * T));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int32_t *err = (int32_t *)((char *)ctx->d_small.p + 64);
  int32_t *bad = err + 1;   // the record kernels' bounds flag
  HIPCHK(ctx, hipMemsetAsync(err, 0, 8, st));
  ParseArgs a{{d1, d2}, {(const int64_t *)B.nl1.p, d2 ? (const int64_t *)B.nl2.p : nullptr}, nf,
              (const char *)B.names.p, (const int32_t *)B.name_off.p, (int32_t)B.ref_names.size(), len1};
  stage_begin(ctx, "bam_parse");
  hipLaunchKernelGGL(k_bam_parse, dim3(grid_for(T, 256, INT32_MAX)), dim3(256), 0, st, a, T, (BamTpl *)B.tpl.p, err);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  int32_t herr = 0;
  HIPCHK(ctx, hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  if (herr) {
    std::string m = "god-aligner input:";
    if (herr & BE_QNAME) m += " malformed FASTQ record;";
    if (herr & BE_QNAME_LEN) m += " read name longer than 254 characters (BAM limit);";
    if (herr & BE_CHROM) m += " qname chrom not among the @SQ names (.ann);";
    if (herr & BE_FIELDS) m += " qname does not parse (readgenerate.parse_qname);";
    if (herr & BE_CIGAR) m += " invalid CIGAR in qname;";
    if (herr & BE_SEQ) m += " quality and sequence mismatch (sequence and quality lengths differ);";
    return arg_fail(ctx, MH_E_ARG, m);
  }
  // record offsets (appended to the store)
  const int64_t n_rec = T * nf;
  MH_TRY(ensure_keep(ctx, B.roff, sizeof(int64_t) * (B.n_rec + n_rec + 1), sizeof(int64_t) * (B.n_rec + 1)));
  MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(int64_t) * scan_partials_count(n_rec + 1) + 64));
  int64_t *roff = (int64_t *)B.roff.p + B.n_rec;
  int64_t *tot = (int64_t *)ctx->d_small.p;
  HIPCHK(ctx, device_scan<int64_t>(st, n_rec + 1, LoadSize{(const BamTpl *)B.tpl.p, nf, n_rec},
                                   StoreOff64{roff, B.bytes}, OpSum{}, (int64_t)0, (int64_t *)ctx->scan_partials.p,
                                   tot));
  int64_t add_bytes = 0;
  HIPCHK(ctx, hipMemcpyAsync(&add_bytes, tot, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  if (sorted_direct && B.n_rec == 0 && n_rec < (int64_t)UINT32_MAX && (B.cap <= 0 || add_bytes <= B.cap)) {
    // the whole input is here (the context's own arenas) and the store is empty: sort first, then every record is
    // written once, straight to its coordinate-sorted place (no input-order copy, no gather)
    MH_TRY(ensure(ctx, B.key, sizeof(uint64_t) * n_rec));
    MH_TRY(ensure(ctx, B.val, sizeof(uint32_t) * n_rec));
    hipLaunchKernelGGL(k_bam_keys, dim3(grid_for(n_rec, 256, INT32_MAX)), dim3(256), 0, st, (const BamTpl *)B.tpl.p,
                       n_rec, nf, (uint64_t *)B.key.p, (uint32_t *)B.val.p);
    HIPCHK(ctx, hipGetLastError());
    B.n_rec = n_rec;
    B.bytes = add_bytes;
    B.sorted = false;
    MH_TRY(bam_sort(ctx, &a));   // sorted keys, order and offsets; the records written by k_bam_write
    B.direct = true;
    int64_t last1 = 0, last2 = 0;
    HIPCHK(ctx, hipMemcpyAsync(&last1, (const int64_t *)B.nl1.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
    if (d2) HIPCHK(ctx, hipMemcpyAsync(&last2, (const int64_t *)B.nl2.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    *used1 = last1 + 1;
    *used2 = d2 ? last2 + 1 : 0;
    *templates = T;
    return MH_OK;
  }
  // bounded HBM: the resident records go to the host first when these would pass the capacity (or do not fit)
  if (B.cap > 0 && B.bytes > B.spilled && B.bytes - B.spilled + add_bytes > B.cap) MH_TRY(bam_spill(ctx));
  if (ensure_keep(ctx, B.recs, B.bytes - B.spilled + add_bytes + 64, B.bytes - B.spilled) != MH_OK) {
    if (B.bytes == B.spilled) return MH_E_OOM;   // (nothing to spill: the error stands)
    ctx->err.clear();
    MH_TRY(bam_spill(ctx));
    MH_TRY(ensure_keep(ctx, B.recs, add_bytes + 64, 0));
  }
  MH_TRY(ensure_keep(ctx, B.key, sizeof(uint64_t) * (B.n_rec + n_rec), sizeof(uint64_t) * B.n_rec));
  MH_TRY(ensure_keep(ctx, B.val, sizeof(uint32_t) * (B.n_rec + n_rec), sizeof(uint32_t) * B.n_rec));
  MH_TRY(ensure_keep(ctx, B.info, sizeof(RInfo) * (B.n_rec + n_rec), sizeof(RInfo) * B.n_rec));
  stage_begin(ctx, "bam_write");
  hipLaunchKernelGGL(k_bam_write<BW_G>, dim3(grid_for(n_rec * BW_G, 256, INT32_MAX)), dim3(256), 0, st, a,
                     (const BamTpl *)B.tpl.p, n_rec, nf, (const uint32_t *)nullptr, (const int64_t *)roff,
                     (uint8_t *)B.recs.p - B.spilled,   // (offsets are the store's; recs holds [spilled, bytes))
                     (uint64_t *)B.key.p + B.n_rec, (uint32_t *)B.val.p + B.n_rec, (RInfo *)B.info.p + B.n_rec,
                     B.n_rec, B.bytes + add_bytes, bad);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  MH_TRY(bam_check_bounds(ctx, bad, "k_bam_write"));
  B.n_rec += n_rec;
  B.bytes += add_bytes;
  B.sorted = false;
  int64_t last1 = 0, last2 = 0;
  HIPCHK(ctx, hipMemcpyAsync(&last1, (const int64_t *)B.nl1.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  if (d2) HIPCHK(ctx, hipMemcpyAsync(&last2, (const int64_t *)B.nl2.p + 4 * T - 1, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  *used1 = last1 + 1;
  *used2 = d2 ? last2 + 1 : 0;
  *templates = T;
  return MH_OK;
}

// pa: the direct sorted write's parse (records not written yet: k_bam_write places them in sorted order);
// null: the records are in recs (input order) and are gathered
int32_t bam_sort(mh_ctx *ctx, const void *pa) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  const int64_t n = B.n_rec;
  if (n == 0 || B.sorted) return MH_OK;
  if (n >= (int64_t)UINT32_MAX) return arg_fail(ctx, MH_E_CAPACITY, "more than 2^32 records in one BAM");
  int tid_bits = 1;
  while ((1ull << tid_bits) < (uint64_t)B.ref_names.size() + 1) tid_bits++;
  const unsigned end_bit = 33 + tid_bits;
  MH_TRY(ensure(ctx, B.key2, sizeof(uint64_t) * n));
  MH_TRY(ensure(ctx, B.val2, sizeof(uint32_t) * n));
  size_t tmp = 0;
  stage_begin(ctx, "bam_sort");
  const uint64_t *kin = (const uint64_t *)B.key.p;
  const uint32_t *vin = (const uint32_t *)B.val.p;
  if (B.use_tie) {
    // records from several ranks: first in their global input order (the tie), then the stable key sort — equal
    // keys keep the one-rank store's input order, whatever order the pieces arrived in
    MH_TRY(ensure(ctx, B.tie2, sizeof(uint64_t) * n));
    MH_TRY(ensure(ctx, B.tval, sizeof(uint32_t) * n));
    MH_TRY(ensure(ctx, B.tkey, sizeof(uint64_t) * n));
    size_t t2 = 0;
    HIPCHK(ctx, rocprim::radix_sort_pairs(nullptr, t2, (uint64_t *)B.tie.p, (uint64_t *)B.tie2.p, (uint32_t *)B.val.p,
                                          (uint32_t *)B.tval.p, (size_t)n, 0u, 64u, st));
    MH_TRY(ensure(ctx, B.sort_tmp, t2 + 256));
    HIPCHK(ctx, rocprim::radix_sort_pairs(B.sort_tmp.p, t2, (uint64_t *)B.tie.p, (uint64_t *)B.tie2.p,
                                          (uint32_t *)B.val.p, (uint32_t *)B.tval.p, (size_t)n, 0u, 64u, st));
    hipLaunchKernelGGL(k_gather_key, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (const uint64_t *)B.key.p,
                       (const uint32_t *)B.tval.p, n, (uint64_t *)B.tkey.p);
    HIPCHK(ctx, hipGetLastError());
    kin = (const uint64_t *)B.tkey.p;
    vin = (const uint32_t *)B.tval.p;
  }
  HIPCHK(ctx, rocprim::radix_sort_pairs(nullptr, tmp, kin, (uint64_t *)B.key2.p, vin, (uint32_t *)B.val2.p, (size_t)n,
                                        0u, end_bit, st));
  MH_TRY(ensure(ctx, B.sort_tmp, tmp + 256));
  HIPCHK(ctx, rocprim::radix_sort_pairs(B.sort_tmp.p, tmp, kin, (uint64_t *)B.key2.p, vin, (uint32_t *)B.val2.p,
                                        (size_t)n, 0u, end_bit, st));
  stage_end(ctx);
  // sorted offsets, then the gather
  MH_TRY(ensure(ctx, B.soff, sizeof(int64_t) * (n + 1)));
  MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(int64_t) * scan_partials_count(n + 1) + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  HIPCHK(ctx, device_scan<int64_t>(st, n + 1, LoadSortedSize{(const uint32_t *)B.val2.p, (const int64_t *)B.roff.p, n},
                                   StoreOff64{(int64_t *)B.soff.p, 0}, OpSum{}, (int64_t)0,
                                   (int64_t *)ctx->scan_partials.p, (int64_t *)ctx->d_small.p));
  MH_TRY(ensure(ctx, B.sinfo, sizeof(RInfo) * n));
  int32_t *bad = (int32_t *)((char *)ctx->d_small.p + 68);
  HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, st));
  if (B.spilled > 0) {   // spilled records: the sorted bytes are assembled on the host when written
    hipLaunchKernelGGL(k_bam_sinfo, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (const uint32_t *)B.val2.p,
                       n, (const RInfo *)B.info.p, (RInfo *)B.sinfo.p, bad);
    HIPCHK(ctx, hipGetLastError());
    MH_TRY(bam_check_bounds(ctx, bad, "k_bam_sinfo"));
    {
      int64_t *hs = pinned_small(ctx);
      if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
      HIPCHK(ctx, hipMemcpyAsync(hs + 24, (const int64_t *)B.soff.p + n, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipMemcpyAsync(hs + 25, (const int64_t *)B.roff.p + n, 8, hipMemcpyDeviceToHost, st));
      SYNCCHK(ctx, hipStreamSynchronize(st));
      if (hs[24] != B.bytes || hs[25] != B.bytes)
        return arg_fail(ctx, MH_E_STATE, "BAM store: record offsets do not add up to the store's size (internal)");
    }
    B.sorted = true;
    return MH_OK;
  }
  MH_TRY(ensure(ctx, B.srecs, B.bytes + 64));
  {   // the offsets must close on the store's byte count (a record-size mismatch would send the copies astray)
    int64_t *hs = pinned_small(ctx);
    if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
    HIPCHK(ctx, hipMemcpyAsync(hs + 24, (const int64_t *)B.soff.p + n, 8, hipMemcpyDeviceToHost, st));
    if (!pa) HIPCHK(ctx, hipMemcpyAsync(hs + 25, (const int64_t *)B.roff.p + n, 8, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    if (hs[24] != B.bytes || (!pa && hs[25] != B.bytes))
      return arg_fail(ctx, MH_E_STATE, "BAM store: record offsets do not add up to the store's size (internal)");
  }
  if (pa) {
    stage_begin(ctx, "bam_write");
    hipLaunchKernelGGL(k_bam_slots, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (const uint32_t *)B.val2.p, n,
                       (uint32_t *)B.val.p);   // (the sort's input values are no longer needed)
    hipLaunchKernelGGL(k_bam_write<BW_G>, dim3(grid_for(n * BW_G, 256, INT32_MAX)), dim3(256), 0, st,
                       *(const ParseArgs *)pa, (const BamTpl *)B.tpl.p, n, B.n_files, (const uint32_t *)B.val.p,
                       (const int64_t *)B.soff.p, (uint8_t *)B.srecs.p, (uint64_t *)nullptr, (uint32_t *)nullptr,
                       (RInfo *)B.sinfo.p, (int64_t)0, B.bytes, bad);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  } else {
    stage_begin(ctx, "bam_gather");
    hipLaunchKernelGGL(k_bam_gather, dim3(grid_for(n * 32, 256, INT32_MAX)), dim3(256), 0, st,
                       (const uint8_t *)B.recs.p, (const int64_t *)B.roff.p, (const uint32_t *)B.val2.p,
                       (const int64_t *)B.soff.p, n, (uint8_t *)B.srecs.p, (const RInfo *)B.info.p,
                       (RInfo *)B.sinfo.p, B.bytes, B.bytes, bad);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  }
  MH_TRY(bam_check_bounds(ctx, bad, pa ? "k_bam_write (sorted places)" : "k_bam_gather"));
  B.sorted = true;
  return MH_OK;
}

// after a direct sorted write, more records: the sorted block becomes the store's input-order prefix (a stable sort
// keeps its order on ties, which is the order it had as input)
__global__ void k_iota(uint32_t *v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

int32_t bam_undirect(mh_ctx *ctx) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  const int64_t n = B.n_rec;
  MH_TRY(ensure(ctx, B.recs, B.bytes + 64));
  MH_TRY(ensure(ctx, B.roff, sizeof(int64_t) * (n + 1)));
  MH_TRY(ensure(ctx, B.key, sizeof(uint64_t) * n + 8));
  MH_TRY(ensure(ctx, B.val, sizeof(uint32_t) * n + 8));
  MH_TRY(ensure(ctx, B.info, sizeof(RInfo) * n + 16));
  HIPCHK(ctx, hipMemcpyAsync(B.recs.p, B.srecs.p, B.bytes, hipMemcpyDeviceToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(B.roff.p, B.soff.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(B.key.p, B.key2.p, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(B.info.p, B.sinfo.p, sizeof(RInfo) * n, hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (uint32_t *)B.val.p, n);
  HIPCHK(ctx, hipGetLastError());
  SYNCCHK(ctx, hipStreamSynchronize(st));
  B.direct = false;
  B.sorted = false;
  return MH_OK;
}

int32_t bam_fetch_sorted(mh_ctx *ctx, uint8_t *recs, int64_t *soff, int32_t *info) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  const int64_t n = B.n_rec;
  if (n == 0) return MH_OK;
  static_assert(sizeof(RInfo) == 16, "RInfo layout");
  if (recs && B.spilled > 0) {   // the sorted stream assembled from the host blocks
    MH_TRY(bam_spill(ctx));
    MH_TRY(bam_sort(ctx));   // (a no-op unless the spill undid a direct write's order)
    BamHostOrder o;
    MH_TRY(bam_host_order(ctx, o));
    bam_assemble(B, o, 0, B.bytes, recs, 16);
    recs = nullptr;
  }
  if (recs) HIPCHK(ctx, hipMemcpyAsync(recs, B.srecs.p, B.bytes, hipMemcpyDeviceToHost, st));
  if (soff) HIPCHK(ctx, hipMemcpyAsync(soff, B.soff.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, st));
  if (info) HIPCHK(ctx, hipMemcpyAsync(info, B.sinfo.p, sizeof(RInfo) * n, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  return MH_OK;
}

// ---- store pieces across ranks (configs[4] on N GPUs) ----------------------------------------------------------
__global__ void k_bam_import_idx(int64_t *roff, int64_t n, int64_t r0, int64_t base, uint32_t *val, int64_t vbase) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) roff[i] = roff[i] - r0 + base;
  if (i < n) val[i] = (uint32_t)(vbase + i);
}

int32_t bam_export(mh_ctx *ctx, int64_t r0, int64_t r1, uint8_t *recs, int64_t *roff, uint64_t *key, int32_t *info) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  if (B.direct) MH_TRY(bam_undirect(ctx));   // (the direct write's sorted order becomes the input order)
  if (r0 < 0 || r1 < r0 || r1 > B.n_rec) return arg_fail(ctx, MH_E_ARG, "record range outside the store");
  const int64_t n = r1 - r0;
  int64_t ab[2] = {0, 0};
  HIPCHK(ctx, hipMemcpyAsync(ab, (const int64_t *)B.roff.p + r0, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(ab + 1, (const int64_t *)B.roff.p + r1, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  if (recs) {   // the bytes [ab[0], ab[1]): the spilled part from the host blocks, the rest from HBM
    int64_t a = ab[0];
    for (const auto &h : B.spill) {
      if (a >= ab[1] || h.b1 <= a) continue;
      const int64_t e = std::min(h.b1, ab[1]);
      HIPCHK(ctx, hipMemcpyAsync(recs + (a - ab[0]), h.p + (a - h.b0), (size_t)(e - a), hipMemcpyDefault, st));
      a = e;
    }
    if (a < ab[1])
      HIPCHK(ctx, hipMemcpyAsync(recs + (a - ab[0]), (const uint8_t *)B.recs.p + (a - B.spilled), (size_t)(ab[1] - a),
                                 hipMemcpyDefault, st));
  }
  if (roff) HIPCHK(ctx, hipMemcpyAsync(roff, (const int64_t *)B.roff.p + r0, 8 * (size_t)(n + 1), hipMemcpyDefault, st));
  if (key && n) HIPCHK(ctx, hipMemcpyAsync(key, (const uint64_t *)B.key.p + r0, 8 * (size_t)n, hipMemcpyDefault, st));
  if (info && n) HIPCHK(ctx, hipMemcpyAsync(info, (const RInfo *)B.info.p + r0, sizeof(RInfo) * n, hipMemcpyDefault, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  return MH_OK;
}

int32_t bam_import(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *key, const int32_t *info,
                   int64_t n, const uint64_t *tie) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  if (!B.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  if (B.direct) MH_TRY(bam_undirect(ctx));
  if (n <= 0) return MH_OK;
  // ties: the records' global input order (pieces from several ranks, in any order); every import of a store gives
  // them or none does
  if (B.n_rec == 0) B.use_tie = tie != nullptr;
  if (B.use_tie != (tie != nullptr)) return arg_fail(ctx, MH_E_ARG, "BAM import: tie order given for some pieces only");
  if (B.n_rec + n >= (int64_t)UINT32_MAX) return arg_fail(ctx, MH_E_CAPACITY, "more than 2^32 records in one BAM");
  int64_t ab[2] = {0, 0};
  HIPCHK(ctx, hipMemcpyAsync(ab, roff, 8, hipMemcpyDefault, st));
  HIPCHK(ctx, hipMemcpyAsync(ab + 1, roff + n, 8, hipMemcpyDefault, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  const int64_t add = ab[1] - ab[0];
  if (add < 0) return arg_fail(ctx, MH_E_ARG, "record offsets decrease");
  if (B.cap > 0 && B.bytes > B.spilled && B.bytes - B.spilled + add > B.cap) MH_TRY(bam_spill(ctx));
  if (ensure_keep(ctx, B.recs, B.bytes - B.spilled + add + 64, B.bytes - B.spilled) != MH_OK) {
    // (as bam_add: when the records do not fit beside the resident ones, the resident ones go to the host first)
    if (B.bytes == B.spilled) return MH_E_OOM;
    ctx->err.clear();
    MH_TRY(bam_spill(ctx));
    MH_TRY(ensure_keep(ctx, B.recs, add + 64, 0));
  }
  MH_TRY(ensure_keep(ctx, B.roff, sizeof(int64_t) * (B.n_rec + n + 1), sizeof(int64_t) * (B.n_rec + 1)));
  MH_TRY(ensure_keep(ctx, B.key, sizeof(uint64_t) * (B.n_rec + n), sizeof(uint64_t) * B.n_rec));
  MH_TRY(ensure_keep(ctx, B.val, sizeof(uint32_t) * (B.n_rec + n), sizeof(uint32_t) * B.n_rec));
  MH_TRY(ensure_keep(ctx, B.info, sizeof(RInfo) * (B.n_rec + n), sizeof(RInfo) * B.n_rec));
  if (tie) {
    MH_TRY(ensure_keep(ctx, B.tie, sizeof(uint64_t) * (B.n_rec + n), sizeof(uint64_t) * B.n_rec));
    HIPCHK(ctx, hipMemcpyAsync((uint64_t *)B.tie.p + B.n_rec, tie, 8 * (size_t)n, hipMemcpyDefault, st));
  }
  if (add) HIPCHK(ctx, hipMemcpyAsync((uint8_t *)B.recs.p + (B.bytes - B.spilled), recs, (size_t)add, hipMemcpyDefault, st));
  int64_t *ro = (int64_t *)B.roff.p + B.n_rec;
  HIPCHK(ctx, hipMemcpyAsync(ro, roff, 8 * (size_t)(n + 1), hipMemcpyDefault, st));
  HIPCHK(ctx, hipMemcpyAsync((uint64_t *)B.key.p + B.n_rec, key, 8 * (size_t)n, hipMemcpyDefault, st));
  HIPCHK(ctx, hipMemcpyAsync((RInfo *)B.info.p + B.n_rec, info, sizeof(RInfo) * n, hipMemcpyDefault, st));
  hipLaunchKernelGGL(k_bam_import_idx, dim3(grid_for(n + 1, 256, INT32_MAX)), dim3(256), 0, st, ro, n, ab[0], B.bytes,
                     (uint32_t *)B.val.p + B.n_rec, B.n_rec);
  HIPCHK(ctx, hipGetLastError());
  SYNCCHK(ctx, hipStreamSynchronize(st));
  B.n_rec += n;
  B.bytes += add;
  B.sorted = false;
  return MH_OK;
}

// ---- bounded HBM: spilled records -----------------------------------------------------------------------------
int32_t bam_spill(mh_ctx *ctx) {
  BamStore &B = ctx->bam;
  if (B.direct) MH_TRY(bam_undirect(ctx));
  const int64_t len = B.bytes - B.spilled;
  if (len <= 0) return MH_OK;
  uint8_t *p = nullptr;
  const bool mapped = !B.spill_dir.empty();
  if (mapped) {   // an unlinked temporary file (samtools sort -m's temporary files): the kernel may write it back
    std::string tmpl = B.spill_dir + "/mitty_bam_spill_XXXXXX";
    std::vector<char> path(tmpl.begin(), tmpl.end());
    path.push_back('\0');
    const int fd = mkstemp(path.data());
    if (fd < 0) return arg_fail(ctx, MH_E_ARG, "BAM spill: cannot create a file in " + B.spill_dir);
    unlink(path.data());
    void *m = MAP_FAILED;
    if (ftruncate(fd, (off_t)len) == 0) m = mmap(nullptr, (size_t)len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return arg_fail(ctx, MH_E_OOM, "BAM spill: cannot map " + std::to_string(len) + " bytes");
    p = (uint8_t *)m;
  } else {
    p = (uint8_t *)malloc((size_t)len);
  }
  if (!p) return arg_fail(ctx, MH_E_OOM, "host memory for spilled BAM records (" + std::to_string(len) + " bytes)");
  stage_begin(ctx, "bam_spill");
  if (hipMemcpyAsync(p, B.recs.p, (size_t)len, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    if (mapped) munmap(p, (size_t)len); else free(p);
    return hip_fail(ctx, hipGetLastError(), "BAM spill D2H", __FILE__, __LINE__);
  }
  stage_end(ctx);
  B.spill.push_back(BamStore::HostBlock{p, B.spilled, B.bytes, mapped});
  B.spilled = B.bytes;   // (the sort's order, offsets and info stay valid: only where the bytes live changed)
  return MH_OK;
}

int32_t bam_host_order(mh_ctx *ctx, BamHostOrder &o) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  const int64_t n = B.n_rec;
  if (!B.sorted) return arg_fail(ctx, MH_E_STATE, "BAM store not sorted (internal)");
  o.val.resize((size_t)n + 1);
  o.roff.resize((size_t)n + 1);
  o.soff.resize((size_t)n + 1);
  if (n) {
    HIPCHK(ctx, hipMemcpyAsync(o.val.data(), B.val2.p, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(o.roff.data(), B.roff.p, 8 * (size_t)(n + 1), hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(o.soff.data(), B.soff.p, 8 * (size_t)(n + 1), hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
  } else {
    o.roff[0] = o.soff[0] = 0;
  }
  return MH_OK;
}

void bam_assemble(const BamStore &B, const BamHostOrder &o, int64_t w0, int64_t w1, uint8_t *dst, int threads) {
  const int64_t n = B.n_rec;
  if (w1 <= w0 || n == 0) return;
  // sorted records overlapping [w0, w1): k0 = the one holding byte w0, k1 = the first starting at or after w1
  const int64_t k0 = std::upper_bound(o.soff.begin(), o.soff.begin() + n + 1, w0) - o.soff.begin() - 1;
  const int64_t k1 = std::lower_bound(o.soff.begin(), o.soff.begin() + n + 1, w1) - o.soff.begin();
  const int64_t nk = k1 - k0;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, nk / 4096));
  auto part = [&](int t) {
    const int64_t a = k0 + nk * t / T, b = k0 + nk * (t + 1) / T;
    size_t blk = 0;
    for (int64_t k = a; k < b; k++) {
      const uint32_t r = o.val[k];
      const int64_t src = o.roff[r], len = o.roff[r + 1] - src, s = o.soff[k];
      const int64_t lo = std::max(s, w0), hi = std::min(s + len, w1);
      if (hi <= lo) continue;
      if (!(B.spill[blk].b0 <= src && src < B.spill[blk].b1))   // the host block holding the record (whole records)
        blk = std::upper_bound(B.spill.begin(), B.spill.end(), src,
                               [](int64_t x, const BamStore::HostBlock &h) { return x < h.b0; }) - B.spill.begin() - 1;
      const BamStore::HostBlock &h = B.spill[blk];
      std::memcpy(dst + (lo - w0), h.p + (src - h.b0) + (lo - s), (size_t)(hi - lo));
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  part(0);
  for (auto &x : th) x.join();
}

// ---- the BAI's device plan -----------------------------------------------------------------------------------
namespace {

// per record: the 16 kbp windows it overlaps take its index unless the record before already overlaps them (that
// one is earlier: a window's first record wins, with few atomics per window); a reference's window count is the
// wave's max per reference, one atomic per wave and reference (one per record, all on one word, took 200 ms for a
// configs[4] store of 17 M records, round 4)
__global__ void k_bai_mark(const RInfo *info, int64_t n, const int64_t *woff, int32_t n_refs, uint32_t *lin,
                           uint32_t *nwin, int32_t *bad) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int mt = -1;          // this record's reference, when it has windows
  uint32_t my = 0;      // its window count (last window + 1)
  if (k < n) {
    const RInfo r = info[k];
    if (r.tid < 0 || r.tid >= n_refs || r.beg < 0 || r.bin >= 37450u) {
      atomicOr(bad, 1);
    } else {
      const int64_t w0 = r.beg >> 14, w1 = (int64_t)(r.end - 1) >> 14;
      if (w1 >= woff[r.tid + 1] - woff[r.tid]) {
        atomicOr(bad, 2);
      } else if (w1 >= 0) {
        int64_t from = w0;
        if (k > 0) {
          const RInfo q = info[k - 1];
          if (q.tid > r.tid || (q.tid == r.tid && q.beg > r.beg)) atomicOr(bad, 4);   // (the store is sorted)
          if (q.tid == r.tid && q.end - 1 >= q.beg) {
            const int64_t p0 = q.beg >> 14, p1 = (int64_t)(q.end - 1) >> 14;
            if (p0 <= w0 && p1 >= w0) from = p1 + 1;   // windows [w0, p1] already have an earlier record
          }
        }
        uint32_t *L = lin + woff[r.tid];
        for (int64_t w = from; w <= w1; w++) atomicMin(&L[w], (uint32_t)k);
        mt = r.tid;
        my = (uint32_t)(w1 + 1);
      }
    }
  }
  uint64_t rem = __ballot(mt >= 0);
  while (rem) {   // per reference present in the wave (sorted records: usually one), its max by a butterfly
    const int t = __shfl(mt, __builtin_ctzll(rem), 64);
    uint32_t v = mt == t ? my : 0u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = (uint32_t)__shfl_xor((int)v, d, 64);
      v = o > v ? o : v;
    }
    if (lane == __builtin_ctzll(rem)) atomicMax(&nwin[t], v);
    rem &= ~__ballot(mt == t);
  }
}

__device__ __forceinline__ bool run_start(const RInfo *info, int64_t k) {
  return k == 0 || info[k - 1].tid != info[k].tid || info[k - 1].bin != info[k].bin;
}
struct LoadRunStart {
  const RInfo *info;
  int64_t n;
  __device__ int64_t operator()(int64_t k) const { return k < n && run_start(info, k) ? 1 : 0; }
};
struct StoreRunStart {
  uint32_t *runs;
  __device__ void operator()(int64_t k, int64_t incl, int64_t ex) const {
    if (incl != ex) runs[ex] = (uint32_t)k;
  }
};

// the plan's offsets: per run (tid << 32 | bin, offset of its first record, offset of its end, records), then per
// window the offset of its first record (-1: none)
__global__ void k_bai_gather(const RInfo *info, const int64_t *soff, const uint32_t *runs, int64_t n_runs, int64_t n,
                             const uint32_t *lin, int64_t n_win, int64_t *out_runs, int64_t *out_win) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_runs) {
    const int64_t kb = runs[i], ke = i + 1 < n_runs ? (int64_t)runs[i + 1] : n;
    const RInfo r = info[kb];
    out_runs[4 * i] = ((int64_t)r.tid << 32) | (int64_t)r.bin;
    out_runs[4 * i + 1] = soff[kb];
    out_runs[4 * i + 2] = soff[ke];
    out_runs[4 * i + 3] = ke - kb;
  }
  if (i < n_win) out_win[i] = lin[i] == 0xffffffffu ? -1 : soff[lin[i]];
}

}  // namespace

int32_t bam_bai_plan(mh_ctx *ctx, BaiPlan &plan, std::vector<int64_t> &offs, bool *ok) {
  BamStore &B = ctx->bam;
  *ok = false;
  const int32_t n_refs = (int32_t)B.ref_names.size();
  plan.refs.assign((size_t)n_refs, BaiRef{});
  offs.clear();
  std::vector<int64_t> hr, hw, woff;
  std::vector<uint32_t> hn;
  bool raw_ok = false;
  MH_TRY(bam_bai_raw(ctx, hr, hw, hn, woff, &raw_ok));
  if (!raw_ok) return MH_OK;   // (outside the device plan's checks: the host plans and reports what it finds)
  const int64_t n_runs = (int64_t)hr.size() / 4, n_win = (int64_t)hw.size();
  // offs: the runs' (first, end) offsets, then the windows'
  offs.resize(2 * (size_t)n_runs + (size_t)n_win);
  for (int64_t r = 0; r < n_runs; r++) {
    offs[2 * r] = hr[4 * r + 1];
    offs[2 * r + 1] = hr[4 * r + 2];
  }
  for (int64_t w = 0; w < n_win; w++) offs[2 * n_runs + w] = hw[w];
  for (int64_t r0 = 0; r0 < n_runs;) {   // the runs of one reference are consecutive (the store is sorted)
    const int32_t t = (int32_t)(hr[4 * r0] >> 32);
    int64_t r1 = r0;
    BaiRef &R = plan.refs[t];
    if (R.n != 0) return MH_OK;   // (a reference's runs apart: not sorted — the host plan reports it)
    while (r1 < n_runs && (int32_t)(hr[4 * r1] >> 32) == t) {
      R.n += hr[4 * r1 + 3];
      R.runs.push_back(BaiRun{(uint32_t)(hr[4 * r1] & 0xffffffff), 2 * r1, 2 * r1 + 1});
      r1++;
    }
    R.vi = 2 * r0;
    R.vj = 2 * (r1 - 1) + 1;
    std::stable_sort(R.runs.begin(), R.runs.end(), [](const BaiRun &x, const BaiRun &y) { return x.bin < y.bin; });
    R.lin.assign(hn[t], -1);
    for (uint32_t w = 0; w < hn[t]; w++)
      if (hw[woff[t] + w] >= 0) R.lin[w] = 2 * n_runs + woff[t] + w;
    r0 = r1;
  }
  *ok = true;
  return MH_OK;
}

// ---- range partition across ranks (configs[4] on N GPUs: every rank sorts and writes one coordinate range) --------
namespace {

constexpr int PART_MAX = 1024;   // destinations (ranks)

// dest = the number of splitters <= key (splitters ascending): the coordinate range the record belongs to
__global__ void k_part_dest(const uint64_t *key, int64_t n, const uint64_t *split, int32_t n_split, uint32_t *dest) {
  __shared__ uint64_t s[PART_MAX];
  for (int i = threadIdx.x; i < n_split; i += blockDim.x) s[i] = split[i];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = key[i];
  int lo = 0, hi = n_split;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid] <= k) lo = mid + 1; else hi = mid;
  }
  dest[i] = (uint32_t)lo;
}

// start[d] = the first position of the dest-sorted records whose destination is >= d (d = 0..n_dest)
__global__ void k_part_starts(const uint32_t *dk, int64_t n, int32_t n_dest, int64_t *start) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  const int32_t lo = k == 0 ? 0 : (int32_t)dk[k - 1] + 1, hi = k == n ? n_dest : (int32_t)dk[k];
  for (int32_t d = lo; d <= hi; d++) start[d] = k;
}

// a segment's layout (bam_part_layout in _native.py): records, 8-aligned; n + 1 record offsets from the segment's
// records; n keys; n BAI infos; n ties
struct PartSeg {
  int64_t o_roff, o_key, o_info, o_tie, total;
};
__host__ __device__ inline PartSeg part_layout(int64_t n, int64_t nb) {
  PartSeg g;
  g.o_roff = (nb + 7) & ~(int64_t)7;
  g.o_key = g.o_roff + 8 * (n + 1);
  g.o_info = g.o_key + 8 * n;
  g.o_tie = g.o_info + 16 * n;
  g.total = g.o_tie + 8 * n;
  return g;
}

// 32 lanes per record (as k_bam_gather): sorted-by-destination position k holds input record ord[k]; its bytes,
// offset, key, info and tie go to its destination's segment
__global__ void __launch_bounds__(256) k_part_write(const uint8_t *src, const int64_t *roff, const uint32_t *ord,
                                                    const uint32_t *dk, const int64_t *soff, const int64_t *start,
                                                    const int64_t *seg, const uint64_t *key, const RInfo *info,
                                                    uint64_t tie_base, int64_t n, uint8_t *out, int64_t src_bytes,
                                                    int64_t out_cap, int32_t *bad) {
  constexpr int G = 32;
  const int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int gl = threadIdx.x & (G - 1);
  if (k >= n) return;
  const uint32_t r = ord[k], d = dk[k];
  if (r >= (uint64_t)n) {
    if (gl == 0) atomicOr(bad, 2);
    return;
  }
  const int64_t s0 = start[d], s1 = start[d + 1], nd = s1 - s0, sb = soff[s0];
  const PartSeg g = part_layout(nd, soff[s1] - sb);
  uint8_t *base = out + seg[d];
  const int64_t a = roff[r], len = roff[r + 1] - a, o = soff[k] - sb;
  if (a < 0 || len < 0 || a + len > src_bytes || seg[d] + g.total > out_cap || o < 0 || o + len > g.o_roff) {
    if (gl == 0) atomicOr(bad, 4);
    return;
  }
  const uint8_t *__restrict__ sp = src + a;
  uint8_t *__restrict__ dp = base + o;
  for (int64_t j0 = 0; j0 < len; j0 += 8 * G) {
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t j = j0 + gl + G * u;
      v[u] = j < len ? sp[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t j = j0 + gl + G * u;
      if (j < len) dp[j] = v[u];
    }
  }
  if (gl == 0) {
    const int64_t j = k - s0;
    int64_t *ro = (int64_t *)(base + g.o_roff);
    ro[j] = o;
    if (j == nd - 1) ro[nd] = o + len;
    ((uint64_t *)(base + g.o_key))[j] = key[r];
    ((RInfo *)(base + g.o_info))[j] = info[r];
    ((uint64_t *)(base + g.o_tie))[j] = tie_base + r;
  }
}

}  // namespace

int32_t bam_partition(mh_ctx *ctx, const uint64_t *split, int32_t n_dest, uint64_t tie_base, int64_t *seg_off,
                      int64_t *seg_n, int64_t *seg_bytes) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  if (n_dest < 1 || n_dest > PART_MAX) return arg_fail(ctx, MH_E_ARG, "partition: 1..1024 destinations");
  for (int32_t i = 1; i + 1 < n_dest; i++)
    if (split[i] < split[i - 1]) return arg_fail(ctx, MH_E_ARG, "partition: splitters not ascending");
  if (B.direct) MH_TRY(bam_undirect(ctx));   // (input order = the direct write's sorted order: ties keep their order)
  if (B.spilled > 0) return arg_fail(ctx, MH_E_STATE, "partition: the store has spilled (stage pieces unbounded)");
  const int64_t n = B.n_rec;
  if (n >= ((int64_t)1 << 30)) return arg_fail(ctx, MH_E_CAPACITY, "partition: more than 2^30 records in one piece");
  MH_TRY(ensure(ctx, B.part_split, 8 * (size_t)n_dest + 64));
  MH_TRY(ensure(ctx, B.part_dest, 4 * (size_t)n + 64));
  MH_TRY(ensure(ctx, B.part_dk, 4 * (size_t)n + 64));
  MH_TRY(ensure(ctx, B.part_ord, 4 * (size_t)n + 64));
  MH_TRY(ensure(ctx, B.part_soff, 8 * (size_t)(n + 1) + 64));
  MH_TRY(ensure(ctx, B.part_start, 8 * (size_t)(n_dest + 1) + 64));
  MH_TRY(ensure(ctx, B.part_seg, 8 * (size_t)(n_dest + 1) + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int64_t *hs = pinned_small(ctx);
  if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  std::vector<int64_t> start((size_t)n_dest + 1, 0), sb((size_t)n_dest + 1, 0);
  if (n > 0) {
    if (n_dest > 1)
      HIPCHK(ctx, hipMemcpyAsync(B.part_split.p, split, 8 * (size_t)(n_dest - 1), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_part_dest, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, (const uint64_t *)B.key.p, n,
                       (const uint64_t *)B.part_split.p, n_dest - 1, (uint32_t *)B.part_dest.p);
    HIPCHK(ctx, hipGetLastError());
    // stable by destination (the records' input order kept inside each destination)
    unsigned end_bit = 1;
    while ((1u << end_bit) < (unsigned)n_dest) end_bit++;
    size_t tmp = 0;
    HIPCHK(ctx, lsd_sort_pairs_iota(nullptr, tmp, nullptr, nullptr, nullptr, n, end_bit, st));
    MH_TRY(ensure(ctx, B.part_tmp, tmp + 256));
    HIPCHK(ctx, lsd_sort_pairs_iota(B.part_tmp.p, tmp, (const uint32_t *)B.part_dest.p, (uint32_t *)B.part_dk.p,
                                    (uint32_t *)B.part_ord.p, n, end_bit, st));
    MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(int64_t) * scan_partials_count(n + 1) + 64));
    HIPCHK(ctx, device_scan<int64_t>(st, n + 1, LoadSortedSize{(const uint32_t *)B.part_ord.p, (const int64_t *)B.roff.p, n},
                                     StoreOff64{(int64_t *)B.part_soff.p, 0}, OpSum{}, (int64_t)0,
                                     (int64_t *)ctx->scan_partials.p, (int64_t *)ctx->d_small.p));
    hipLaunchKernelGGL(k_part_starts, dim3(grid_for(n + 1, 256, INT32_MAX)), dim3(256), 0, st,
                       (const uint32_t *)B.part_dk.p, n, n_dest, (int64_t *)B.part_start.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(start.data(), B.part_start.p, 8 * start.size(), hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    for (int32_t d = 0; d <= n_dest; d++)
      HIPCHK(ctx, hipMemcpyAsync(&sb[d], (const int64_t *)B.part_soff.p + start[d], 8, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    if (start[n_dest] != n || sb[n_dest] != B.bytes)
      return arg_fail(ctx, MH_E_STATE, "partition: record counts or offsets do not add up (internal)");
  }
  std::vector<int64_t> seg((size_t)n_dest + 1, 0);
  for (int32_t d = 0; d < n_dest; d++) {
    seg_n[d] = start[d + 1] - start[d];
    seg_bytes[d] = sb[d + 1] - sb[d];
    seg[d + 1] = seg[d] + part_layout(seg_n[d], seg_bytes[d]).total;
  }
  for (int32_t d = 0; d <= n_dest; d++) seg_off[d] = seg[d];
  MH_TRY(ensure(ctx, B.send, (size_t)seg[n_dest] + 64));
  B.send_bytes = seg[n_dest];
  if (n > 0) {
    HIPCHK(ctx, hipMemcpyAsync(B.part_seg.p, seg.data(), 8 * seg.size(), hipMemcpyHostToDevice, st));
    int32_t *bad = (int32_t *)((char *)ctx->d_small.p + 76);
    HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, st));
    hipLaunchKernelGGL(k_part_write, dim3(grid_for(n * 32, 256, INT32_MAX)), dim3(256), 0, st, (const uint8_t *)B.recs.p,
                       (const int64_t *)B.roff.p, (const uint32_t *)B.part_ord.p, (const uint32_t *)B.part_dk.p,
                       (const int64_t *)B.part_soff.p, (const int64_t *)B.part_start.p, (const int64_t *)B.part_seg.p,
                       (const uint64_t *)B.key.p, (const RInfo *)B.info.p, tie_base, n, (uint8_t *)B.send.p,
                       B.bytes, seg[n_dest], bad);
    HIPCHK(ctx, hipGetLastError());
    MH_TRY(bam_check_bounds(ctx, bad, "k_part_write"));
  }
  return MH_OK;
}

int32_t bam_bai_raw(mh_ctx *ctx, std::vector<int64_t> &runs, std::vector<int64_t> &win, std::vector<uint32_t> &nwin,
                    std::vector<int64_t> &woff, bool *ok) {
  BamStore &B = ctx->bam;
  hipStream_t st = ctx->stream;
  *ok = false;
  const int64_t n = B.n_rec;
  const int32_t n_refs = (int32_t)B.ref_names.size();
  woff.assign((size_t)n_refs + 1, 0);
  for (int32_t t = 0; t < n_refs; t++) woff[t + 1] = woff[t] + (B.ref_len[t] >> 14) + 1;
  const int64_t n_win = woff[n_refs];
  runs.clear();
  win.assign((size_t)n_win, -1);
  nwin.assign((size_t)n_refs, 0);
  if (n == 0) {
    *ok = true;
    return MH_OK;
  }
  if (!B.sorted) return arg_fail(ctx, MH_E_STATE, "BAI plan of an unsorted store (internal)");
  MH_TRY(ensure(ctx, B.bai_lin, 4 * (size_t)n_win + 4 * (size_t)n_refs + 8 * (size_t)(n_refs + 1) + 64));
  uint32_t *lin = (uint32_t *)B.bai_lin.p, *dn = lin + n_win;
  int64_t *d_woff = (int64_t *)(((uintptr_t)(dn + n_refs) + 7) & ~(uintptr_t)7);
  MH_TRY(ensure(ctx, B.bai_runs, 4 * (size_t)n + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int32_t *bad = (int32_t *)((char *)ctx->d_small.p + 72);
  int64_t *total = (int64_t *)((char *)ctx->d_small.p + 80);
  MH_TRY(ensure(ctx, ctx->scan_partials, scan_lb_scratch_bytes<int64_t>(n)));
  int64_t *hs = pinned_small(ctx);
  if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  stage_begin(ctx, "bam_bai_plan");
  HIPCHK(ctx, hipMemsetAsync(lin, 0xff, 4 * (size_t)n_win, st));
  HIPCHK(ctx, hipMemsetAsync(dn, 0, 4 * (size_t)n_refs, st));
  HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, st));
  HIPCHK(ctx, hipMemcpyAsync(d_woff, woff.data(), 8 * woff.size(), hipMemcpyHostToDevice, st));
  const RInfo *info = (const RInfo *)B.sinfo.p;
  hipLaunchKernelGGL(k_bai_mark, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, info, n,
                     (const int64_t *)d_woff, n_refs, lin, dn, bad);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, device_scan_sum<int64_t>(st, n, LoadRunStart{info, n}, StoreRunStart{(uint32_t *)B.bai_runs.p},
                                       ctx->scan_partials.p, total));
  HIPCHK(ctx, hipMemcpyAsync(hs + 28, total, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(hs + 29, bad, 4, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  const int64_t n_runs = hs[28];
  if ((int32_t)(hs[29] & 0xffffffff)) {   // outside the device plan's checks
    stage_end(ctx);
    return MH_OK;
  }
  MH_TRY(ensure(ctx, B.bai_out, 8 * (size_t)(4 * n_runs + n_win) + 64));
  int64_t *out_runs = (int64_t *)B.bai_out.p, *out_win = out_runs + 4 * n_runs;
  const int64_t m = n_runs > n_win ? n_runs : n_win;
  hipLaunchKernelGGL(k_bai_gather, dim3(grid_for(m, 256, INT32_MAX)), dim3(256), 0, st, info,
                     (const int64_t *)B.soff.p, (const uint32_t *)B.bai_runs.p, n_runs, n, (const uint32_t *)lin, n_win,
                     out_runs, out_win);
  HIPCHK(ctx, hipGetLastError());
  runs.resize(4 * (size_t)n_runs);
  HIPCHK(ctx, hipMemcpyAsync(runs.data(), out_runs, 8 * runs.size(), hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(win.data(), out_win, 8 * win.size(), hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(nwin.data(), dn, 4 * nwin.size(), hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  stage_end(ctx);
  *ok = true;
  return MH_OK;
}

void bam_free_spill(BamStore &B) {
  for (auto &h : B.spill) {
    if (h.mapped) munmap(h.p, (size_t)(h.b1 - h.b0)); else free(h.p);
  }
  B.spill.clear();
  B.spilled = 0;
}

void bam_release(BamStore &B) {
  bam_free_spill(B);
  for (DevBuf *b : {&B.names, &B.name_off, &B.nl1, &B.nl2, &B.tpl, &B.roff, &B.recs, &B.key, &B.val, &B.info,
                    &B.key2, &B.val2, &B.sort_tmp, &B.soff, &B.srecs, &B.sinfo, &B.in1, &B.in2, &B.bai_lin,
                    &B.bai_runs, &B.bai_out, &B.tie, &B.tie2, &B.tval, &B.tkey, &B.part_dest, &B.part_dk,
                    &B.part_ord, &B.part_soff, &B.part_start, &B.part_seg, &B.part_split, &B.part_tmp, &B.send})
    release(*b);
  B.use_tie = false;
  B.send_bytes = 0;
  B.n_rec = B.bytes = 0;
  B.n_files = 0;
  B.refs_set = false;
  B.sorted = false;
  B.direct = false;
}

}  // namespace mh
