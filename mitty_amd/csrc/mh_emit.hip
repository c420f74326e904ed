// mh_emit.hip — read emission (reference readgenerate.read_generating_worker + rpc.generate_read + fastq_lines,
// mitty/simulation/readgenerate.py:184-230, mitty/simulation/rpc.py:119-160).
//
// Per template the reference: finds each mate's start/end node (searchsorted 'right' on node keys, rpc.py:127-130),
// derives POS, CIGAR, the variant-size list and the sequence (rpc.py:144-160), drops the pair if either read has
// more than two 'N' (readgenerate.py:204), reverse-complements mate 1 (:205-206) and writes the qname
// '@{sample}:{worker}:{ps}:{cnt}|{chrom}|{cpy}|{strand}|{pos}|{rlen}|{cigar}|{v,..}|...' into both FASTQ files
// (:222-230), cnt counting only kept templates.
//
// Device plan (two passes over the template arrays, one over the bases):
//   k_emit_measure  one thread per template: node search (start/end node of both mates, kept for pass 2),
//                   CIGAR / v-list text lengths, N count from the haplotype's N runs (no base reads), keep flag,
//                   per-file record length without the cnt digits.
//   scan            (kept, bytes1, bytes2) -> cnt and exact byte offsets; the cnt digits are added in closed form
//                   (sum_{c<=K} digits(c)), so one scan suffices.
//   k_emit_write    32 templates per 256-thread workgroup:
//                     B0  every thread issues its 16-byte haplotype gathers (both mates of every template) into an
//                         LDS window buffer — all gathers of the tile in flight at once;
//                     A   one owner thread per template formats the qname into the file-1 LDS image;
//                     B1  one wave per (template, file) copies the qname into the file-2 image and writes
//                         '\n' seq '\n+\n' qual '\n' from the LDS windows (reverse complement for mate 1; with
//                         corruption len(seq) placeholder qualities, k_cr_inplace corrupts the record afterwards);
//                     C   both images leave LDS as 16-byte aligned stores (byte stores only at the ragged edges of
//                         the workgroup's output range; neighbouring workgroups own disjoint byte ranges).
// The sequence of a read is hap[p - p_min, min(p + l, hap_end) - p_min): non-'D' nodes tile sample coordinates
// contiguously, so the reference's per-node slice concatenation (rpc.py:146) is one contiguous range.
#include <cstdlib>
#include <cstring>

#include "mh_corrupt.h"
#include "mh_device.h"
#include "mh_internal.h"
#include "mh_scan.h"

namespace mh {

namespace {

struct HapView {
  const int64_t *keys, *ps, *pr, *oplen;
  const uint8_t *op;
  int64_t n_nodes;
  const uint8_t *hap;
  const uint8_t *rc;    // reverse complement of hap (str.maketrans('ATCGN', 'TAGCN') + [::-1]), same length
  const int32_t *bkt;   // node-search buckets (Hap::bkt)
  const Node16 *nd;     // packed node copy (Hap::nd)
  int64_t n_bkt;
  int64_t p_min, hap_len;
  const int64_t *nrs, *nre;
  int64_t n_runs;
};

__device__ __forceinline__ int64_t upper_bound(const int64_t *a, int64_t n, int64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// searchsorted(keys, x, 'right') (rpc.py:127-130) through the bucket table: the answer lies in
// [bkt[k], bkt[k+1]] for x's bucket k, a few keys at most.
__device__ __forceinline__ int64_t node_upper(const HapView &h, int64_t x) {
  int64_t k = (x - h.p_min) >> NODE_BKT_SHIFT;
  if (k < 0) return upper_bound(h.keys, h.n_nodes, x);
  if (k >= h.n_bkt) k = h.n_bkt - 1;
  int64_t lo = h.bkt[k], hi = k + 1 < h.n_bkt ? h.bkt[k + 1] : h.n_nodes;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (h.nd[mid].key() <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// searchsorted(keys, x, 'right') - 1 from a node k0 whose key is <= x: nodes average ~770 bp, so the end node of a
// read is usually k0 or the next one (adjacent 32-byte records) — no second bucket search.
__device__ __forceinline__ int64_t node_walk(const HapView &h, int64_t k0, int64_t x) {
  int64_t k = k0;
  while (k + 1 < h.n_nodes && h.nd[k + 1].key() <= x) k++;
  return k;
}

__device__ __forceinline__ int ndig_u(uint64_t v) {
  if (v <= 0xffffffffull) {
    uint32_t x = (uint32_t)v;
    return x < 10u ? 1 : x < 100u ? 2 : x < 1000u ? 3 : x < 10000u ? 4 : x < 100000u ? 5 : x < 1000000u ? 6
         : x < 10000000u ? 7 : x < 100000000u ? 8 : x < 1000000000u ? 9 : 10;
  }
  int d = 1;
  while (v >= 10) { v /= 10; d++; }
  return d;
}
__device__ __forceinline__ int ndig_s(int64_t v) { return v < 0 ? 1 + ndig_u((uint64_t)(-v)) : ndig_u((uint64_t)v); }

// decimal digits of a value >= 2^32, most significant first, through put(c) (no digit array: a private array would
// be placed in scratch memory); never on the hot path (positions and counts fit 32 bits)
#define put_big(v)                                                          \
  do {                                                                      \
    uint64_t _d = 1;                                                        \
    while ((v) / _d >= 10u) _d *= 10u;                                      \
    for (; _d; _d /= 10u) put((uint8_t)('0' + ((v) / _d) % 10u));           \
  } while (0)

__device__ __forceinline__ char *put_u(char *d, uint64_t v) {
  int nd = ndig_u(v);
  if (v <= 0xffffffffull) {
    uint32_t x = (uint32_t)v;
    for (int i = nd - 1; i >= 0; i--) { d[i] = (char)('0' + x % 10u); x /= 10u; }
  } else {
    for (int i = nd - 1; i >= 0; i--) { d[i] = (char)('0' + v % 10u); v /= 10u; }
  }
  return d + nd;
}
__device__ __forceinline__ char *put_s(char *d, int64_t v) {
  if (v < 0) { *d++ = '-'; return put_u(d, (uint64_t)(-v)); }
  return put_u(d, (uint64_t)v);
}
__device__ __forceinline__ char *put_str(char *d, const char *s, int n) {
  for (int i = 0; i < n; i++) d[i] = s[i];
  return d + n;
}

struct ReadInfo {
  int64_t n0, n1, pos, hap_a;
  int32_t cigar_len, vlist_len, seq_len;
  bool special;
};

__device__ __forceinline__ int64_t node_count(const Node16 &n, int64_t p, int64_t l) {
  const int64_t ol = n.oplen(), ps = n.ps();
  if (n.code() == 3) return ol;
  int64_t hi = p + l - ps < ol ? p + l - ps : ol;
  int64_t lo = p - ps > 0 ? p - ps : 0;
  return hi - lo;
}
__device__ __forceinline__ int64_t node_count(const HapView &h, int64_t k, int64_t p, int64_t l) {
  return node_count(h.nd[k], p, l);
}
__device__ __forceinline__ int64_t node_v(const Node16 &n) {
  const int c = n.code();
  return c == 1 ? 0 : (c == 2 ? n.oplen() : -n.oplen());
}
__device__ __forceinline__ int64_t node_v(const HapView &h, int64_t k) { return node_v(h.nd[k]); }

// POS / special-CIGAR / sequence range of a read whose start and end nodes are known (rpc.py:144-160); n0 is
// node r.n0.
__device__ __forceinline__ void read_place(const HapView &h, const Node16 &n0, int64_t p, int64_t l, ReadInfo &r) {
  r.special = false;
  if (n0.code() == 2) {   // 'I'
    if (r.n0 == r.n1) {
      r.special = true;
      r.pos = n0.pr() - 1;
    } else {
      r.pos = n0.pr();
    }
  } else {
    r.pos = p - n0.ps() + n0.pr();
  }
  int64_t a = p - h.p_min, b = p + l - h.p_min;
  if (b > h.hap_len) b = h.hap_len;
  r.hap_a = a;
  r.seq_len = (int32_t)(b > a ? b - a : 0);
}

// rpc.get_begin_end_nodes + the lengths of rpc.generate_read's outputs.  Requires p >= p_min (n0 >= 0).
__device__ void read_info(const HapView &h, int64_t p, int64_t l, ReadInfo &r) {
  r.n0 = node_upper(h, p) - 1;
  r.n1 = node_upper(h, p + l - 1) - 1;
  int32_t cl = 0, vl = 0;
  bool first = true;
  for (int64_t k = r.n0; k <= r.n1; k++) {
    cl += ndig_s(node_count(h, k, p, l)) + 1;
    if (h.op[k] != '=') {
      vl += ndig_s(node_v(h, k)) + (first ? 0 : 1);
      first = false;
    }
  }
  read_place(h, h.nd[r.n0], p, l, r);
  if (r.special) cl = 1 + ndig_s(p - h.ps[r.n0]) + 1 + ndig_s(l) + 1;
  r.cigar_len = cl;
  r.vlist_len = vl;
}

__device__ char *write_cigar(char *d, const HapView &h, int64_t p, int64_t l, const ReadInfo &r) {
  if (r.special) {
    *d++ = '>';
    d = put_s(d, p - h.ps[r.n0]);
    *d++ = ':';
    d = put_s(d, l);
    *d++ = 'I';
    return d;
  }
  for (int64_t k = r.n0; k <= r.n1; k++) {
    d = put_s(d, node_count(h, k, p, l));
    *d++ = (char)h.op[k];
  }
  return d;
}
__device__ char *write_vlist(char *d, const HapView &h, const ReadInfo &r) {
  bool first = true;
  for (int64_t k = r.n0; k <= r.n1; k++) {
    if (h.op[k] == '=') continue;
    if (!first) *d++ = ',';
    d = put_s(d, node_v(h, k));
    first = false;
  }
  return d;
}

// Number of 'N' in hap[a, b) from n sorted runs [rs[r], re[r]) (e.g. staged in LDS), capped at 3.
__device__ __forceinline__ int count_N_runs(const int64_t *rs, const int64_t *re, int64_t n, int64_t a, int64_t b) {
  if (n == 0 || b <= a) return 0;
  int64_t lo = 0, hi = n;   // first run with end > a
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (re[mid] <= a) lo = mid + 1; else hi = mid;
  }
  int64_t c = 0;
  for (int64_t r = lo; r < n && rs[r] < b && c <= 2; r++) {
    const int64_t s = rs[r] > a ? rs[r] : a, e = re[r] < b ? re[r] : b;
    if (e > s) c += e - s;
  }
  return (int)(c > 3 ? 3 : c);
}

// Number of 'N' in hap[a, b), capped at 3 (the filter only needs > 2).
__device__ __forceinline__ int count_N(const HapView &h, int64_t a, int64_t b) {
  if (h.n_runs == 0 || b <= a) return 0;
  int64_t r = upper_bound(h.nre, h.n_runs, a);   // first run with end > a
  int64_t c = 0;
  for (; r < h.n_runs && h.nrs[r] < b && c <= 2; r++) {
    int64_t s = h.nrs[r] > a ? h.nrs[r] : a, e = h.nre[r] < b ? h.nre[r] : b;
    if (e > s) c += e - s;
  }
  return (int)(c > 3 ? 3 : c);
}

struct Rec {
  int32_t keep, len1, len2, rest;   // rest: length of the reads part of the qname (formatted into the slot)
  int32_t n0[2], n1[2];             // start / end node per mate (pass 2 skips the searches)
};

struct E3 {
  int64_t kept, b1, b2;
  __device__ E3 operator+(const E3 &o) const { return E3{kept + o.kept, b1 + o.b1, b2 + o.b2}; }
};

// Sum of digits(c) for c = 1..K  ((K+1)*nd - (10^nd - 1)/9, nd = digits(K)).
__device__ __forceinline__ int64_t digit_sum(int64_t K) {
  if (K <= 0) return 0;
  int nd = ndig_u((uint64_t)K);
  int64_t rep = 0;
  for (int i = 0; i < nd; i++) rep = rep * 10 + 1;
  return (K + 1) * nd - rep;
}

struct QFixed {
  const char *prefix;   // "@{stub}:"
  const char *mid;      // "|{chrom}|{cpy}"
  int32_t prefix_len, mid_len;
};

constexpr int MS_RUNS = 128;  // N runs staged in LDS by k_emit_measure (more: searched in global memory)

// Six consecutive nodes from k0 (clamped to the last node) in registers: with the start node of mate 0 known (the
// sampling side's packed index), both mates' start and end nodes and their qname parts usually come from these six
// (96 bytes, one random access) — mate 1 starts tl - rlen bases after mate 0, a few hundred bases.  (Round 5 loaded
// three nodes per mate after a bucket search each: 237 -> 222 us per chr1-size unit alone.)
struct Nodes6 {
  Node16 v0, v1, v2, v3, v4, v5;
  int64_t k0;
  __device__ __forceinline__ Node16 at(const HapView &h, int64_t k) const {
    const int64_t d = k - k0;
    if (d < 0 || d > 5) return h.nd[k];
    Node16 o;   // (field by field: a select of whole structs would go through scratch memory)
    o.a = d == 0 ? v0.a : d == 1 ? v1.a : d == 2 ? v2.a : d == 3 ? v3.a : d == 4 ? v4.a : v5.a;
    o.b = d == 0 ? v0.b : d == 1 ? v1.b : d == 2 ? v2.b : d == 3 ? v3.b : d == 4 ? v4.b : v5.b;
    return o;
  }
  // searchsorted(keys, x, 'right') - 1 from node k (key_k <= x)
  __device__ __forceinline__ int64_t walk(const HapView &h, int64_t k, int64_t x) const {
    while (k + 1 < h.n_nodes && at(h, k + 1).key() <= x) k++;
    return k;
  }
};
__device__ __forceinline__ Nodes6 nodes6(const HapView &h, int64_t k0) {
  const int64_t last = h.n_nodes - 1;
  auto c = [&](int64_t d) { return h.nd[k0 + d < last ? k0 + d : last]; };
  return Nodes6{c(0), c(1), c(2), c(3), c(4), c(5), k0};
}
__device__ __forceinline__ int32_t read_part_len6(const HapView &h, const Nodes6 &q, int64_t n0, int64_t n1,
                                                  bool special, int64_t pos, int64_t p, int64_t rlen) {
  int32_t L = 3 + ndig_s(pos) + 1 + ndig_s(rlen) + 1 + 1;
  if (special) L += 1 + ndig_s(p - q.at(h, n0).ps()) + 1 + ndig_s(rlen) + 1;
  int32_t nv = 0;
  for (int64_t k = n0; k <= n1; k++) {
    const Node16 n = q.at(h, k);
    if (!special) L += ndig_s(node_count(n, p, rlen)) + 1;
    if (n.code() != 0) {
      L += ndig_s(node_v(n)) + (nv ? 1 : 0);
      nv++;
    }
  }
  return L;
}

// One thread per template: start/end node of both mates, POS, the N filter (readgenerate.py:201-204), the qname
// reads part's length (not its text: the writer formats it) and the record lengths without the cnt digits, into
// Rec; per 32-template tile the sums (kept, bytes file 1, bytes file 2) into tsum (null: none); the longest record
// (+20) and the longest reads part + '\n' as maxima (one atomic per wave).  n0a (null: none): mate 0's start node per
// template from the sampling side (StoreCompact), checked against its nodes before use — then one random access of
// six nodes serves both mates (Nodes6) instead of two bucket searches and two three-node loads (222 -> ... us per
// chr1-size unit alone, round 6).
__global__ void __launch_bounds__(256) k_emit_measure(HapView h, int64_t m, const int64_t *pos0, const int64_t *pos1,
                                                      const int8_t *fo0, int64_t rlen, QFixed q, int32_t corrupt,
                                                      Rec *recs, int4 *tsum, int32_t *max_rec, const int32_t *n0a) {
  __shared__ int64_t s_rs[MS_RUNS], s_re[MS_RUNS];   // the N runs, when they fit
  const bool runs_lds = h.n_runs <= MS_RUNS;
  if (runs_lds)
    for (int i = threadIdx.x; i < h.n_runs; i += 256) {
      s_rs[i] = h.nrs[i];
      s_re[i] = h.nre[i];
    }
  __syncthreads();
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int32_t local_max = 0;
  int32_t nbytes = 0;
  int32_t sk = 0, s1 = 0, s2 = 0;   // this template's share of the tile sums
  if (t < m) {
    ReadInfo r[2];
    const int64_t p[2] = {pos0[t], pos1[t]};
    const int f0 = fo0[t];   // file f holds mate (f == fo0 ? 0 : 1)
    // rpc.get_begin_end_nodes (rpc.py:119-130): mate 0's start node from the sampling side's index when it checks
    // out (searchsorted - 1: key <= p0 < next key), else by the bucketed search; six nodes from there in registers;
    // mate 1 (p1 >= p0 for every sampled template) walks on from mate 0's start node
    int64_t a0 = n0a ? (int64_t)n0a[t] : -1;
    Nodes6 q6;
    bool ok = false;
    if (a0 >= 0 && a0 < h.n_nodes) {
      q6 = nodes6(h, a0);
      ok = q6.v0.key() <= p[0] && (a0 + 1 >= h.n_nodes || q6.v1.key() > p[0]);
    }
    if (!ok) {
      a0 = node_upper(h, p[0]) - 1;
      q6 = nodes6(h, a0);
    }
    r[0].n0 = a0;
    r[0].n1 = q6.walk(h, a0, p[0] + rlen - 1);
    r[1].n0 = p[1] >= p[0] ? q6.walk(h, a0, p[1]) : node_upper(h, p[1]) - 1;
    r[1].n1 = q6.walk(h, r[1].n0, p[1] + rlen - 1);
    read_place(h, q6.at(h, r[0].n0), p[0], rlen, r[0]);
    read_place(h, q6.at(h, r[1].n0), p[1], rlen, r[1]);
    int keep;
    if (runs_lds) {
      keep = count_N_runs(s_rs, s_re, h.n_runs, r[0].hap_a, r[0].hap_a + r[0].seq_len) <= 2 &&
             count_N_runs(s_rs, s_re, h.n_runs, r[1].hap_a, r[1].hap_a + r[1].seq_len) <= 2;
    } else {
      keep = count_N(h, r[0].hap_a, r[0].hap_a + r[0].seq_len) <= 2 &&
             count_N(h, r[1].hap_a, r[1].hap_a + r[1].seq_len) <= 2;
    }
    Rec out{0, 0, 0, 0, {(int32_t)r[0].n0, (int32_t)r[1].n0}, {(int32_t)r[0].n1, (int32_t)r[1].n1}};
    if (keep) {
      const int32_t l0 = read_part_len6(h, q6, r[0].n0, r[0].n1, r[0].special, r[0].pos, p[0], rlen);
      const int32_t l1 = read_part_len6(h, q6, r[1].n0, r[1].n1, r[1].special, r[1].pos, p[1], rlen);
      const int32_t rest = l0 + l1;
      const int32_t ql = q.prefix_len + q.mid_len + rest;
      const int32_t s_f1 = f0 == 0 ? r[0].seq_len : r[1].seq_len;
      const int32_t s_f2 = f0 == 0 ? r[1].seq_len : r[0].seq_len;
      const int32_t q1 = corrupt ? s_f1 : (int32_t)rlen, q2 = corrupt ? s_f2 : (int32_t)rlen;
      out.keep = 1 | ((f0 == 0 ? l0 : l1) << 1);   // kept; the first read's part length (where the second starts)
      out.len1 = ql + 1 + s_f1 + 3 + q1 + 1;
      out.len2 = ql + 1 + s_f2 + 3 + q2 + 1;
      out.rest = rest;
      local_max = (out.len1 > out.len2 ? out.len1 : out.len2) + 20;
      nbytes = rest + 1;
      sk = 1;
      s1 = out.len1;
      s2 = out.len2;
    }
    recs[t] = out;
  }
  if (tsum != nullptr) {   // the tile = the 32 lanes of a wave half
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) {
      sk += __shfl_xor(sk, d, 64);
      s1 += __shfl_xor(s1, d, 64);
      s2 += __shfl_xor(s2, d, 64);
    }
    if ((threadIdx.x & 31) == 0 && t < m) tsum[t >> 5] = make_int4(sk, s1, s2, 0);
  }
  int32_t local_slot = nbytes;
  for (int d = 32; d >= 1; d >>= 1) {   // one atomic per wave
    int32_t o = __shfl_xor(local_max, d, 64);
    local_max = o > local_max ? o : local_max;
    o = __shfl_xor(local_slot, d, 64);
    local_slot = o > local_slot ? o : local_slot;
  }
  // one lane per wave, and only when the (possibly stale) current maximum is lower: same-address atomics from every
  // wave of the launch serialize at the memory side
  if ((threadIdx.x & 63) == 0) {
    if (local_max > 0 && local_max > __builtin_nontemporal_load(max_rec)) atomicMax(max_rec, local_max);
    if (local_slot > 0 && local_slot > __builtin_nontemporal_load(max_rec + 3)) atomicMax(max_rec + 3, local_slot);
  }
}

struct LoadRec {
  const Rec *recs; int64_t m;
  __device__ E3 operator()(int64_t t) const {
    if (t >= m) return E3{0, 0, 0};
    const Rec &r = recs[t];
    return r.keep ? E3{1, r.len1, r.len2} : E3{0, 0, 0};
  }
};
struct StoreOff {
  E3 *off;
  int64_t base;   // templates kept before this slice; cnt of the slice's k-th kept template = base + k + 1
  __device__ void operator()(int64_t t, E3, E3 excl) const {
    int64_t ds = digit_sum(base + excl.kept) - digit_sum(base);
    off[t] = E3{base + excl.kept, excl.b1 + ds, excl.b2 + ds};
  }
};

struct LoadKeep {   // N filter only (readgenerate.py:201-204), for mh_count_kept
  HapView h; const int64_t *pos0, *pos1; int64_t m, rlen;
  __device__ int64_t operator()(int64_t t) const {
    if (t >= m) return 0;
    ReadInfo r[2];
    read_info(h, pos0[t], rlen, r[0]);
    read_info(h, pos1[t], rlen, r[1]);
    return count_N(h, r[0].hap_a, r[0].hap_a + r[0].seq_len) <= 2 &&
           count_N(h, r[1].hap_a, r[1].hap_a + r[1].seq_len) <= 2;
  }
};

constexpr int EW_T = 32;        // templates per workgroup
constexpr int EW_THREADS = 256;
constexpr int EW_WAVES = EW_THREADS / 64;

struct TplMeta {
  int32_t loc[2];       // record offset inside each LDS image
  int32_t qlen;         // qname length (with cnt)
  int32_t keep;         // bit 0: kept; bit 1: fo0 (file 0 holds mate fo0)
  int32_t seq_len[2];   // per mate
  int32_t win[2];       // per mate: offset of the first read base inside the LDS window buffer
};

__device__ __forceinline__ uint8_t comp(uint8_t c) {
  // str.maketrans('ATCGN', 'TAGCN'): everything else passes through
  return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
}

// LDS: meta[EW_T] | windows[EW_T][2][win_stride] | image 0 [cap+16] | image 1 [cap+16]
__global__ void __launch_bounds__(EW_THREADS) k_emit_write(HapView h, int64_t m, const int64_t *pos0,
                                                           const int64_t *pos1, const int8_t *fo0, int64_t rlen,
                                                           QFixed q, const Rec *recs, const E3 *off, char *out1,
                                                           char *out2, int write2, int32_t cap, int32_t win_stride,
                                                           int32_t corrupt, int32_t *err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TplMeta *meta = (TplMeta *)smem;
  uint8_t *wins = (uint8_t *)smem + ((sizeof(TplMeta) * EW_T + 15) / 16) * 16;
  char *img[2];
  img[0] = (char *)wins + (size_t)EW_T * 2 * win_stride;
  img[1] = img[0] + cap + 16;
  __shared__ int64_t s_sb_end;

  const int64_t t0 = (int64_t)blockIdx.x * EW_T;
  const int64_t t1 = t0 + EW_T < m ? t0 + EW_T : m;
  const int nfile = write2 ? 2 : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunks = win_stride / 16;      // 16-byte gathers per mate window

  int64_t sb = t0;
  while (sb < t1) {
    // ---- sub-batch [sb, sb_end): the largest prefix whose images fit `cap` bytes (normally the whole tile) --
    {
      int64_t t = sb + 1 + threadIdx.x;
      int fits = 0;
      if (threadIdx.x < EW_T && t <= t1) {
        E3 a = off[sb], b = off[t];
        fits = (b.b1 - a.b1 <= cap) && (!write2 || b.b2 - a.b2 <= cap);
      }
      int cnt = __syncthreads_count(fits);
      if (threadIdx.x == 0) s_sb_end = sb + cnt;
      __syncthreads();
    }
    const int64_t sb_end = s_sb_end;
    if (sb_end == sb) {   // one record larger than the image (host sizes cap from the measured maximum)
      if (threadIdx.x == 0) atomicOr(err, 1);
      return;
    }
    const int nb = (int)(sb_end - sb);
    const E3 base = off[sb];
    const int64_t g0[2] = {base.b1, base.b2};
    const int al[2] = {(int)(g0[0] & 15), (int)(g0[1] & 15)};

    // ---- B0: gather both mates' haplotype windows of every template into LDS (all loads in flight) --------
    for (int it = threadIdx.x; it < nb * 2 * chunks; it += EW_THREADS) {
      const int j = it / (2 * chunks), rem = it - j * 2 * chunks, s = rem / chunks, c = rem - s * chunks;
      const int64_t t = sb + j;
      const int64_t p = s ? pos1[t] : pos0[t];
      int64_t a = p - h.p_min;
      if (a > h.hap_len) a = h.hap_len;
      const int64_t a16 = a & ~(int64_t)15;
      if (a16 + 16 * c < a + rlen && recs[t].keep) {
        uint4 v = *(const uint4 *)(h.hap + a16 + 16 * c);
        *(uint4 *)(wins + (size_t)(j * 2 + s) * win_stride + 16 * c) = v;
      }
    }

    // ---- A: owner threads format the qname into image 0 and record metadata ------------------------------
    if (threadIdx.x < nb) {
      const int64_t t = sb + threadIdx.x;
      TplMeta &mt = meta[threadIdx.x];
      const Rec rc = recs[t];
      mt.keep = rc.keep;
      if (rc.keep) {
        ReadInfo r[2];
        const int64_t p[2] = {pos0[t], pos1[t]};
        for (int s = 0; s < 2; s++) {
          r[s].n0 = rc.n0[s];
          r[s].n1 = rc.n1[s];
          read_place(h, h.nd[r[s].n0], p[s], rlen, r[s]);
          mt.seq_len[s] = r[s].seq_len;
          mt.win[s] = (threadIdx.x * 2 + s) * win_stride + (int)(r[s].hap_a & 15);
        }
        const E3 o = off[t];
        const int f0 = fo0[t];
        mt.loc[0] = (int)(o.b1 - g0[0]) + al[0];
        mt.loc[1] = (int)(o.b2 - g0[1]) + al[1];
        char *d = img[0] + mt.loc[0];
        char *d0 = d;
        d = put_str(d, q.prefix, q.prefix_len);
        d = put_s(d, o.kept + 1);
        d = put_str(d, q.mid, q.mid_len);
        for (int fr = 0; fr < 2; fr++) {              // reads in file order: reads[fo] = mate s
          const int s = fr == f0 ? 0 : 1;
          *d++ = '|'; *d++ = (char)('0' + s);
          *d++ = '|'; d = put_s(d, r[s].pos);
          *d++ = '|'; d = put_s(d, rlen);
          *d++ = '|'; d = write_cigar(d, h, p[s], rlen, r[s]);
          *d++ = '|'; d = write_vlist(d, h, r[s]);
        }
        mt.qlen = (int32_t)(d - d0);
        mt.keep = 1 | (f0 << 1);
      }
    }
    __syncthreads();

    // ---- B1: one wave per (template, file): qname copy (file 2), bases, separators, qualities -------------
    for (int pair = wave; pair < nb * nfile; pair += EW_WAVES) {
      const int j = pair / nfile, f = pair - j * nfile;
      const TplMeta &mt = meta[j];
      if (!(mt.keep & 1)) continue;
      const int f0 = mt.keep >> 1;
      const int s = f == f0 ? 0 : 1;                  // mate held by file f
      const int S = mt.seq_len[s];
      const int Q = corrupt ? S : (int)rlen;          // corrupt_single_read emits len(seq) qualities
      char *d0 = img[f] + mt.loc[f];
      if (f == 1)
        for (int i = lane; i < mt.qlen; i += 64) d0[i] = img[0][mt.loc[0] + i];
      char *d = d0 + mt.qlen;                         // '\n' seq '\n+\n' qual '\n'
      const uint8_t *w = wins + mt.win[s];
      for (int n = lane; n < S; n += 64) d[1 + n] = (char)(s ? comp(w[S - 1 - n]) : w[n]);
      for (int n = lane; n < Q; n += 64) d[4 + S + n] = '~';
      if (lane == 0) {
        d[0] = '\n';
        d[1 + S] = '\n';
        d[2 + S] = '+';
        d[3 + S] = '\n';
        d[4 + S + Q] = '\n';
      }
    }
    __syncthreads();

    // ---- C: images -> file arenas (16-byte aligned stores; byte stores at the ragged edges) --------------
    {
      const E3 endo = off[sb_end];
      const int64_t g1[2] = {endo.b1, endo.b2};
      for (int f = 0; f < nfile; f++) {
        const int64_t G0 = g0[f], G1 = g1[f];
        if (G1 <= G0) continue;
        char *out = f ? out2 : out1;
        const char *im = img[f] + al[f];   // im[g - G0] is global byte g
        int64_t A0 = (G0 + 15) & ~(int64_t)15, A1 = G1 & ~(int64_t)15;
        if (A0 > G1) A0 = G1;
        if (A1 < A0) A1 = A0;
        for (int64_t g = G0 + threadIdx.x; g < A0; g += EW_THREADS) out[g] = im[g - G0];
        const int64_t nvec = (A1 - A0) >> 4;
        for (int64_t v = threadIdx.x; v < nvec; v += EW_THREADS) {
          const int64_t g = A0 + (v << 4);
          *(uint4 *)(out + g) = *(const uint4 *)(im + (g - G0));
        }
        for (int64_t g = A1 + threadIdx.x; g < G1; g += EW_THREADS) out[g] = im[g - G0];
      }
    }
    __syncthreads();
    sb = sb_end;
  }
}

// ---- direct writer -------------------------------------------------------------------------------------------
// The default emission kernel.  k_emit_measure has recorded per template its start/end nodes, keep flag and record
// lengths (without the cnt digits) and per 32-template tile the sums (kept, bytes per file); a small scan over the
// tiles gives each tile's prefix (k_tile_scan).  Per tile, every FASTQ record is three byte strings held in LDS:
//   Q  the qname line: head ('@stub:' cnt '|chrom|cpy') + the reads part ('|strand|POS|rlen|CIGAR|v,..' per read,
//      formatted here from the template's nodes) and '\n';
//   B  the bases: the haplotype window of the file's mate, gathered in 16-byte chunks (mate 1 from the reverse-
//      complement haplotype, so B reads forward in both cases);
//   T  '\n+\n' + rlen '~' + '\n', one copy per workgroup (identical for every perfect read).
// Phase 1: waves 1-3 issue all gathers of the tile; wave 0 (lane = read) formats the qname parts, scans the tile's
// record lengths, numbers the kept templates (cnt = cnt_base + kept before + 1, readgenerate.py:209) and adds the cnt
// digits in closed form (digit_sum); owner lanes write the metadata and the qname heads.  One barrier.  Phase 2
// writes the tile's bytes as aligned 16-byte stores straight to the arenas, in two sweeps:
//   pure  chunks inside one string of one record: one unaligned 16-byte LDS read (v_alignbyte) and one store;
//   seam  the (at most four) chunks per record that straddle strings or records — record start (previous record's
//         T end + Q), Q|B, B|T, and the tile's ragged end — merged per dword with byte masks (v_bfi); the tile's
//         first and last chunks are byte stores of the tile's own bytes (the neighbouring tiles own the rest).
// With corruption the records carry len(seq) placeholder qualities and the writer also leaves each record's
// first-base offset for k_cr_inplace.
constexpr int ED_T = 32;
constexpr int ED_THREADS = 256;
constexpr int ED_PAD = 32;   // LDS padding around every string (unaligned reads of masked-out bytes stay in range)
constexpr int ED_CRB = 15;   // bases per corruption block (CI_BLK)
constexpr int ED_GMAX = 7;   // window chunks per gather thread (3 threads per mate): up to 21 chunks, rlen <= 321

// EW_PROF (calibration builds only: make prof): per-phase shader-clock sums of k_emit_tiles' waves (lane 0), read
// back by mh_ew_prof (scripts/calib_writer_phases.py).  Slots: 0 wave 0's formatting, 1 waves 1-3's gathers (sum of
// the three), 2 / 3 their waits at the barrier, 4 the corruption rows' layering (all waves), 5 the seam sweep (with
// its barrier), 6 the chunk sweep; 7 tiles.
#ifdef EW_PROF
__device__ unsigned long long ew_prof[16];
struct EwProf {
  uint64_t t, a[8];
  __device__ void mark(int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    a[i] += now - t;
    t = now;
  }
};
#define EWP_PARAM , EwProf &P_
#define EWP_ARG , P_
#define EWP_BEGIN                                 \
  EwProf P_;                                      \
  for (int i_ = 0; i_ < 8; i_++) P_.a[i_] = 0;    \
  P_.t = __builtin_amdgcn_s_memtime()
#define EWP(i) P_.mark(i)
#define EWP_END                                                                          \
  if ((threadIdx.x & 63) == 0) {                                                         \
    if (threadIdx.x == 0) P_.a[7] = 1;                                                   \
    for (int i_ = 0; i_ < 8; i_++) atomicAdd(&ew_prof[i_], (unsigned long long)P_.a[i_]); \
  }
#else
#define EWP_PARAM
#define EWP_ARG
#define EWP_BEGIN
#define EWP(i)
#define EWP_END
#endif

struct DMeta {
  int32_t rel[2];    // record start relative to the tile's first byte, per file
  int32_t len[2];    // record length per file (0: template dropped by the N filter)
  int32_t qb;        // LDS offset of Q (qname '@' ... '\n')
  int32_t sb;        // Q length = offset of the first base
  int32_t bb[2];     // LDS offset of B per file (forward order)
  int32_t S[2];      // bases per file
  int32_t tb[2];     // LDS offset of the record's T (the shared one)
  int32_t tn[2];     // T length: rlen + 4, or S + 4 with corruption (qualities = len(seq))
};

// 16 bytes at an arbitrary byte offset of the dynamic LDS block: one ds_read_b128 (gfx950 reads LDS unaligned; was
// five aligned dword reads + v_alignbyte).  (Offsets, not pointers: an integer round trip of an LDS pointer turns
// its reads into flat loads.)
__device__ __forceinline__ uint4 lds_load16(const char *lds, uint32_t off) {
  uint4 v;
  __builtin_memcpy(&v, lds + off, 16);
  return v;
}
// bytes i (0..3) of a dword whose byte i sits at offset x0 + i, with x0 + i < n
__device__ __forceinline__ uint32_t lt_mask(int32_t x0, int32_t n) {
  int32_t k = n - x0;
  k = k < 0 ? 0 : (k > 4 ? 4 : k);
  return (uint32_t)((1ull << (8 * k)) - 1ull);
}

__device__ __forceinline__ uint32_t u4get(const uint4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// qname head constants by value (kernel arguments: uniform indexing reads them through the scalar cache)
struct QHead {
  uint32_t w[24];    // prefix ('@stub:') then mid ('|chrom|cpy'), packed little-endian
  int32_t lp, lm;
  __device__ __forceinline__ uint8_t at(int i) const { return (uint8_t)(w[i >> 2] >> (8 * (i & 3))); }
};

// the 16 bytes at record offsets x0 .. x0+15 of record (j, f) — previous record's T end | Q | B | T — merged per dword
// with byte masks (v_bfi)
template <int CR>
__device__ __forceinline__ uint4 seam_chunk(const char *smem, const DMeta *meta, int j, int f, int32_t x0,
                                            int32_t o_t, int32_t TL) {
  const DMeta &M = meta[j];
  const int32_t rel = M.rel[f], sb = M.sb, S = M.S[f], tl = sb + S, qb = M.qb, bb = M.bb[f], tb = M.tb[f],
                tn = M.tn[f];
  int32_t pte = o_t + TL;                                   // end of the previous record's T
  if (CR && x0 < 0 && rel > 0)                              // the previous kept record of this file in the tile
    for (int pj = j - 1; pj >= 0; pj--)
      if (meta[pj].len[f] > 0) {
        pte = meta[pj].tb[f] + meta[pj].tn[f];
        break;
      }
  const uint4 vp = lds_load16(smem, (uint32_t)(pte + (x0 < 0 ? x0 : -16)));
  const uint4 vq = lds_load16(smem, (uint32_t)(qb + (x0 < -16 ? -16 : (x0 > sb ? sb : x0))));
  int32_t yb = x0 - sb;
  yb = yb < -16 ? -16 : (yb > S ? S : yb);
  const uint4 vb = lds_load16(smem, (uint32_t)(bb + yb));
  int32_t yt = x0 - tl;
  yt = yt < -16 ? -16 : (yt > tn ? tn : yt);
  const uint4 vt = lds_load16(smem, (uint32_t)(tb + yt));
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int32_t x = x0 + 4 * k;
    const uint32_t mb = lt_mask(x, tl), mq = lt_mask(x, sb), mp = lt_mask(x, 0);
    uint32_t v = (u4get(vb, k) & mb) | (u4get(vt, k) & ~mb);
    v = (u4get(vq, k) & mq) | (v & ~mq);
    w[k] = (u4get(vp, k) & mp) | (v & ~mp);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// The output sweeps of a 32-template tile whose strings and metadata are in LDS: LPR lanes per record (record
// r = file f, template j), passes over the tile's NF * ED_T records.  gbase: arena offset of the tile's first byte per
// file; span: the tile's bytes per file.
template <int NF, int LPR, int CR>
__device__ __forceinline__ void ed_output(const DMeta *meta, int nt, const int64_t gbase[2], const int32_t span[2],
                                          int32_t o_t, int32_t TL, int32_t o_s, bool staged, char *const *arena
                                          EWP_PARAM) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  constexpr int RPP = ED_THREADS / LPR;                        // records per pass
  const int q = tid % LPR;
  // seams (record-relative): 0 = record start (previous record's T end | Q), sb = Q|B, tl = B|T, L = the tile's
  // ragged end (a record end inside the tile is the next record's start seam); a chunk holding several seams
  // belongs to the first of them.  Lane q < 4 of a record computes seam q into LDS (the tile's ragged edges go
  // straight out as byte stores).
  for (int r = tid / LPR; r < NF * ED_T; r += RPP) {
    const int f = NF == 2 ? r / ED_T : 0, j = r % ED_T;
    if (j >= nt || q >= 4) continue;
    const DMeta &M = meta[j];
    const int32_t L = M.len[f];
    if (L == 0) continue;
    const int32_t rel = M.rel[f];
    const int64_t ga = gbase[f] + rel;                        // arena offset of the record's first byte
    const int32_t sb = M.sb, S = M.S[f], tl = sb + S;
    const int b = q;
    const bool tile_end = rel + L == span[f];
    const int32_t spb = b == 0 ? 0 : b == 1 ? sb : b == 2 ? tl : L;
    const int64_t cg = (ga + spb) >> 4;
    bool skip = (b == 3 && !tile_end) || ((ga + spb) & 15) == 0;   // aligned: both sides are pure chunks
    skip |= b > 0 && (ga & 15) != 0 && (ga >> 4) == cg;
    skip |= b > 1 && ((ga + sb) & 15) != 0 && ((ga + sb) >> 4) == cg;
    skip |= b > 2 && ((ga + tl) & 15) != 0 && ((ga + tl) >> 4) == cg;
    if (skip) continue;
    const int32_t x0 = (int32_t)((cg << 4) - ga);
    const int32_t lo = (rel == 0 && x0 < 0) ? -x0 : 0;        // tile start: the previous tile owns the rest
    const int32_t hi = b == 3 ? L - x0 : 16;                    // tile end: the next tile owns the rest
    const uint4 wv = seam_chunk<CR>(smem, meta, j, f, x0, o_t, TL);
    if (lo == 0 && hi == 16) {
      if (staged) *(uint4 *)(smem + o_s + (r * 4 + b) * 16) = wv;
      else *(uint4 *)(arena[f] + (cg << 4)) = wv;
    } else {
      const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
      char *g = arena[f] + (cg << 4);
      for (int k = lo; k < hi; k++) g[k] = (char)(w[k >> 2] >> (8 * (k & 3)));
    }
  }
  // (an LDS-only barrier here — the ragged-edge byte stores above need not land before the chunk sweep — measured no
  // faster than the full one, round 3; merging the seam chunks in the chunk sweep instead of staging them, with no
  // second barrier and 4 KB less LDS, measured 1.5 % slower on the WGS line, round 4)
  if (staged) __syncthreads();
  EWP(5);
  // every full chunk of each record: one unaligned LDS read (or a seam) and one aligned 16-byte store
  for (int r = tid / LPR; r < NF * ED_T; r += RPP) {
    const int f = NF == 2 ? r / ED_T : 0, j = r % ED_T;
    if (j >= nt) continue;
    const DMeta &M = meta[j];
    const int32_t L = M.len[f];
    const int32_t rel = M.rel[f];
    const int64_t ga = gbase[f] + rel;
    const int32_t sb = M.sb, tl = sb + M.S[f], qb = M.qb, bb = M.bb[f], tb = M.tb[f];
    char *const out = arena[f];
    const int64_t c0 = ga >> 4;
    int32_t x0 = (int32_t)((c0 << 4) - ga) + 16 * q;
    for (int64_t cg = c0 + q; x0 + 16 <= L; cg += LPR, x0 += 16 * LPR) {
      const int b = x0 < 0 ? 0 : (x0 < sb && x0 + 16 > sb) ? 1 : (x0 < tl && x0 + 16 > tl) ? 2 : -1;
      if (b == 0 && rel == 0) continue;                         // ragged tile start, already written
      uint4 v;
      if (b >= 0 && !staged) continue;                          // seam chunk, stored by the seam pass
      if (CR < 2 && b < 0 && x0 >= tl + 3 && x0 + 16 <= tl + TL - 1) {
        v = make_uint4(0x7e7e7e7eu, 0x7e7e7e7eu, 0x7e7e7e7eu, 0x7e7e7e7eu);   // inside T's '~' run: no LDS read
      } else {
        const int32_t src = b >= 0 ? o_s + (r * 4 + b) * 16
                                   : (x0 + 16 <= sb ? qb + x0 : (x0 + 16 <= tl ? bb + (x0 - sb) : tb + (x0 - tl)));
        v = lds_load16(smem, (uint32_t)src);
      }
      *(uint4 *)(out + (cg << 4)) = v;
    }
  }
  EWP(6);
}

__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
  int total;
  return wave_sum_incl(v, total);
}

// tile sums of k_emit_measure -> tile prefixes (kept, bytes per file without the cnt digits)
struct LoadTile {
  const int4 *ts; int64_t n;
  __device__ E3 operator()(int64_t i) const {
    if (i >= n) return E3{0, 0, 0};
    const int4 v = ts[i];
    return E3{v.x, v.y, v.z};
  }
};
struct StoreTile {
  E3 *pre;
  __device__ void operator()(int64_t i, E3, E3 excl) const { pre[i] = excl; }
};

struct TArgs {
  HapView h;
  int64_t m;
  const int64_t *pos0, *pos1;
  const int8_t *fo0;
  const Rec *recs;          // k_emit_measure's records
  const E3 *tpre;           // per tile: kept templates and record bytes (no cnt digits) before it
  char *arena[2];
  int64_t used[2];          // arena offset of the emission's first byte per file
  int64_t cnt_base;         // templates kept before the emission's first one (cnt numbering)
  uint2 *crec;              // corruption: per record the first base's arena offset and S (k_cr_inplace's words)
  int32_t rlen, win_stride, head, qstride;
  const uint4 *crow;        // corruption rows (CR 2, k_cr_rows): per block of 15 bases its qualities + 33, and
  const uint32_t *ccode;    //   its 2-bit substitution codes; slot (file * nb + block) * m + template
  int32_t nb;               // blocks per record row
  // the single-pass writer (k_emit_fused): no measure pass, its tiles' prefixes by a decoupled look-back
  uint64_t *lb;             // look-back scratch: ticket word (64 B), then 3 aggregate and 3 inclusive words per tile
  int64_t ntiles;
  uint32_t tbase, epoch;    // the ticket counter's value at launch; this launch's epoch (mh_scan.h lb_reserve)
  uint32_t *fault;          // the context's fault word: 1 look-back timeout, 2 qname row overflow, 4 arena overflow
  const int64_t *cur_in;    // arena ends after the previous unit of the chain (null: used[])
  int64_t *cur_out;         // after this unit: kept, end of file 1, end of file 2 (device cursor; the last tile)
  int64_t *res;             // kept, bytes 1, bytes 2, end 1, end 2 (mapped host memory; the last tile)
  int64_t cap[2];           // arena capacities (bytes)
  int32_t hcap;             // qname row room for the reads part and its '\n'
};

// CR: the corrupt layout — len(seq) qualities per record (illumina.corrupt_single_read, illumina.py:140-162): T is
// read from the shared string for S + 4 bytes, whose last one k_cr_inplace turns into the '\n' (and the
// placeholders into qualities) when it corrupts the record.
__device__ __forceinline__ uint32_t lds_put_u(char *lds, uint32_t o, uint64_t v) {
  if (v > 0xffffffffull) {
    auto put = [&](uint8_t c) { lds[o++] = (char)c; };
    put_big(v);
    return o;
  }
  uint32_t x = (uint32_t)v;
  const int nd = ndig_u(x);
  for (int i = nd - 1; i >= 0; i--) {
    lds[o + i] = (char)('0' + x % 10u);
    x /= 10u;
  }
  return o + nd;
}
__device__ __forceinline__ uint32_t lds_put_s(char *lds, uint32_t o, int64_t v) {
  if (v < 0) {
    lds[o] = '-';
    return lds_put_u(lds, o + 1, (uint64_t)(-v));
  }
  return lds_put_u(lds, o, (uint64_t)v);
}

#define NODE_AT(k)                                                                                       \
  Node16 n;                                                                                              \
  {                                                                                                      \
    const int64_t i_ = (k) - n0;                                                                         \
    if (i_ > 3) {                                                                                        \
      const uint64_t *g_ = (const uint64_t *)(h.nd + (k));                                               \
      n.a = g_[0];                                                                                       \
      n.b = g_[1];                                                                                       \
    } else {                                                                                             \
      n.a = i_ == 0 ? q0.a : i_ == 1 ? q1.a : i_ == 2 ? q2.a : q3.a;                                     \
      n.b = i_ == 0 ? q0.b : i_ == 1 ? q1.b : i_ == 2 ? q2.b : q3.b;                                     \
    }                                                                                                    \
  }

// FU: the single-pass writer — wave 0 finds each read's nodes, applies the N filter and measures the records itself
// (what k_emit_measure wrote to Rec), publishes the tile's sums and takes its prefix by a decoupled look-back over
// the earlier tiles of the launch (mh_scan.h's status words), instead of reading the measure pass's records and the
// tile scan's prefixes.
template <int NF, int LPR, int CR, int GW, bool FU = false>
__device__ __forceinline__ void emit_tile(const TArgs &A, const QHead &qh, const int64_t tile) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int64_t s_g[2];      // arena offset of the tile's first byte per file
  __shared__ int32_t s_span[2];   // the tile's bytes per file
  __shared__ int32_t s_skip;      // FU: the tile's records would pass the arena's end (reported, nothing stored)
  // LDS layout (byte offsets): meta | pad | windows [ED_T][2][win_stride] | pad | qname buffers [ED_T][qstride] |
  // pad | T | pad | seam chunks [NF][ED_T][4] x 16 B | dump (16 B)
  DMeta *meta = (DMeta *)smem;
  const HapView &h = A.h;
  const int32_t win_stride = A.win_stride, qstride = A.qstride, head = A.head;
  const int32_t o_win = (int32_t)(((sizeof(DMeta) * ED_T + ED_PAD + 15) / 16) * 16);
  const int32_t o_q = o_win + ED_T * 2 * win_stride + ED_PAD;
  const int32_t o_t = o_q + ED_T * qstride + ED_PAD;
  const int32_t o_s = o_t + (A.rlen + 4 + 2 * ED_PAD + 15) / 16 * 16;
  // seam chunks through LDS (in order with the others); CR 2 stores them from the seam pass (4 KB less LDS: with the
  // per-record T strings that is 5 instead of 4 workgroups per CU, 0.77 vs 0.73 G/s on the corrupt bench)
  const bool staged = CR != 2;
  const int32_t o_dump = o_s + (staged ? NF * ED_T * 4 * 16 : 0);   // 16-byte sink for unused gathers
  const int32_t TL = A.rlen + 4;                      // T = '\n+\n' + rlen '~' + '\n' (readgenerate.py:229)
  // CR 2: per record its own T ('\n+\n' + S qualities + '\n') at o_tr + record * TS, laid from the corruption rows
  const int32_t TS = (A.rlen + 4 + 15) / 16 * 16;   // (a read 16 bytes past a T lands in the next one or the pad)
  const int32_t o_tr = o_dump + 16 + ED_PAD;
  const int tid = threadIdx.x;
  EWP_BEGIN;
  const int Lp = qh.lp, Lm = qh.lm;
  const int64_t t0 = tile * ED_T;
  const int nt = (int)(t0 + ED_T < A.m ? ED_T : A.m - t0);
  const int chunks = win_stride / 16;
  // CR 2: the tile's row slots (file f, template j, block b: slot f * ED_T * nb + j * nb + b), the first RK per thread
  // loaded before the gathers so they are in flight with them
  constexpr int RK = 3;
  const int32_t nb = CR == 2 ? A.nb : 1, nsl = NF * ED_T * nb;
  auto slot_g = [&](int32_t sl, int *sf, int *sj, int *sb_) -> int64_t {
    const int f = sl / (ED_T * nb), rem = sl - f * ED_T * nb, j = rem / nb;
    *sf = f;
    *sj = j;
    *sb_ = rem - j * nb;
    return j < nt ? ((int64_t)f * nb + (rem - j * nb)) * A.m + t0 + j : 0;
  };
  uint4 rq[RK];
  uint32_t rcw[RK];
  if (CR == 2) {
#pragma unroll
    for (int k = 0; k < RK; k++) {
      int sf, sj, sbk;
      const int32_t sl = tid + k * ED_THREADS;
      const int64_t g = sl < nsl ? slot_g(sl, &sf, &sj, &sbk) : 0;
      rq[k] = A.crow[g];
      rcw[k] = A.ccode[g];
    }
  }
  for (int i = tid; i < TL; i += ED_THREADS)
    smem[o_t + i] = (char)(i == 0 || i == 2 || i == TL - 1 ? '\n' : i == 1 ? '+' : '~');
  if (tid >= 64 * (4 - GW)) {
    // the last GW waves: the gathers (GW threads per mate window), all in flight together; an unused chunk re-reads
    // the first one
    constexpr int GM = (3 * ED_GMAX + GW - 1) / GW;
    const int g = tid - 64 * (4 - GW), pr = g / GW, q3 = g - GW * pr;
    const int jg = pr >> 1, sg = pr & 1;
    const int64_t tg = t0 + (jg < nt ? jg : 0);
    const bool kg = jg < nt;
    const int64_t pg = sg ? A.pos1[tg] : A.pos0[tg];
    int64_t ag = pg - h.p_min, eg = pg + A.rlen - h.p_min;
    if (eg > h.hap_len) eg = h.hap_len;
    if (ag > h.hap_len) ag = h.hap_len;
    const int64_t lg = eg > ag ? eg - ag : 0;
    // mate 1: a forward range of the reverse-complement haplotype
    const int64_t a2g = sg ? h.hap_len - ag - lg : ag;
    const int64_t a16 = a2g & ~(int64_t)15;
    const uint8_t *hsrc = (sg ? h.rc : h.hap) + a16;
    uint4 wv[GM];
    uint32_t use = 0;
#pragma unroll
    for (int k = 0; k < GM; k++) {
      const int c = q3 + GW * k;
      const bool u = kg && c < chunks && a16 + 16 * c < a2g + lg;
      use |= (uint32_t)u << k;
      wv[k] = *(const uint4 *)(hsrc + (u ? 16 * c : 0));
    }
    const int32_t slot = o_win + (jg * 2 + sg) * win_stride;
#pragma unroll
    for (int k = 0; k < GM; k++) {
      const int c = q3 + GW * k;
      *(uint4 *)(smem + (((use >> k) & 1) ? slot + 16 * c : o_dump)) = wv[k];
    }
  }
  if (tid < 64) {
    // wave 0: lane = read (template jf, mate s)
    const int jf = tid >> 1, s = tid & 1;
    const bool valid = jf < nt;
    const int64_t tf = t0 + (valid ? jf : 0);
    const int64_t p = s ? A.pos1[tf] : A.pos0[tf];
    const int fo = A.fo0[tf];
    const int fr = s == 0 ? fo : 1 - fo;   // the read's place in the qname = its file (reads[fo] = mate 0, :207)
    const int64_t rl = A.rlen;
    int64_t a = p - h.p_min, e = p + rl - h.p_min;   // the read's bases: hap[a, a + S)
    if (e > h.hap_len) e = h.hap_len;
    if (a > h.hap_len) a = h.hap_len;
    const int32_t S = (int32_t)(e > a ? e - a : 0);
    int64_t n0, n1;
    Node16 q0, q1, q2, q3;   // the read's nodes: the first four loaded together (a 150-bp read spans one to three)
    ReadInfo ri;
    bool keep;
    int32_t rest, flen, lw;  // both reads' qname parts; the file-1 read's part (where the other starts); record bytes
    E3 P;                    // kept templates and record bytes (no cnt digits) before the tile
    if constexpr (FU) {
      // rpc.get_begin_end_nodes (rpc.py:119-130): the start node by the bucketed search, the end node from the four
      // nodes loaded at once (further only past them)
      n0 = node_upper(h, p) - 1;
      const int64_t last = h.n_nodes - 1;
      q0 = h.nd[n0];
      q1 = h.nd[n0 + 1 < last ? n0 + 1 : last];
      q2 = h.nd[n0 + 2 < last ? n0 + 2 : last];
      q3 = h.nd[n0 + 3 < last ? n0 + 3 : last];
      const int64_t x = p + rl - 1;
      n1 = n0;
      if (n0 + 1 <= last && q1.key() <= x) {
        n1 = n0 + 1;
        if (n0 + 2 <= last && q2.key() <= x) {
          n1 = n0 + 2;
          if (n0 + 3 <= last && q3.key() <= x) n1 = node_walk(h, n0 + 3, x);
        }
      }
      ri.n0 = n0;
      ri.n1 = n1;
      read_place(h, q0, p, rl, ri);
      // the read's qname part length (readgenerate.py:223-225; k_emit_measure's read_part_len)
      int32_t L = 3 + ndig_s(ri.pos) + 1 + ndig_s(rl) + 1 + 1;
      if (ri.special) L += 1 + ndig_s(p - q0.ps()) + 1 + ndig_s(rl) + 1;
      int32_t nv = 0;
      for (int64_t k = n0; k <= n1; k++) {
        NODE_AT(k)
        if (!ri.special) L += ndig_s(node_count(n, p, rl)) + 1;
        if (n.code() != 0) {
          L += ndig_s(node_v(n)) + (nv ? 1 : 0);
          nv++;
        }
      }
      // the N filter (readgenerate.py:201-204) over both mates: the pair's two lanes exchange their verdicts and parts
      const int kr = count_N(h, a, a + S) <= 2;
      const int ko = __shfl_xor(kr, 1, 64);
      const int32_t Lo = __shfl_xor(L, 1, 64);
      keep = valid && kr && ko;
      rest = L + Lo;
      flen = fr == 0 ? L : Lo;
      lw = keep ? Lp + Lm + rest + 1 + S + 3 + (CR ? S : (int32_t)rl) + 1 : 0;
      P = E3{0, 0, 0};
    } else {
      // the measure pass's record: keep | first part length << 1, record lengths, both parts' length, nodes
      const int4 r0 = *(const int4 *)(A.recs + tf), r1 = *(const int4 *)((const char *)(A.recs + tf) + 16);
      P = A.tpre[tile];
      n0 = s ? r1.y : r1.x;
      n1 = s ? r1.w : r1.z;
      keep = valid && (r0.x & 1);
      rest = r0.w;
      flen = r0.x >> 1;
      lw = keep ? (fr == 0 ? r0.y : r0.z) : 0;
      q0 = h.nd[n0];
      q1 = h.nd[n0 + 1 <= n1 ? n0 + 1 : n0];
      q2 = h.nd[n0 + 2 <= n1 ? n0 + 2 : n0];
      q3 = h.nd[n0 + 3 <= n1 ? n0 + 3 : n0];
      ri.n0 = n0;
      ri.n1 = n1;
      if (keep) read_place(h, q0, p, rl, ri);
    }
    // this read's record (file fr) without the cnt digits; the wave's inclusive sums of (kept, bytes per file)
    const int32_t ik = wave_incl_scan(keep && fr == 0 ? 1 : 0);
    const int32_t i0 = wave_incl_scan(fr == 0 ? lw : 0);
    const int32_t i1 = wave_incl_scan(fr == 1 ? lw : 0);
    const int32_t tk = __shfl(ik, 63, 64), tb0 = __shfl(i0, 63, 64), tb1 = __shfl(i1, 63, 64);
    const int lane = tid;
    uint64_t *const lb_agg = FU ? A.lb + 8 : nullptr, *const lb_inc = FU ? lb_agg + 3 * A.ntiles : nullptr;
    if constexpr (FU) {   // the tile's sums out first: later tiles' look-backs wait for them, not for the formatting
      const int64_t tv = lane == 0 ? tk : lane == 1 ? tb0 : tb1;
      if (lane < 3) lb_put((tile == 0 ? lb_inc : lb_agg) + (size_t)lane * A.ntiles + tile, tv, tile == 0 ? 2u : 1u,
                           A.epoch);
    }
    bool fmt = keep;
    if (FU && keep && rest + 1 > A.hcap) {   // (the splice's bound was wrong: reported, the row never overrun)
      fmt = false;
      if (A.fault) __hip_atomic_fetch_or(A.fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (fmt) {
      // the read's part of the qname at its place (readgenerate.py:223-225); read 1 ends at `rest`, where the '\n' goes
      uint32_t o = (uint32_t)(o_q + jf * qstride + head);
      if (fr == 1) o += (uint32_t)flen;   // after the first read's part
      smem[o] = '|';
      smem[o + 1] = (char)('0' + s);
      smem[o + 2] = '|';
      o = lds_put_s(smem, o + 3, ri.pos);
      smem[o] = '|';
      o = lds_put_s(smem, o + 1, rl);
      smem[o++] = '|';
      if (ri.special) {
        smem[o] = '>';
        o = lds_put_s(smem, o + 1, p - q0.ps());
        smem[o] = ':';
        o = lds_put_s(smem, o + 1, rl);
        smem[o++] = 'I';
      } else {
        for (int64_t k = n0; k <= n1; k++) {
          NODE_AT(k)
          o = lds_put_s(smem, o, node_count(n, p, rl));
          smem[o++] = (char)n.op();
        }
      }
      smem[o++] = '|';
      bool first = true;
      for (int64_t k = n0; k <= n1; k++) {
        NODE_AT(k)
        if (n.code() == 0) continue;
        if (!first) smem[o++] = ',';
        o = lds_put_s(smem, o, node_v(n));
        first = false;
      }
      if (fr == 1) smem[o] = '\n';
    }
    int64_t u0 = A.used[0], u1 = A.used[1];   // arena offsets of the emission's first byte
    if constexpr (FU) {
      // the look-back (mh_scan.h k_scan_lb's, three fields): lane l reads tile j - l's words; the nearest tile with an
      // inclusive prefix ends the walk, the aggregates after it are summed
      if (tile > 0) {
        // (lane l reads tiles j - LB_TPL l - t, t < LB_TPL: a wave step covers 64 LB_TPL tiles; four tiles per lane
        // measured slower than one: 2.47 against 1.92 ms per chr1-size unit alone, the polls' traffic)
        constexpr int LB_TPL = 1;
        E3 prefix{0, 0, 0};
        for (int64_t j = tile - 1;; j -= 64 * LB_TPL) {
          bool is_inc = false, ok = false;
          E3 val{0, 0, 0};
          uint32_t spins = 0;
          while (!ok) {
            // this lane's tiles, nearest first: aggregates summed up to the first inclusive prefix (taken, then stop)
            bool ready = true, hit = false;
            E3 v{0, 0, 0};
#pragma unroll
            for (int t = 0; t < LB_TPL; t++) {
              const int64_t jj = j - LB_TPL * lane - t;
              uint64_t wi[3], wa[3];
#pragma unroll
              for (int k = 0; k < 3; k++) {
                wi[k] = jj >= 0 ? lb_get(lb_inc + (size_t)k * A.ntiles + jj) : 0;
                wa[k] = jj >= 0 ? lb_get(lb_agg + (size_t)k * A.ntiles + jj) : 0;
              }
              if (jj < 0 || hit) continue;
              bool all_inc = true, all_agg = true;
#pragma unroll
              for (int k = 0; k < 3; k++) {
                all_inc &= lb_flag(wi[k], A.epoch) == 2u;
                all_agg &= lb_flag(wa[k], A.epoch) == 1u;
              }
              const uint64_t *w = all_inc ? wi : wa;
              if (all_inc || all_agg) {
                v = v + E3{(int64_t)(w[0] >> LB_VAL_SHIFT), (int64_t)(w[1] >> LB_VAL_SHIFT),
                           (int64_t)(w[2] >> LB_VAL_SHIFT)};
                hit = all_inc;
              } else {
                ready = false;
              }
            }
            if (ready) {
              ok = true;
              is_inc = hit || j - LB_TPL * lane < 0;   // (past tile 0: nothing further back)
              val = v;
            } else if (++spins > (1u << 24)) {   // (a bound on the wait: reported, never a hung GPU)
              ok = is_inc = true;
              if (A.fault) __hip_atomic_fetch_or(A.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
              __builtin_amdgcn_s_sleep(1);
            }
          }
          const uint64_t bal = __ballot(is_inc);
          const int first = bal ? __builtin_ctzll(bal) : 64;   // nearest lane whose tiles reach an inclusive prefix
          if (lane > first) val = E3{0, 0, 0};
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) val = val + shfl_xor_t(val, d);
          prefix = prefix + val;
          if (first < 64) break;
        }
        P = prefix;
        const E3 mine = prefix + E3{tk, tb0, tb1};
        const int64_t mv = lane == 0 ? mine.kept : lane == 1 ? mine.b1 : mine.b2;
        if (lane < 3) lb_put(lb_inc + (size_t)lane * A.ntiles + tile, mv, 2u, A.epoch);
      }
    }
    if (A.cur_out) {   // a chained unit (mh_emit_reads_async): no host readback between units
      if (A.cur_in) {  // where the previous unit's writer ended
        u0 = A.cur_in[1];
        u1 = A.cur_in[2];
      }
      if (tile == A.ntiles - 1 && lane == 0) {   // the unit's totals: the next unit's start, the host's readback
        const E3 T = P + E3{tk, tb0, tb1};
        const int64_t ds = digit_sum(A.cnt_base + T.kept) - digit_sum(A.cnt_base);
        const int64_t b1 = T.b1 + ds, b2 = NF == 2 ? T.b2 + ds : 0;
        A.cur_out[0] = T.kept;
        A.cur_out[1] = u0 + b1;
        A.cur_out[2] = u1 + b2;
        A.res[0] = T.kept;
        A.res[1] = b1;
        A.res[2] = b2;
        A.res[3] = u0 + b1;
        A.res[4] = u1 + b2;
      }
    }
    // sums over the tile's templates before this one (the inclusive value of lane 2 jf - 1)
    const int src = jf ? 2 * jf - 1 : 0;
    int32_t xk = __shfl(ik, src, 64), x0 = __shfl(i0, src, 64), x1 = __shfl(i1, src, 64);
    if (jf == 0) xk = x0 = x1 = 0;
    const int64_t K0 = A.cnt_base + P.kept;                          // templates kept before the tile
    const int64_t ds0 = digit_sum(K0) - digit_sum(A.cnt_base);       // cnt digits of the emission's records before it
    const int64_t g0 = u0 + P.b1 + ds0;
    const int64_t g1 = u1 + P.b2 + ds0;
    if (tid == 0) {
      const int64_t dst = digit_sum(K0 + tk) - digit_sum(K0);        // ... of the tile's records
      s_g[0] = g0;
      s_g[1] = g1;
      s_span[0] = (int32_t)(tb0 + dst);
      s_span[1] = (int32_t)(tb1 + dst);
      s_skip = 0;
      if (FU && (g0 + tb0 + dst > A.cap[0] || (NF == 2 && g1 + tb1 + dst > A.cap[1]))) {
        s_skip = 1;
        if (A.fault) __hip_atomic_fetch_or(A.fault, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (valid) {
      DMeta &mt = meta[jf];
      const int64_t cnt = K0 + xk + 1;                               // 1-based among kept templates (:209-210)
      const int nd = ndig_u((uint64_t)cnt);
      const int32_t rel = (int32_t)((fr == 0 ? x0 : x1) + digit_sum(K0 + xk) - digit_sum(K0));
      mt.len[fr] = keep ? lw + nd : 0;
      mt.rel[fr] = rel;
      const int32_t lh = Lp + nd + Lm;
      const int32_t qb = o_q + jf * qstride + head - lh, sb = lh + rest + 1;
      if (keep) {
        // mate 1 reads the reverse complement forward: from rc at hap_len - a - S
        const int32_t lead = !s ? (int32_t)(a & 15) : (int32_t)((h.hap_len - a - S) & 15);
        mt.bb[fr] = o_win + (jf * 2 + s) * win_stride + lead;
        mt.S[fr] = S;
        mt.tb[fr] = CR == 2 ? o_tr + (NF == 2 ? jf * 2 + fr : jf) * TS : o_t;
        mt.tn[fr] = CR ? S + 4 : TL;
        if (fr == 0) {   // the qname head ('@stub:' cnt '|chrom|cpy'), right-aligned before the reads part
          mt.qb = qb;
          mt.sb = sb;
          char *d = smem + qb;
          for (int i = 0; i < Lp; i++) d[i] = (char)qh.at(i);
          uint32_t x = (uint32_t)cnt;
          for (int i = nd - 1; i >= 0; i--) { d[Lp + i] = (char)('0' + x % 10u); x /= 10u; }
          for (int i = 0; i < Lm; i++) d[Lp + nd + i] = (char)qh.at(Lp + i);
        }
      }
      if (CR == 1 && (NF == 2 || fr == 0)) {   // the record's first base, for the corruption pass (S = 0: dropped)
        const uint64_t so = (uint64_t)((fr ? g1 : g0) + rel + sb);
        A.crec[tf * NF + fr] = make_uint2((uint32_t)so, (uint32_t)(so >> 32) << 16 | (uint32_t)(keep ? S : 0));
      }
    }
  }
  EWP(tid < 64 ? 0 : 1);
  __syncthreads();
  EWP(tid < 64 ? 2 : 3);
  if (CR == 2) {
    // each row slot of a kept record: its qualities into the record's T, its substitutions into the window
    // (base_rot[b][code - 1], illumina.py:131-136,159-160); block 0 also writes T's separators
    auto lay = [&](int32_t sl, uint4 q, uint32_t code) {
      int f, j, b;
      (void)slot_g(sl, &f, &j, &b);
      if (j >= nt) return;
      const DMeta &M = meta[j];
      if (M.len[f] == 0) return;
      const int32_t S = M.S[f];
      char *const T = smem + M.tb[f];
      if (b == 0) {
        T[0] = '\n';
        T[1] = '+';
        T[2] = '\n';
        T[3 + S] = '\n';
      }
      const int n0 = ED_CRB * b;
      if (n0 >= S) return;
      char *const d = T + 3 + n0;
      if (S - n0 >= ED_CRB) {
        __builtin_memcpy(d, &q.x, 4);
        __builtin_memcpy(d + 4, &q.y, 4);
        __builtin_memcpy(d + 8, &q.z, 4);
        const uint16_t w2 = (uint16_t)q.w;
        __builtin_memcpy(d + 12, &w2, 2);
        d[14] = (char)(q.w >> 16);
      } else {
        const int cnt = S - n0;
        for (int k = 0; k < cnt; k++) d[k] = (char)(u4get(q, k >> 2) >> (8 * (k & 3)));
        code &= (1u << (2 * cnt)) - 1u;
      }
      char *const bs = smem + M.bb[f] + n0;
      while (code) {
        const int k = __builtin_ctz(code) >> 1;
        const uint32_t c = (code >> (2 * k)) & 3u;
        code &= ~(3u << (2 * k));
        bs[k] = (char)rot_base((uint8_t)bs[k], c - 1u);
      }
    };
#pragma unroll
    for (int k = 0; k < RK; k++)
      if (tid + k * ED_THREADS < nsl) lay(tid + k * ED_THREADS, rq[k], rcw[k]);
    for (int32_t sl = tid + RK * ED_THREADS; sl < nsl; sl += ED_THREADS) {   // (records of more than 23 blocks)
      int sf, sj, sbk;
      const int64_t g = slot_g(sl, &sf, &sj, &sbk);
      lay(sl, A.crow[g], A.ccode[g]);
    }
    __syncthreads();
    EWP(4);
  }
  const int64_t gbase[2] = {s_g[0], s_g[1]};
  const int32_t span[2] = {s_span[0], s_span[1]};
  if (FU && s_skip) return;
  ed_output<NF, LPR, CR>(meta, nt, gbase, span, o_t, TL, o_s, staged, A.arena EWP_ARG);
  EWP_END;
}

// One workgroup per 32-template tile.  (A grid-stride loop over tiles kept ~140 VGPRs live across iterations — three
// waves per SIMD instead of eight — and the launch of 184 k workgroups costs only ~0.35 ms of a 2.6 ms chr1-unit
// writer (round 3), so there is no persistent variant.)
template <int NF, int LPR, int CR, int GW>
__global__ void __launch_bounds__(ED_THREADS) k_emit_tiles(TArgs A, QHead qh) {
  emit_tile<NF, LPR, CR, GW>(A, qh, blockIdx.x);
}

// The single-pass writer: tiles numbered by an atomic ticket in the order they start (HIP promises no dispatch
// order), so every tile a look-back waits for is already running.
template <int NF, int LPR, int CR, int GW>
__global__ void __launch_bounds__(ED_THREADS) k_emit_fused(TArgs A, QHead qh) {
  __shared__ int64_t s_tile;
  if (threadIdx.x == 0) s_tile = (int64_t)(uint32_t)(atomicAdd((uint32_t *)A.lb, 1u) - A.tbase);
  __syncthreads();
  emit_tile<NF, LPR, CR, GW, true>(A, qh, s_tile);
}

// ---- BQ corruption of the emitted records (illumina.corrupt_template, illumina.py:139-162) ---------------------
// After the writer (same stream), over the records it laid out with len(seq) placeholder qualities:
//   k_cr_recs     one thread per template: each record's first-base offset in its arena and S (0: dropped), packed
//                 in 8 bytes (offset low word | offset high bits << 16 | S);
//   k_cr_inplace  one item per 15-base block of every record (five Philox triple draws); qualities stored, the
//                 record's last byte set to '\n', substituted bases replaced from the block's prefetched bases;
//                 the rare bases whose draw lands on a threshold (full 53-bit decisions) in a loop after the block.  Persistent workgroups stage the bucket-table rows of the read positions and the low
//                 threshold bytes in LDS once, so a base's BQ is one LDS byte read (plus a short walk in a flagged
//                 bucket); the next item's record word is loaded while the current one computes.
constexpr int CI_THREADS = 1024;
constexpr int CI_BLK = 15;   // bases per item: five triple draws

struct CiArgs {
  int64_t p_min, hap_len;
  int64_t m;
  const int64_t *pos0, *pos1;
  const int8_t *fo0;
  const Rec *recs;
  const E3 *off;
  char *arena[2];         // the emission's first byte per file
  const uint2 *crec;      // [m * nf] per record: k_cr_recs' packed offset and S
  int32_t rlen, nf, lh0;  // lh0: qname head bytes without the cnt digits ('@stub:' + '|chrom|cpy')
  CorruptCfg cc;
};

// The LDS-table BQ step of one base (k_cr_inplace's walk): bk = the base's bucket row, tp = its threshold-pair row.
// Entries below h1 = w >> 16 (capped at 93); *amb when one equals h1, or three or more of the bucket's lie below it.
// (base + 32-bit offset form: with global tables a uniform base and 32-bit lane offsets, not 64-bit lane pointers)
__device__ __forceinline__ uint32_t cr_walk_at(const uint8_t *bk, uint32_t obk, const uint16_t *tp, uint32_t otp,
                                               uint32_t w, uint32_t *amb) {
  const uint32_t e = bk[obk + (w >> 24)];
  const uint32_t c = e & 0x7fu, fl = e >> 7;
  const uint32_t pa = tp[otp + c], pb = tp[otp + c + 1];
  const uint32_t lo = (w >> 16) & 0xffu;
  const uint32_t v0 = pa & 0xffu, v1 = pa >> 8, v2 = pb >> 8;
  const uint32_t b0 = fl & (uint32_t)(v0 < lo), b1 = b0 & (uint32_t)(v1 < lo), b2 = b1 & (uint32_t)(v2 < lo);
  const uint32_t vn = b1 ? v2 : (b0 ? v1 : v0);
  *amb = b2 | (fl & (uint32_t)(vn == lo));
  return c + b0 + b1;
}
__device__ __forceinline__ uint32_t cr_lds_walk(const uint8_t *bk, const uint16_t *tp, uint32_t w, uint32_t *amb) {
  return cr_walk_at(bk, 0u, tp, 0u, w, amb);
}

// One full 15-base block of a record with the tables in LDS: five triple draws, per base a BQ step and the U2
// decision, the qualities stored; then the rare bases (f64 decisions), then the substituted bases with their choices
// (the triple's 10-bit field, or the base's own draw when it is 1023) — the same stream and decisions as the guarded
// path in k_cr_inplace, with no per-base guards so the fifteen bases' LDS reads can be in flight together.
// bk / tp: the bucket and threshold-pair rows of base n0 (row j of base n0 + j at bk + j * CB_ROW, tp + j * n_bq).
__device__ __forceinline__ void cr_full_block(const uint8_t *bk, const uint16_t *tp, const uint16_t *fp,
                                              const CorruptCfg &cc, uint2 key, uint32_t tl, uint32_t th, int f,
                                              int n0, char *seq, uint64_t sa, uint4 g0, uint4 g1, char *qual) {
  const int n_bq = cc.n_bq;
  // in phases, so each phase's fifteen LDS reads are in flight together (the arrays are registers: constant indices)
  uint32_t W[CI_BLK], RW[CI_BLK / 3], E[CI_BLK], P[CI_BLK], V2[CI_BLK], F[CI_BLK], BQ[CI_BLK];
  const uint32_t cw = ((uint32_t)f << 16) | (uint32_t)n0 / 3u;
#pragma unroll
  for (int g = 0; g < CI_BLK / 3; g++) {   // the five triple draws
    const uint4 r = philox4x32_10(make_uint4(tl, th, cw + (uint32_t)g, cc.c3), key);
    W[3 * g] = r.x;
    W[3 * g + 1] = r.y;
    W[3 * g + 2] = r.z;
    RW[g] = r.w;
  }
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) E[j] = bk[j * CB_ROW + (W[j] >> 24)];   // bucket entries
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) {   // threshold pairs of entries c, c + 1 (only a flagged bucket uses them)
    const uint16_t *t = tp + j * n_bq + (E[j] & 0x7fu);
    P[j] = t[0];
    V2[j] = ((const uint8_t *)t)[3];
  }
  uint32_t ps = 0, px = 0;
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) {   // BQ steps (as cr_lds_walk), then Fp16 of each
    const uint32_t e = E[j], c = e & 0x7fu, fl = e >> 7, pa = P[j];
    const uint32_t lo = (W[j] >> 16) & 0xffu;
    const uint32_t v0 = pa & 0xffu, v1 = pa >> 8, v2 = V2[j];
    const uint32_t b0 = fl & (uint32_t)(v0 < lo), b1 = b0 & (uint32_t)(v1 < lo), b2 = b1 & (uint32_t)(v2 < lo);
    const uint32_t vn = b1 ? v2 : (b0 ? v1 : v0);
    const uint32_t amb = b2 | (fl & (uint32_t)(vn == lo));
    BQ[j] = c + b0 + b1;
    px |= amb << j;
    F[j] = fp[BQ[j]];
  }
  uint32_t qd0 = 0, qd1 = 0, qd2 = 0, qd3 = 0;
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) {   // U2 decisions
    const uint32_t amb = (px >> j) & 1u, pth = F[j], h2 = W[j] & 0xffffu;
    ps |= (uint32_t)(!amb && h2 < pth) << j;
    px |= (uint32_t)(h2 == pth) << j;
    const uint32_t qv = (BQ[j] + 33u) << (8 * (j & 3));
    if (j < 4) qd0 |= qv; else if (j < 8) qd1 |= qv; else if (j < 12) qd2 |= qv; else qd3 |= qv;
  }
  const uint32_t rw0 = RW[0], rw1 = RW[1], rw2 = RW[2], rw3 = RW[3], rw4 = RW[4];
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) {
    const uint32_t q = j < 4 ? qd0 : j < 8 ? qd1 : j < 12 ? qd2 : qd3;
    qual[n0 + j] = (char)(q >> (8 * (j & 3)));
  }
  // rare: the full 53-bit decisions (U1 or U2 within 2^-16 of a threshold)
  while (px) {
    const int j = __builtin_ctz(px);
    px &= px - 1;
    const int n = n0 + j;
    // the base's word from the block's draws (a select chain: W is in registers; recomputing its Philox draw cost
    // ~100 instructions per pass of this loop, which a wave takes whenever one of its lanes has a flagged base)
    uint32_t w = W[0];
#pragma unroll
    for (int i = 1; i < CI_BLK; i++) w = j == i ? W[i] : w;
    uint32_t amb;
    const uint32_t bq = cr_lds_walk(bk + j * CB_ROW, tp + j * n_bq, w, &amb);
    const uint32_t x = cq_exact_body(cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq, cc.k0, cc.k1, cc.c3, tl, th, f, n,
                                     w, bq, amb);
    qual[n] = (char)((x & 0xffu) + 33);
    ps |= (x >> 8) << j;
  }
  if (!ps) return;
  // the substituted bases (about 0.7 of 15 at a 4.7 % error rate): base_rot[b][choice]
  const uint32_t sh = (uint32_t)(sa & 15);
  const uint32_t o = sh >> 2, bsh = 8 * (sh & 3);
  const uint32_t d0 = o == 0 ? g0.x : o == 1 ? g0.y : o == 2 ? g0.z : g0.w;
  const uint32_t d1 = o == 0 ? g0.y : o == 1 ? g0.z : o == 2 ? g0.w : g1.x;
  const uint32_t d2 = o == 0 ? g0.z : o == 1 ? g0.w : o == 2 ? g1.x : g1.y;
  const uint32_t d3 = o == 0 ? g0.w : o == 1 ? g1.x : o == 2 ? g1.y : g1.z;
  const uint32_t d4 = o == 0 ? g1.x : o == 1 ? g1.y : o == 2 ? g1.z : g1.w;
  const uint32_t bw0 = (uint32_t)(((uint64_t)d1 << 32 | d0) >> bsh), bw1 = (uint32_t)(((uint64_t)d2 << 32 | d1) >> bsh),
                 bw2 = (uint32_t)(((uint64_t)d3 << 32 | d2) >> bsh), bw3 = (uint32_t)(((uint64_t)d4 << 32 | d3) >> bsh);
  do {
    const int j = __builtin_ctz(ps);
    ps &= ps - 1;
    const int g = j / 3, k = j - 3 * g;
    const uint32_t rw = g == 0 ? rw0 : g == 1 ? rw1 : g == 2 ? rw2 : g == 3 ? rw3 : rw4;
    const uint32_t c10 = (rw >> (10 * k)) & 1023u;
    uint32_t chv;
    if (c10 == 1023u)   // rejected: the base's own draw (t, f | 0x8000, n)
      chv = __umulhi(philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)(n0 + j), cc.c3),
                                   key).x, 3u);
    else
      chv = c10 % 3u;
    const uint32_t bw = j < 4 ? bw0 : j < 8 ? bw1 : j < 12 ? bw2 : bw3;
    seq[n0 + j] = (char)rot_base((uint8_t)(bw >> (8 * (j & 3))), chv);
  } while (ps);
}

__global__ void __launch_bounds__(256) k_cr_recs(CiArgs A, uint2 *crec) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= A.m) return;
  const int4 rc = *(const int4 *)(A.recs + t);   // keep, len1, len2, rest
  const int fo = A.fo0[t];
  const E3 o = A.off[t];
  for (int f = 0; f < A.nf; f++) {
    const int64_t p = f == fo ? A.pos0[t] : A.pos1[t];   // file f holds mate f == fo ? 0 : 1
    int64_t a = p - A.p_min, e = p + A.rlen - A.p_min;
    if (e > A.hap_len) e = A.hap_len;
    if (a > A.hap_len) a = A.hap_len;
    const uint32_t S = rc.x && e > a ? (uint32_t)(e - a) : 0u;
    // '@stub:' cnt '|chrom|cpy' reads-part '\n' | bases | '\n+\n' | qualities | '\n'
    const uint64_t so = (uint64_t)((f ? o.b2 : o.b1) + A.lh0 +
                                   ndig_u((uint64_t)(o.kept + 1)) + rc.w + 1);
    crec[t * A.nf + f] = make_uint2((uint32_t)so, (uint32_t)(so >> 32) << 16 | S);
  }
}

// PF (two files): a workgroup corrupts one file's records only (file = blockIdx.x & 1), so it stages that file's tables
// alone — half the LDS, two workgroups (8 waves per SIMD) per CU instead of one.
template <bool LDS_TAB, bool PF, int THR>
__global__ void __launch_bounds__(THR, PF ? THR / 128 : THR / 256) k_cr_inplace(CiArgs A) {   // (PF: two per CU)
  // LDS: bucket entries [NT][rlen][CB_ROW] | Fp16[100] | low-byte pairs of the thresholds [NT][rlen][n_bq] (u16);
  // NT = 2 files, or 1 with PF
  extern __shared__ __attribute__((aligned(16))) uint8_t ctab[];
  constexpr int NT = PF ? 1 : 2;
  const int f_pf = PF ? (int)(blockIdx.x & 1u) : 0;
  const CorruptCfg &cc = A.cc;
  const int rlen = A.rlen, n_bq = cc.n_bq;
  const uint32_t lim_all = n_bq < 93 ? (uint32_t)n_bq : 93u;
  const int32_t row_bytes = rlen * CB_ROW;   // per file
  const uint16_t *fp16 = (const uint16_t *)(ctab + NT * row_bytes);
  const int32_t o_t8 = NT * row_bytes + 256;
  if (LDS_TAB) {
    for (int ft = 0; ft < NT; ft++) {
      const int f = PF ? f_pf : ft;
      const uint4 *src = (const uint4 *)(cc.bk + (int64_t)f * cc.max_bp * CB_ROW);
      uint4 *dst = (uint4 *)(ctab + ft * row_bytes);
      for (int i = threadIdx.x; i < row_bytes / 16; i += THR) dst[i] = src[i];
      // per entry j: its low byte | (entry j + 1's low byte when j + 1 < min(n_bq, 93) lies in j's bucket, else 0xff) << 8
      const uint16_t *t16 = cc.T16 + (int64_t)f * cc.max_bp * n_bq;
      for (int i = threadIdx.x; i < rlen * n_bq; i += THR) {
        const int j = i % n_bq;
        const uint32_t a = t16[i], b = j + 1 < (int)lim_all ? t16[i + 1] : 0xffffu;
        ((uint16_t *)(ctab + o_t8))[ft * rlen * n_bq + i] = (uint16_t)((a & 0xffu) | ((b >> 8) == (a >> 8) ? (b & 0xffu) << 8 : 0xff00u));
      }
    }
    for (int i = threadIdx.x; i < 100; i += THR) ((uint16_t *)fp16)[i] = cc.Fp16[i];
    __syncthreads();
  }
  // the BQ step of base n of file f for the draw's high 16 bits: entries below h1 (capped at 93), amb when one
  // equals h1 — or when three or more of the bucket's entries lie below h1 (rare): amb sends the base to the exact
  // path, whose f64 search gives the same step.  LDS: the bucket entry, then for a flagged bucket the low bytes of
  // its first three entries from two pair reads, without branches.  Global: bq_walk_g.
  const uint16_t *t8p = (const uint16_t *)(ctab + o_t8);
  auto walk = [&](int f, int n, uint32_t h1, bool *amb) -> uint32_t {
    if (!LDS_TAB) return bq_walk_g(cc, f, n, h1, amb);
    const int row = (PF ? 0 : f * rlen) + n;
    const uint32_t e = ctab[row * CB_ROW + (int)(h1 >> 8)];
    const uint32_t c = e & 0x7fu;
    // entry c's low byte | entry c + 1's (0xff when outside the bucket) << 8; the same pair of entry c + 1.  A 0xff
    // stand-in never counts as below, and makes amb conservative when lo = 255 (the exact path decides the same).
    const uint32_t pa = t8p[row * n_bq + c], pb = t8p[row * n_bq + c + 1];
    const uint32_t lo = h1 & 0xffu;
    const uint32_t fl = e >> 7;
    const uint32_t v0 = pa & 0xffu, v1 = pa >> 8, v2 = pb >> 8;
    // (bitwise, not short-circuit: no branches)
    const uint32_t b0 = fl & (uint32_t)(v0 < lo), b1 = b0 & (uint32_t)(v1 < lo), b2 = b1 & (uint32_t)(v2 < lo);
    const uint32_t vn = b1 ? v2 : (b0 ? v1 : v0);   // the first entry not below h1 so far
    *amb = (b2 | (fl & (uint32_t)(vn == lo))) != 0u;
    return c + b0 + b1;
  };
  auto fp = [&](uint32_t bq) -> uint32_t { return LDS_TAB ? fp16[bq] : cc.Fp16[bq]; };
  const uint2 key = make_uint2(cc.k0, cc.k1);
  // items: 15-base blocks of the records, NB per record (block b = bases 15b .. 15b + 14: five triple draws)
  // (PF: items of this workgroup's file only; an item's unit q is then the template, its record 2 q + file)
  const uint32_t NB = (uint32_t)(rlen + CI_BLK - 1) / CI_BLK;
  const uint32_t n_items = (uint32_t)(A.m * (PF ? 1 : A.nf)) * NB;
  const uint32_t stride = (PF ? gridDim.x >> 1 : gridDim.x) * THR;
  const uint32_t nb_magic = 0xffffffffu / NB + 1u;   // umulhi(i, nb_magic) is i / NB or one more
  auto unit_of = [&](uint32_t i) -> uint32_t {
    i = i < n_items ? i : 0u;
    const uint32_t q = __umulhi(i, nb_magic);
    return q * NB > i ? q - 1 : q;
  };
  auto rec_of = [&](uint32_t i) -> uint32_t { return PF ? 2u * unit_of(i) + (uint32_t)f_pf : unit_of(i); };
  uint32_t i = (PF ? blockIdx.x >> 1 : blockIdx.x) * THR + threadIdx.x;
  uint2 R = A.crec[rec_of(i)];                         // this item's record word; the next one is in flight below
  for (; i < n_items; i += stride) {
    const uint32_t uq = unit_of(i);
    const uint32_t rr = PF ? 2u * uq + (uint32_t)f_pf : uq;
    const uint2 Rn = A.crec[rec_of(i + stride)];     // prefetch
    const uint32_t S = R.y & 0xffffu;
    const int n0 = CI_BLK * (int)(i - uq * NB);
    if ((uint32_t)n0 < S) {
      const int cnt = S - n0 < CI_BLK ? (int)S - n0 : CI_BLK;
      const int f = A.nf == 2 ? (int)(rr & 1) : 0;
      const int64_t tt = (int64_t)(A.nf == 2 ? rr >> 1 : rr) + cc.t_base;
      const uint32_t tl = (uint32_t)tt, th = (uint32_t)(tt >> 32);
      char *const seq = (f ? A.arena[1] : A.arena[0]) + (((uint64_t)(R.y >> 16) << 32) | R.x);
      char *const qual = seq + S + 3;
      // the block's bases: the two aligned 16-byte chunks holding them, shifted into bw[0..3] (base j = byte j)
      const uint64_t sa = (uint64_t)(seq + n0);
      const uint4 *sp = (const uint4 *)(sa & ~(uint64_t)15);
      const uint4 g0 = sp[0], g1 = sp[1];
      uint32_t qd[4] = {0, 0, 0, 0};   // the block's qualities, packed
      uint32_t px = 0, pc = 0, ps = 0;   // bases needing the f64 decisions / a fallback choice draw; substituted
      uint32_t ch = 0;                   // choices of the substituted bases (2 bits each)
      if (LDS_TAB && cnt == CI_BLK) {
        // A full block (every block of a 150-bp read): no per-base guards, so the bases' LDS reads interleave; the
        // choices are derived for the substituted bases only (cr_full_block).
        const int row0 = (PF ? 0 : f * rlen) + n0;
        cr_full_block(ctab + row0 * CB_ROW, t8p + row0 * n_bq, fp16, cc, key, tl, th, f, n0, seq, sa, g0, g1, qual);
        if (n0 + cnt == (int)S) qual[S] = '\n';
        R = Rn;
        continue;
      }
#pragma unroll
      for (int g = 0; g < CI_BLK / 3; g++) {
        if (3 * g < cnt) {
          const uint4 r = philox4x32_10(
              make_uint4(tl, th, ((uint32_t)f << 16) | ((uint32_t)n0 / 3u + (uint32_t)g), cc.c3), key);
#pragma unroll
          for (int k = 0; k < 3; k++) {
            const int j = 3 * g + k;
            if (j < cnt) {
              const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : r.z;
              bool amb;
              const uint32_t bq = walk(f, n0 + j, w >> 16, &amb);
              const uint32_t pth = fp(bq), h2 = w & 0xffffu;
              const uint32_t c10 = (r.w >> (10 * k)) & 1023u;
              const bool sub = !amb && h2 < pth;
              px |= (uint32_t)(amb || h2 == pth) << j;
              ps |= (uint32_t)sub << j;
              pc |= (uint32_t)(sub && c10 == 1023u) << j;
              ch |= (c10 % 3u) << (2 * j);
              qd[j >> 2] |= (bq + 33u) << (8 * (j & 3));
            }
          }
        }
      }
      char *const qb = qual + n0;
      if (cnt == CI_BLK) {
#pragma unroll
        for (int j = 0; j < CI_BLK; j++) qb[j] = (char)(qd[j >> 2] >> (8 * (j & 3)));
      } else {
#pragma unroll
        for (int j = 0; j < CI_BLK; j++)
          if (j < cnt) qb[j] = (char)(qd[j >> 2] >> (8 * (j & 3)));
      }
      if (n0 + cnt == (int)S) qual[S] = '\n';
      // rare: the full 53-bit decisions (the choice bits come from the same triple draw)
      while (px) {
        const int j = __builtin_ctz(px);
        px &= px - 1;
        const int n = n0 + j;
        const uint4 r = philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | ((uint32_t)n / 3u), cc.c3), key);
        const int k = n % 3;
        const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : r.z;
        bool amb;
        const uint32_t bq = walk(f, n, w >> 16, &amb);
        const uint32_t x = cq_exact_body(cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq, cc.k0, cc.k1, cc.c3, tl, th, f,
                                         n, w, bq, amb);
        qual[n] = (char)((x & 0xffu) + 33);
        const uint32_t c10 = (r.w >> (10 * k)) & 1023u;
        ps |= (x >> 8) << j;
        pc |= (uint32_t)((x >> 8) && c10 == 1023u) << j;
      }
      // rare: a substituted base whose 10 choice bits are 1023 (rejected): its own draw (t, f | 0x8000, n)
      while (pc) {
        const int j = __builtin_ctz(pc);
        pc &= pc - 1;
        const uint4 c = philox4x32_10(
            make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)(n0 + j), cc.c3), key);
        ch = (ch & ~(3u << (2 * j))) | (__umulhi(c.x, 3u) << (2 * j));
      }
      // the substituted bases: base_rot[b][choice]
      if (ps) {
        const uint32_t sh = (uint32_t)(sa & 15);
        const uint32_t o = sh >> 2, bsh = 8 * (sh & 3);
        // dwords o .. o + 4 of the 32 loaded bytes, then byte-aligned
        const uint32_t d0 = o == 0 ? g0.x : o == 1 ? g0.y : o == 2 ? g0.z : g0.w;
        const uint32_t d1 = o == 0 ? g0.y : o == 1 ? g0.z : o == 2 ? g0.w : g1.x;
        const uint32_t d2 = o == 0 ? g0.z : o == 1 ? g0.w : o == 2 ? g1.x : g1.y;
        const uint32_t d3 = o == 0 ? g0.w : o == 1 ? g1.x : o == 2 ? g1.y : g1.z;
        const uint32_t d4 = o == 0 ? g1.x : o == 1 ? g1.y : o == 2 ? g1.z : g1.w;
        const uint32_t bw0 = (uint32_t)(((uint64_t)d1 << 32 | d0) >> bsh), bw1 = (uint32_t)(((uint64_t)d2 << 32 | d1) >> bsh),
                       bw2 = (uint32_t)(((uint64_t)d3 << 32 | d2) >> bsh), bw3 = (uint32_t)(((uint64_t)d4 << 32 | d3) >> bsh);
        do {   // one iteration per substituted base of the lane (about 0.7 of 15 at a 4.7 % error rate)
          const int j = __builtin_ctz(ps);
          ps &= ps - 1;
          const uint32_t bw = j < 4 ? bw0 : j < 8 ? bw1 : j < 12 ? bw2 : bw3;
          seq[n0 + j] = (char)rot_base((uint8_t)(bw >> (8 * (j & 3))), (ch >> (2 * j)) & 3u);
        } while (ps);
      }
    }
    R = Rn;
  }
}

static_assert(ED_CRB == CI_BLK, "the writer's row blocks are the corruption blocks");

// ---- corruption rows (the direct writer's mode): the BQ draws before the writer -----------------------------------
// k_cr_cols runs the items, stream and decisions of k_cr_inplace over every block of every record up to rlen (a
// record of S < rlen bases uses the first S: the draws are counted by (template, file, triple), not by S) without
// touching the arenas: per block one aligned 16-byte row slot (its qualities + 33) and one word of 2-bit
// substitution codes (choice + 1; 0: the base stays), slot (file * NB + block) * m + template (column-major: a
// tile's 32 slots of one block are contiguous, and k_cr_cols writes whole lines).  The writer
// (k_emit_tiles<.., 2>) lays the qualities into per-record T strings in LDS and applies the codes to its windows, so
// the corrupted records leave the writer in its aligned 16-byte stores (no partial-line rewrite afterwards).

// The row pass's BQ step from the fine table (k_cr_cols' LDS): entries of row j below h1 (capped at 93) from the
// bucket entry e = bkf[j][h1 >> CF_SHIFT]; a flagged bucket (a threshold inside it) walks the row's T16 entries from
// there, *amb when one equals h1.  The same counts and ambiguity as cr_walk_at's 256-bucket table and its pairs.
__device__ __forceinline__ uint32_t cr_fine_walk(uint32_t e, const uint16_t *t16, uint32_t lim, uint32_t h1,
                                                 uint32_t *amb) {
  uint32_t c = e & 0x7fu;
  *amb = 0;
  if (e & 0x80u) {
    while (c < lim && t16[c] < h1) c++;
    *amb = c < lim && t16[c] == h1;
  }
  return c;
}

// One flagged draw (a threshold inside its bucket, or U2 on Fp16[bq]) of base n0 + j, resolved alone: its triple's
// draw again, the walk from the bucket entry, then the 16-bit U2 decision or the full 53-bit ones.  Returns the
// quality byte (bq + 33) | the base's substitution code << 8 (choice + 1, 0: the base stays).  n0 is a multiple of 3
// (15 * block).
__device__ __forceinline__ uint32_t cr_px_resolve(const uint8_t *bkf, const uint16_t *t16, const uint16_t *fp,
                                                  const CorruptCfg &cc, uint2 key, uint32_t tl, uint32_t th, int f,
                                                  int n0, int j, uint32_t lim) {
  const int n = n0 + j;
  const uint4 r = philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | ((uint32_t)n / 3u), cc.c3), key);
  const int k = j % 3;
  const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : r.z;
  uint32_t amb;
  const uint32_t bq = cr_fine_walk(bkf[j * CF_ROW + (w >> (16 + CF_SHIFT))], t16 + j * cc.n_bq, lim, w >> 16, &amb);
  const uint32_t pth = fp[bq], h2 = w & 0xffffu;
  const uint32_t x = amb || h2 == pth ? cq_exact_body(cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq, cc.k0, cc.k1,
                                                      cc.c3, tl, th, f, n, w, bq, amb)
                                      : bq | (h2 < pth ? 0x100u : 0u);
  uint32_t code = 0;
  if (x >> 8) {
    const uint32_t c10 = (r.w >> (10 * k)) & 1023u;
    code = 1u + (c10 == 1023u ? __umulhi(philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)n,
                                                                   cc.c3), key).x, 3u)
                              : c10 % 3u);
  }
  return ((x & 0xffu) + 33u) | code << 8;
}

// A full block's fast step with the fine table in LDS, into registers: per base one bucket byte and the Fp16 of its
// BQ decide (about 98 % of draws).  Qualities + 33 into qd[4] (the flagged bases' bytes are placeholders), the
// substituted bases into *ps, the flagged ones (left to the caller: cr_px_resolve) into *px; RW: the triples' fourth
// words (the choice bits).  bkf: base n0's row (row j at bkf + j * CF_ROW).
__device__ __forceinline__ void cr_block_fast(const uint8_t *bkf, const uint16_t *fp, const CorruptCfg &cc, uint2 key,
                                              uint32_t tl, uint32_t th, int f, int n0, uint32_t *qd, uint32_t *ps_o,
                                              uint32_t *px_o, uint32_t *RW) {
  uint32_t W[CI_BLK], E[CI_BLK], F[CI_BLK];
  const uint32_t cw = ((uint32_t)f << 16) | (uint32_t)n0 / 3u;
#pragma unroll
  for (int g = 0; g < CI_BLK / 3; g++) {
    const uint4 r = philox4x32_10(make_uint4(tl, th, cw + (uint32_t)g, cc.c3), key);
    W[3 * g] = r.x;
    W[3 * g + 1] = r.y;
    W[3 * g + 2] = r.z;
    RW[g] = r.w;
  }
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) E[j] = bkf[j * CF_ROW + (W[j] >> (16 + CF_SHIFT))];
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) F[j] = fp[E[j] & 0x7fu];
  uint32_t ps = 0, px = 0, qd0 = 0, qd1 = 0, qd2 = 0, qd3 = 0;
#pragma unroll
  for (int j = 0; j < CI_BLK; j++) {
    const int32_t d = (int32_t)(W[j] & 0xffffu) - (int32_t)F[j];   // U2's top 16 bits against Fp16[bq]
    ps |= ((uint32_t)d >> 31) << j;
    px |= (uint32_t)(d == 0 || (E[j] & 0x80u)) << j;
    const uint32_t qv = ((E[j] & 0x7fu) + 33u) << (8 * (j & 3));
    if (j < 4) qd0 |= qv; else if (j < 8) qd1 |= qv; else if (j < 12) qd2 |= qv; else qd3 |= qv;
  }
  qd[0] = qd0;
  qd[1] = qd1;
  qd[2] = qd2;
  qd[3] = qd3;
  *ps_o = ps & ~px;
  *px_o = px;
}

// The block's substitution codes (2 bits per base: choice + 1) from the triples' choice bits: randint(0, 3) as
// c10 % 3, or (c10 == 1023, rejected) the base's own draw (t, f | 0x8000, n)
__device__ __forceinline__ uint32_t cr_block_codes(uint32_t ps, const uint32_t *RW, const CorruptCfg &cc, uint2 key,
                                                   uint32_t tl, uint32_t th, int f, int n0) {
  uint32_t cd = 0;
#ifdef EW_CALIB_NOPS
  ps = 0;
#endif
  while (ps) {
    const int j = __builtin_ctz(ps);
    ps &= ps - 1;
    const int g = j / 3, k = j - 3 * g;
    const uint32_t rw = g == 0 ? RW[0] : g == 1 ? RW[1] : g == 2 ? RW[2] : g == 3 ? RW[3] : RW[4];
    const uint32_t c10 = (rw >> (10 * k)) & 1023u;
    uint32_t chv;
    if (c10 == 1023u)
      chv = __umulhi(philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)(n0 + j), cc.c3),
                                   key).x, 3u);
    else
      chv = c10 % 3u;
    cd |= (chv + 1u) << (2 * j);
  }
  return cd;
}


// The corruption rows: a workgroup per (block column, template chunk) stages only its column's tables (bucket rows
// and threshold pairs of 15 positions of one file: 6.7 KB; a record-major pass staging a whole file's 67 KB was
// LDS-bound at 4.3 ms per chr1 unit, round 3), so occupancy is bound by registers, not LDS; its threads take
// consecutive templates, so the slots it writes are contiguous.  The items, stream and decisions of k_cr_inplace,
// over every block of every record up to rlen.
//
// The flagged draws (~2.2 % of draws: ~21 per wave and block) are resolved by the whole wave at once (round 5): a
// lane looping over its own flagged bases ran the wave for the busiest of its 64 lanes (~2.2 Philox draws and walks
// per block, a third of the kernel's vector instructions); instead each wave lists its (lane, base) items in LDS,
// one lane takes one item (its draw, walk and decision), and writes the quality byte and the substitution bit back
// into the owner's LDS slot.  A wave with more than CC_PX_CAP items (none seen; the tables would need far more
// thresholds per bucket) resolves them lane by lane as before.
constexpr int CC_THREADS = 256;
constexpr int CC_WAVES = CC_THREADS / 64;
constexpr int CC_PER_WG = 16 * CC_THREADS;   // templates per workgroup (2048 or 8192: within noise)
constexpr int CC_PX_CAP = 64;
struct CcWave {
  uint4 qd[64];
  uint32_t code[64];
  uint16_t item[CC_PX_CAP];   // lane | base << 6
};
// the column tables' LDS, then the waves' item areas (16-aligned)
__host__ __device__ constexpr size_t cc_tables_lds(int32_t n_bq) {
  return ((size_t)CI_BLK * CF_ROW + 256 + (size_t)CI_BLK * n_bq * 2 + 15) / 16 * 16;
}

// at most 80 VGPRs (6 waves per SIMD; 87 unbounded, 5 waves): 2.7 % faster, one spilled word outside the loop
__global__ void __launch_bounds__(CC_THREADS) __attribute__((amdgpu_waves_per_eu(6))) k_cr_cols(CiArgs A, uint4 *rows, uint32_t *codes) {
  const int32_t per_wg = CC_PER_WG;
  extern __shared__ __attribute__((aligned(16))) uint8_t ctab[];
  const CorruptCfg &cc = A.cc;
  const int rlen = A.rlen, n_bq = cc.n_bq;
  const int NB = (rlen + CI_BLK - 1) / CI_BLK;
  const int col = (int)blockIdx.y, f = col / NB, b = col - f * NB, n0 = CI_BLK * b;
  const int cnt = rlen - n0 < CI_BLK ? rlen - n0 : CI_BLK;
  // LDS: fine bucket rows [15][CF_ROW] | Fp16[100] (256 B) | T16 rows [15][n_bq] | the waves' CcWave areas
  const int32_t o_fp = CI_BLK * CF_ROW, o_t16 = o_fp + 256;
  {
    const uint4 *src = (const uint4 *)(cc.bkf + ((int64_t)f * cc.max_bp + n0) * CF_ROW);
    uint4 *dst = (uint4 *)ctab;
    for (int i = threadIdx.x; i < cnt * CF_ROW / 16; i += CC_THREADS) dst[i] = src[i];
    const uint16_t *t16 = cc.T16 + ((int64_t)f * cc.max_bp + n0) * n_bq;
    for (int i = threadIdx.x; i < cnt * n_bq; i += CC_THREADS) ((uint16_t *)(ctab + o_t16))[i] = t16[i];
    for (int i = threadIdx.x; i < 100; i += CC_THREADS) ((uint16_t *)(ctab + o_fp))[i] = cc.Fp16[i];
  }
  __syncthreads();
  const uint8_t *bkf = ctab;
  const uint16_t *fp16 = (const uint16_t *)(ctab + o_fp);
  const uint16_t *t16 = (const uint16_t *)(ctab + o_t16);
  const int lane = (int)(threadIdx.x & 63);
  CcWave &cw = ((CcWave *)(ctab + cc_tables_lds(n_bq)))[threadIdx.x >> 6];
  const uint32_t lim = n_bq < 93 ? (uint32_t)n_bq : 93u;
  const uint2 key = make_uint2(cc.k0, cc.k1);
  const int64_t tb = (int64_t)blockIdx.x * per_wg, te = tb + per_wg < A.m ? tb + per_wg : A.m;
  uint4 *const orow = rows + (int64_t)col * A.m;
  uint32_t *const ocode = codes + (int64_t)col * A.m;
  // every wave runs the workgroup's trip count (the flagged draws are resolved wave-wide): lanes past te compute
  // and store nothing
  for (int64_t t0 = tb; t0 < te; t0 += CC_THREADS) {
    const int64_t t = t0 + threadIdx.x;
    const bool act = t < te;
    const int64_t tt = t + cc.t_base;
    const uint32_t tl = (uint32_t)tt, th = (uint32_t)(tt >> 32);
    uint4 qo;
    uint32_t code;
    if (cnt == CI_BLK) {
      uint32_t qd[4], ps, px, RW[CI_BLK / 3];
      cr_block_fast(bkf, fp16, cc, key, tl, th, f, n0, qd, &ps, &px, RW);
      code = cr_block_codes(ps, RW, cc, key, tl, th, f, n0);   // the fast bases' codes (RW dies here)
      if (!act) px = 0;
#ifdef EW_CALIB_NOPX
      px = 0;
#endif
      if (__ballot(px != 0)) {   // wave-uniform
        // list the wave's flagged (lane, base) items
        int total = 0;
        for (uint32_t m = px;;) {
          const uint64_t bal = __ballot(m != 0);
          if (!bal) break;
          if (m) {
            const int pos = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (pos < CC_PX_CAP) cw.item[pos] = (uint16_t)(lane | __builtin_ctz(m) << 6);
            m &= m - 1;
          }
          total += (int)__popcll(bal);
        }
        if (total <= CC_PX_CAP) {
          cw.qd[lane] = make_uint4(qd[0], qd[1], qd[2], qd[3]);
          cw.code[lane] = code;
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          if (lane < total) {
            const uint32_t it = cw.item[lane];
            const int src = (int)(it & 63u), j = (int)(it >> 6);
            const int64_t ts = tt - lane + src;
            const uint32_t x = cr_px_resolve(bkf, t16, fp16, cc, key, (uint32_t)ts, (uint32_t)(ts >> 32), f, n0, j, lim);
            ((uint8_t *)&cw.qd[src])[j] = (uint8_t)x;
            if (x >> 8) atomicOr(&cw.code[src], (x >> 8) << (2 * j));
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          const uint4 q = cw.qd[lane];
          qd[0] = q.x;
          qd[1] = q.y;
          qd[2] = q.z;
          qd[3] = q.w;
          code = cw.code[lane];
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
        } else {
          while (px) {   // the lane's own flagged bases, one by one
            const int j = __builtin_ctz(px);
            px &= px - 1;
            const uint32_t x = cr_px_resolve(bkf, t16, fp16, cc, key, tl, th, f, n0, j, lim);
            const uint32_t sh = 8u * (uint32_t)(j & 3), mk = ~(0xffu << sh), qv = (x & 0xffu) << sh;
            if (j < 4) qd[0] = (qd[0] & mk) | qv; else if (j < 8) qd[1] = (qd[1] & mk) | qv;
            else if (j < 12) qd[2] = (qd[2] & mk) | qv; else qd[3] = (qd[3] & mk) | qv;
            code |= (x >> 8) << (2 * j);
          }
        }
      }
      qo = make_uint4(qd[0], qd[1], qd[2], qd[3]);
    } else {   // a short last block: per triple, per base (as corrupt_triple, into the slot)
      if (!act) continue;
      uint32_t qd[4] = {0, 0, 0, 0}, cd = 0;
#pragma unroll
      for (int g = 0; g < CI_BLK / 3; g++) {
        if (3 * g >= cnt) continue;
        const uint4 r = philox4x32_10(
            make_uint4(tl, th, ((uint32_t)f << 16) | ((uint32_t)n0 / 3u + (uint32_t)g), cc.c3), key);
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const int j = 3 * g + k;
          if (j >= cnt) continue;
          const int n = n0 + j;
          const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : r.z;
          uint32_t amb;
          uint32_t bq = cr_fine_walk(bkf[j * CF_ROW + (w >> (16 + CF_SHIFT))], t16 + j * n_bq, lim, w >> 16, &amb);
          const uint32_t pth = fp16[bq], h2 = w & 0xffffu;
          bool sub;
          if (amb || h2 == pth) {
            const uint32_t x = cq_exact(cc.cum, cc.phred, cc.guide, cc.max_bp, cc.n_bq, cc.k0, cc.k1, cc.c3, tl, th,
                                        f, n, w, bq, amb);
            bq = x & 0xffu;
            sub = x >> 8;
          } else {
            sub = h2 < pth;
          }
          qd[j >> 2] |= (bq + 33u) << (8 * (j & 3));
          if (sub) {
            uint32_t c10 = (r.w >> (10 * k)) & 1023u;
            if (c10 == 1023u)
              c10 = __umulhi(philox4x32_10(make_uint4(tl, th, ((uint32_t)f << 16) | 0x8000u | (uint32_t)n, cc.c3),
                                           key).x, 3u);
            cd |= (c10 % 3u + 1u) << (2 * j);
          }
        }
      }
      qo = make_uint4(qd[0], qd[1], qd[2], qd[3]);
      code = cd;
    }
    if (act) {
      orow[t] = qo;
      ocode[t] = code;
    }
  }
}

// the row pass's LDS (per-file tables, or both files' with one file), 0 when the tables do not fit
static size_t cr_rows_lds(int32_t nf, int64_t rlen, int32_t n_bq) {
  const size_t lds = (size_t)(nf == 2 ? 1 : 2) * rlen * (CB_ROW + 2 * n_bq) + 256 + 16;
  return lds <= 150 * 1024 ? lds : 0;
}

// the corruption rows of one emission (m templates, nf files) on stream `st`, before its writer
static int32_t launch_cr_rows(mh_ctx *ctx, hipStream_t st, int64_t m, int32_t nf, int32_t rlen, const CorruptCfg &cc,
                              uint4 *rows, uint32_t *codes) {
  if (m <= 0) return MH_OK;
  const int64_t NB = (rlen + CI_BLK - 1) / CI_BLK;
  if (m * nf * NB >= ((int64_t)1 << 31)) return arg_fail(ctx, MH_E_STATE, "corruption rows: bad shape");
  CiArgs A{0, 0, m, nullptr, nullptr, nullptr, nullptr, nullptr, {nullptr, nullptr}, nullptr, rlen, nf, 0, cc};
  stage_begin(ctx, "emit_corrupt_rows");
  const size_t lds_c = cc_tables_lds(cc.n_bq) + CC_WAVES * sizeof(CcWave);
  const int64_t gx = (m + CC_PER_WG - 1) / CC_PER_WG;
  if (gx >= INT32_MAX || nf * NB > 65535) return arg_fail(ctx, MH_E_CAPACITY, "corruption rows: grid");
  hipLaunchKernelGGL(k_cr_cols, dim3((unsigned)gx, (unsigned)(nf * NB)), dim3(CC_THREADS), lds_c, st, A, rows, codes);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  return MH_OK;
}

// rows mode: the buffers for an emission of m templates (before any stream waits: a reallocation drains the writers)
static int32_t cr_rows_alloc(mh_ctx *ctx, int64_t m, int32_t nf, int64_t rlen) {
  const int64_t NB = (rlen + CI_BLK - 1) / CI_BLK;
  MH_TRY(ensure(ctx, ctx->cr_rows, (size_t)(m * nf * NB) * 16 + 64));
  MH_TRY(ensure(ctx, ctx->cr_codes, (size_t)(m * nf * NB) * 4 + 64));
  return MH_OK;
}
// rows mode for this emission: the row pass queued on the writer stream `st`, right before its writer (one row set
// serves every unit, in stream order; the pass on a stream of its own beside the previous writer was within noise)
static int32_t cr_rows_prepare(mh_ctx *ctx, hipStream_t st, int64_t m, int32_t nf, int32_t rlen, const CorruptCfg &cc,
                               TArgs &A) {
  const int64_t NB = (rlen + CI_BLK - 1) / CI_BLK;
  if (ctx->cr_rows.cap < (size_t)(m * nf * NB) * 16 + 64 || ctx->cr_codes.cap < (size_t)(m * nf * NB) * 4 + 64)
    return arg_fail(ctx, MH_E_STATE, "corruption rows not allocated");
  uint4 *rows = (uint4 *)ctx->cr_rows.p;
  uint32_t *codes = (uint32_t *)ctx->cr_codes.p;
  MH_TRY(launch_cr_rows(ctx, st, m, nf, rlen, cc, rows, codes));
  A.crow = rows;
  A.ccode = codes;
  A.nb = (int32_t)NB;
  return MH_OK;
}

// the corruption pass over one emission's records (on stream `st`, after its writer)
int32_t launch_cr_inplace(mh_ctx *ctx, hipStream_t st, const HapView &hv, int64_t m, const int64_t *pos0,
                          const int64_t *pos1, const int8_t *fo0, const Rec *recs, const E3 *off, uint2 *crec,
                          char *o1, char *o2, int32_t nf, int32_t lh0, int32_t rlen, const CorruptCfg &cc,
                          bool crec_ready = false) {
  if (m <= 0) return MH_OK;
  int ncu = 0;
  HIPCHK(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  if (ncu <= 0) ncu = 256;
  // per-file workgroups (two files): each stages one file's tables
  const bool pf = nf == 2;
  const size_t lds = (size_t)(pf ? 1 : 2) * rlen * (CB_ROW + 2 * cc.n_bq) + 256 + 16;   // (+16: the walk reads pairs c + 1 <= n_bq + 1)
  const bool lds_tab = lds <= 150 * 1024 && !getenv("MH_CR_GLOBAL");   // MH_CR_GLOBAL: tables from global (tests)
  const int64_t NB = (rlen + CI_BLK - 1) / CI_BLK;
  if (m * nf * NB >= ((int64_t)1 << 31)) return arg_fail(ctx, MH_E_CAPACITY, "too many reads in one emission for the corruption pass");
  const int per_cu = lds_tab ? (lds <= 78 * 1024 ? 2 : 1) : 2;   // 1024-thread workgroups
  // per-file workgroups of 512 threads (4 waves per SIMD, up to 128 VGPRs: the full-block path's phases keep their
  // fifteen LDS reads in flight); at 1024 threads (64 VGPRs) that path spills and takes 8.3 instead of 5.6-5.8 ms per
  // chr1 unit (profiles/r03/experiments_r03.txt)
  const int thr = lds_tab && pf ? 512 : CI_THREADS;
  int64_t grid = std::min<int64_t>((int64_t)ncu * per_cu, (m * nf * NB + thr - 1) / thr);
  if (grid < 1) grid = 1;
  if (pf) grid = (grid + 1) & ~(int64_t)1;   // even: workgroup pairs (file 0, file 1)
  CiArgs A{hv.p_min, hv.hap_len, m, pos0, pos1, fo0, recs, off, {o1, o2}, crec, rlen, nf, lh0, cc};
  stage_begin(ctx, "emit_corrupt");
  if (!crec_ready) {   // (the fused writer wrote the record words itself)
    hipLaunchKernelGGL(k_cr_recs, dim3(grid_for(m, 256, INT32_MAX)), dim3(256), 0, st, A, crec);
    HIPCHK(ctx, hipGetLastError());
  }
  if (lds_tab && pf)
    hipLaunchKernelGGL((k_cr_inplace<true, true, 512>), dim3((unsigned)grid), dim3(512), lds, st, A);
  else if (lds_tab)
    hipLaunchKernelGGL((k_cr_inplace<true, false, CI_THREADS>), dim3((unsigned)grid), dim3(CI_THREADS), lds, st, A);
  else
    hipLaunchKernelGGL((k_cr_inplace<false, false, CI_THREADS>), dim3((unsigned)grid), dim3(CI_THREADS), 0, st, A);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  return MH_OK;
}

// ---- rpc.generate_read facade: per-read text into host-visible buffers ------------------------------------
__global__ void k_rb_measure(HapView h, int64_t n, const int64_t *p, const int64_t *l, int64_t *pos, int64_t *n0,
                             int64_t *n1, int64_t *lens, int32_t *err) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (p[i] < h.p_min || l[i] < 1) {
    atomicOr(err, 1);
    lens[3 * i] = lens[3 * i + 1] = lens[3 * i + 2] = 0;
    pos[i] = n0[i] = n1[i] = -1;
    return;
  }
  ReadInfo r;
  read_info(h, p[i], l[i], r);
  pos[i] = r.pos;
  n0[i] = r.n0;
  n1[i] = r.n1;
  lens[3 * i] = r.cigar_len;
  lens[3 * i + 1] = r.vlist_len;
  lens[3 * i + 2] = r.seq_len;
}
__global__ void k_rb_write(HapView h, int64_t n, const int64_t *p, const int64_t *l, const int64_t *offs, char *cigar,
                           char *vlist, char *seq) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || p[i] < h.p_min || l[i] < 1) return;
  ReadInfo r;
  read_info(h, p[i], l[i], r);
  write_cigar(cigar + offs[3 * i], h, p[i], l[i], r);
  write_vlist(vlist + offs[3 * i + 1], h, r);
  char *d = seq + offs[3 * i + 2];
  for (int k = 0; k < r.seq_len; k++) d[k] = (char)h.hap[r.hap_a + k];
}

HapView view_of(const Hap &h) {
  return HapView{(const int64_t *)h.keys.p, (const int64_t *)h.ps.p, (const int64_t *)h.pr.p,
                 (const int64_t *)h.oplen.p, (const uint8_t *)h.op.p, h.n_nodes, (const uint8_t *)h.hap.p,
                 (const uint8_t *)h.rc.p, (const int32_t *)h.bkt.p, (const Node16 *)h.nd.p, h.n_bkt, h.p_min,
                 h.hap_len, (const int64_t *)h.nrun_s.p, (const int64_t *)h.nrun_e.p, h.n_runs};
}

}  // namespace

#ifdef EW_PROF
extern "C" int mh_ew_prof(unsigned long long *out) {   // the sums since the last call (then zeroed)
  unsigned long long z[16] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ew_prof), sizeof(z)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(ew_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif


int32_t count_kept(mh_ctx *ctx, const Hap &h, int64_t t_begin, int64_t t_end, int64_t *out_kept) {
  auto tit = ctx->tsets.find(ctx->cur_tpl);
  if (tit == ctx->tsets.end() || !tit->second.valid)
    return arg_fail(ctx, MH_E_STATE, "no templates: call mh_sample_templates / mh_use_templates first");
  const TplSet &tp = tit->second;
  if (t_end > tp.n) t_end = tp.n;
  *out_kept = 0;
  if (t_begin >= t_end) return MH_OK;
  const int64_t m = t_end - t_begin;
  hipStream_t st = ctx->stream;
  MH_TRY(ensure(ctx, ctx->scan_partials, sizeof(int64_t) * scan_partials_count(m) + 64));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int64_t *tot = (int64_t *)ctx->d_small.p;
  HIPCHK(ctx, device_reduce<int64_t>(st, m, LoadKeep{view_of(h), (const int64_t *)tp.pos0.p + t_begin,
                                                     (const int64_t *)tp.pos1.p + t_begin, m, tp.rlen},
                                     OpSum{}, (int64_t)0, (int64_t *)ctx->scan_partials.p, tot));
  HIPCHK(ctx, hipMemcpyAsync(out_kept, tot, 8, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  return MH_OK;
}

// Sum of digits(c) for c = 1..K (host side of digit_sum)
static int64_t digit_sum_host(int64_t K) {
  if (K <= 0) return 0;
  int nd = 1;
  for (int64_t v = K; v >= 10; v /= 10) nd++;
  int64_t rep = 0;
  for (int i = 0; i < nd; i++) rep = rep * 10 + 1;
  return (K + 1) * nd - rep;
}

// dynamic LDS of k_emit_tiles: metadata, windows, qname buffers, T, seam chunks, dump
// qname rows: a multiple of 16 bytes plus 4 (an odd number of dwords), so wave 0's lanes (one qname row per template)
// writing the same column land on 32 different LDS banks instead of 8
constexpr int32_t ED_QPAD = 4;
// the direct writer's instantiation: CR mode (0 perfect, 1 in-place corruption after it, 2 corruption rows), one or
// two files
using EwKernel = void (*)(TArgs, QHead);
static EwKernel ew_kernel(int cr, bool two) {
  return cr == 2 ? (two ? k_emit_tiles<2, 4, 2, 3> : k_emit_tiles<1, 8, 2, 3>)
         : cr == 1 ? (two ? k_emit_tiles<2, 4, 1, 3> : k_emit_tiles<1, 8, 1, 3>)
                   : (two ? k_emit_tiles<2, 4, 0, 3> : k_emit_tiles<1, 8, 0, 3>);
}

static size_t ed_lds_bytes(int32_t win_stride, int32_t qstride, int64_t rlen, int nf, bool rows) {
  const bool staged = !rows;   // (rows: the seam chunks stored by the seam pass, no LDS for them)
  const size_t TS = (size_t)((rlen + 4 + 15) / 16 * 16);   // CR 2: a T per record (emit_tile)
  return ((sizeof(DMeta) * ED_T + ED_PAD + 15) / 16) * 16 + (size_t)ED_T * 2 * win_stride + ED_PAD +
         (size_t)ED_T * qstride + ED_PAD + (size_t)((rlen + 4 + 2 * ED_PAD + 15) / 16 * 16) +
         (staged ? (size_t)nf * ED_T * 4 * 16 : 0) + 16 + (rows ? ED_PAD + (size_t)nf * ED_T * TS + 16 : 0);
}

int32_t emit_reads(mh_ctx *ctx, const Hap &h, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                   int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end, int64_t cnt_base,
                   bool prepare_only, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2) {
  auto tit = ctx->tsets.find(ctx->cur_tpl);
  if (tit == ctx->tsets.end() || !tit->second.valid)
    return arg_fail(ctx, MH_E_STATE, "no templates: call mh_sample_templates / mh_use_templates first");
  const TplSet &tp = tit->second;
  hipStream_t st = ctx->stream;
  if (t_end < 0 || t_end > tp.n) t_end = tp.n;
  if (t_begin > t_end) t_begin = t_end;
  const int64_t m = t_end - t_begin;
  const int64_t *pos0 = (const int64_t *)tp.pos0.p + t_begin, *pos1 = (const int64_t *)tp.pos1.p + t_begin;
  const int8_t *fo0 = (const int8_t *)tp.fo0.p + t_begin;
  const int64_t rlen = tp.rlen;
  std::string prefix = std::string("@") + serial_stub + ":";
  std::string mid = std::string("|") + chrom + "|" + std::to_string(cpy);
  if (prefix.size() + mid.size() > 4000) return arg_fail(ctx, MH_E_ARG, "sample/chrom names too long");
  // prepare_only with null outputs: return without waiting for the measure pass (its totals are read back when the
  // unit's writer is queued), so a batch's measure passes run back to back with no host round trip between them
  const bool defer = prepare_only && !out_kept;
  if (!defer) {
    *out_kept = 0;
    *out_b1 = 0;
    *out_b2 = 0;
  }
  if (m == 0) return MH_OK;
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  char *small = (char *)ctx->d_small.p;
  int32_t *err = (int32_t *)(small + 36);
  char *d_prefix = small + 256;
  char *d_mid = small + 256 + 4096;
  QFixed q{d_prefix, d_mid, (int32_t)prefix.size(), (int32_t)mid.size()};
  HapView hv = view_of(h);
  // the direct writer (corruption too; mh_set_emit_mode(1) forces the LDS-image writer): record offsets from per-tile
  // prefixes; the LDS-image writer reads per-template offsets
  const bool direct = !ctx->emit_lds_only;
  const int64_t ntiles = (m + ED_T - 1) / ED_T;

  // ---- measure + tile prefixes (skipped when mh_emit_prepare already ran them for this unit) ------------------------
  EmitPrep &pp = tp.prep;
  const bool have_prep = !prepare_only && pp.valid && pp.slot == slot && pp.t_begin == t_begin && pp.t_end == t_end &&
                         pp.cnt_base == cnt_base && pp.prefix == prefix && pp.mid == mid && pp.direct == direct;
  if (pp.valid && !have_prep) {   // a stale preparation: its buffer set is free again
    ctx->eset[pp.set].prepared = false;
    pp.valid = false;
  }
  int32_t set;
  E3 ht;
  int32_t hm4[4] = {0, 0, 0, 0};   // max record length + 20, -, -, longest reads part + '\n'
  // the scans' totals (kept, bytes without the cnt digits) -> the emission's totals
  auto totals = [&](const E3 &t) {
    const int64_t ds = digit_sum_host(cnt_base + t.kept) - digit_sum_host(cnt_base);
    return E3{t.kept, t.b1 + ds, t.b2 + ds};
  };
  stage_begin(ctx, "emit");
  // what the writer waits for on the main stream: everything queued there so far, or (a deferred preparation) only
  // this unit's measure pass and tile scan — not the measure passes of the units prepared after it
  hipEvent_t writer_dep = nullptr;
  if (have_prep) {
    set = pp.set;
    if (pp.deferred) {   // the measure pass's totals, copied to the set's pinned readback
      const EmitSet &es = ctx->eset[set];
      writer_dep = es.rb;
      SYNCCHK(ctx, hipEventSynchronize(es.rb));
      std::memcpy(&ht, es.h_stat, sizeof(E3));
      std::memcpy(hm4, (const char *)es.h_stat + 32, sizeof(hm4));
      ht = totals(ht);
      pp.deferred = false;
    } else {
      ht = E3{pp.ht.kept, pp.ht.b1, pp.ht.b2};
      std::memcpy(hm4, pp.hm4, sizeof(hm4));
    }
    pp.valid = false;
  } else {
    // this unit's buffer set; the writer that last read it (N_ESET units ago) must be done before the measure
    // refills it
    set = ctx->eset_i;
    EmitSet &es = ctx->eset[set];
    if (es.prepared) {
      stage_end(ctx);
      return arg_fail(ctx, MH_E_STATE, "more units prepared than emission buffer sets (emit the prepared units first)");
    }
    ctx->eset_i = (ctx->eset_i + 1) % mh_ctx::N_ESET;
    if (es.busy) HIPCHK(ctx, hipStreamWaitEvent(st, es.done, 0));
    if (m > ctx->eset_max_m) ctx->eset_max_m = m;
    const int64_t mm = ctx->eset_max_m, mt = (mm + ED_T - 1) / ED_T;
    MH_TRY(ensure(ctx, es.recs, sizeof(Rec) * mm));
    MH_TRY(ensure(ctx, es.tsum, sizeof(int4) * (size_t)mt));
    MH_TRY(ensure(ctx, es.tpre, sizeof(E3) * (size_t)mt));
    if (!direct) MH_TRY(ensure(ctx, es.off, sizeof(E3) * (m + 1)));
    if (ctx->corrupt_on) MH_TRY(ensure(ctx, es.crrec, 16 * (size_t)m + 64));   // 8 bytes per record
    MH_TRY(ensure(ctx, ctx->scan_partials, scan_lb_scratch_bytes<E3>(direct ? ntiles : m + 1)));
    MH_TRY(ensure(ctx, es.stat, 64));
    char *stat = (char *)es.stat.p;        // per set: a deferred readback must not see the next unit's totals
    E3 *tot = (E3 *)stat;                  // [0, 24)
    int32_t *max_rec = (int32_t *)(stat + 32);   // [32, 48); the overflow area's fill at 48
    HIPCHK(ctx, hipMemsetAsync(stat, 0, 64, st));
    Rec *recs = (Rec *)es.recs.p;
    stage_begin(ctx, "emit_measure");
    hipLaunchKernelGGL(k_emit_measure, dim3(grid_for(m, 256, INT32_MAX)), dim3(256), 0, st, hv, m, pos0, pos1, fo0,
                       rlen, q, (int32_t)ctx->corrupt_on, recs, (int4 *)es.tsum.p, max_rec,
                       tp.has_n0 ? (const int32_t *)tp.n0.p + t_begin : nullptr);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    stage_begin(ctx, "emit_scan");
    if (direct)
      HIPCHK(ctx, device_scan_sum<E3>(st, ntiles, LoadTile{(const int4 *)es.tsum.p, ntiles},
                                      StoreTile{(E3 *)es.tpre.p}, ctx->scan_partials.p, tot));
    else
      HIPCHK(ctx, device_scan_sum<E3>(st, m + 1, LoadRec{recs, m}, StoreOff{(E3 *)es.off.p, cnt_base},
                                      ctx->scan_partials.p, tot));
    stage_end(ctx);
    if (defer) {
      // the totals (stat + 0) and the maxima (stat + 32) in one copy: a small copy costs a blit launch
      HIPCHK(ctx, hipMemcpyAsync(es.h_stat, stat, 48, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipEventRecord(es.rb, st));
    } else {
      int64_t *hs = pinned_small(ctx);
      if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
      HIPCHK(ctx, hipMemcpyAsync(hs, stat, 48, hipMemcpyDeviceToHost, st));   // totals at + 0, maxima at + 32
      SYNCCHK(ctx, hipStreamSynchronize(st));
      std::memcpy(&ht, hs, sizeof(E3));
      std::memcpy(hm4, hs + 4, sizeof(hm4));
      ht = totals(ht);
    }
    if (prepare_only) {
      stage_end(ctx);
      pp.valid = true;
      pp.set = set;
      pp.slot = slot;
      pp.t_begin = t_begin;
      pp.t_end = t_end;
      pp.cnt_base = cnt_base;
      pp.prefix = prefix;
      pp.mid = mid;
      pp.direct = direct;
      pp.deferred = defer;
      es.prepared = true;
      if (!defer) {
        pp.ht = E3h{ht.kept, ht.b1, ht.b2};
        std::memcpy(pp.hm4, hm4, sizeof(hm4));
        *out_kept = ht.kept;
        *out_b1 = ht.b1;
        *out_b2 = write_fastq2 ? ht.b2 : 0;
      }
      return MH_OK;
    }
  }
  EmitSet &es = ctx->eset[set];
  es.prepared = false;
  const Rec *recs = (const Rec *)es.recs.p;
  const int32_t hmax = hm4[0], hslot = hm4[3];

  // ---- the writer ------------------------------------------------------------------------------------------------
  // arenas: append after what is already there
  const int64_t need1 = ctx->used1 + ht.b1, need2 = ctx->used2 + (write_fastq2 ? ht.b2 : 0);
  MH_TRY(ensure_keep(ctx, ctx->out1, need1 + 64, ctx->used1));
  if (write_fastq2) MH_TRY(ensure_keep(ctx, ctx->out2, need2 + 64, ctx->used2));

  int32_t cap = 16 * 1024;
  while (cap < hmax) cap *= 2;
  if (cap > 64 * 1024) {
    stage_end(ctx);
    return arg_fail(ctx, MH_E_CAPACITY, "a FASTQ record exceeds 64 KiB");
  }
  const int32_t win_stride = (int32_t)(((rlen + 31) / 16) * 16);
  size_t lds = ((sizeof(TplMeta) * EW_T + 15) / 16) * 16 + (size_t)EW_T * 2 * win_stride + 2 * (size_t)(cap + 16);
  CorruptCfg cc{0, nullptr, nullptr, 0, 0, 0, 0, 0, 0};
  if (ctx->corrupt_on && es.crrec.cap < 16 * (size_t)m + 64) {   // corruption switched on after this unit's measure
    MH_TRY(sync_writers(ctx));
    MH_TRY(ensure(ctx, es.crrec, 16 * (size_t)m + 64));
  }
  if (ctx->corrupt_on) {
    if (rlen > ctx->corrupt_max_bp) {
      stage_end(ctx);
      return arg_fail(ctx, MH_E_ARG, "read length exceeds the BQ model's max_bp");
    }
    cc = corrupt_cfg(ctx, unit_key, t_begin);
  }
  if (lds > 160 * 1024) {
    stage_end(ctx);
    return arg_fail(ctx, MH_E_CAPACITY, "read length too large for the LDS staging layout");
  }
  char *o1 = (char *)ctx->out1.p + ctx->used1;
  char *o2 = write_fastq2 ? (char *)ctx->out2.p + ctx->used2 : nullptr;
  const int32_t head = (int32_t)(((q.prefix_len + q.mid_len + 10 + 16) + 15) / 16 * 16);
  // qname buffer per template (emit_tile): head room, then the reads part (hslot: the longest reads part + '\n' of
  // the unit, from the measure pass)
  const int32_t qstride = head + (hslot > 16 ? (hslot + 15) / 16 * 16 : 16) + 32 + ED_QPAD;
  const bool cr_rows = ctx->corrupt_on && cr_rows_lds(write_fastq2 ? 2 : 1, rlen, ctx->corrupt_n_bq);
  const size_t lds_d = ed_lds_bytes(win_stride, qstride, rlen, write_fastq2 ? 2 : 1, cr_rows);
  QHead qh{};
  const bool head_fits = prefix.size() + mid.size() <= sizeof(qh.w);
  if (head_fits) {
    std::string pm = prefix + mid;
    std::memcpy(qh.w, pm.data(), pm.size());
    qh.lp = (int32_t)prefix.size();
    qh.lm = (int32_t)mid.size();
  }
  if (direct && head_fits && win_stride <= 16 * 3 * ED_GMAX && lds_d <= 64 * 1024 &&
      cnt_base + m < (int64_t)UINT32_MAX) {
    if (cr_rows) MH_TRY(cr_rows_alloc(ctx, m, write_fastq2 ? 2 : 1, rlen));
    // the direct writer, queued on the writer stream: the call returns while it runs, so the next unit's measure pass
    // and the next job's sampling overlap it
    if (!writer_dep) {
      HIPCHK(ctx, hipEventRecord(ctx->ev_ready, st));
      writer_dep = ctx->ev_ready;
    }
    HIPCHK(ctx, hipStreamWaitEvent(ctx->wstream, writer_dep, 0));
    ctx->stage_stream = ctx->wstream;
    TArgs A{hv, m, pos0, pos1, fo0, recs, (const E3 *)es.tpre.p, {(char *)ctx->out1.p, (char *)ctx->out2.p},
            {ctx->used1, ctx->used2}, cnt_base, (uint2 *)es.crrec.p, (int32_t)rlen, win_stride, head,
            qstride};
    if (cr_rows) MH_TRY(cr_rows_prepare(ctx, ctx->wstream, m, write_fastq2 ? 2 : 1, (int32_t)rlen, cc, A));
    stage_begin(ctx, "emit_write");   // (after the row pass: the stage times the writer alone)
    auto kfn = ew_kernel(cr_rows ? 2 : ctx->corrupt_on ? 1 : 0, write_fastq2);
    hipLaunchKernelGGL(kfn, dim3((unsigned)ntiles), dim3(ED_THREADS), lds_d, ctx->wstream, A, qh);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    hipStream_t tail = ctx->wstream;   // the stream whose last work is this unit's last
    if (ctx->corrupt_on && !cr_rows)   // (tables too large for the row pass's LDS): in place after the writer
      MH_TRY(launch_cr_inplace(ctx, tail, hv, m, pos0, pos1, fo0, recs, nullptr, (uint2 *)es.crrec.p,
                               (char *)ctx->out1.p, (char *)ctx->out2.p, write_fastq2 ? 2 : 1,
                               (int32_t)(prefix.size() + mid.size()), (int32_t)rlen, cc, true));
    stage_end(ctx);   // "emit"
    ctx->stage_stream = nullptr;
    HIPCHK(ctx, hipEventRecord(es.done, tail));
    HIPCHK(ctx, hipEventRecord(ctx->ev_writer, tail));
    MH_TRY(mark_used(ctx, h.used, h.used_set));     // the haplotype and the templates stay live until then
    MH_TRY(mark_used(ctx, tp.used, tp.used_set));
    es.busy = true;
    ctx->writer_pending = true;
  } else {
    // LDS-image writer: the fallback (very long qnames or names; synchronous, main stream); per-template offsets
    if (direct) {
      MH_TRY(ensure(ctx, es.off, sizeof(E3) * (m + 1)));
      MH_TRY(ensure(ctx, ctx->scan_partials, scan_lb_scratch_bytes<E3>(m + 1)));
      HIPCHK(ctx, device_scan_sum<E3>(st, m + 1, LoadRec{recs, m}, StoreOff{(E3 *)es.off.p, cnt_base},
                                      ctx->scan_partials.p, (E3 *)((char *)ctx->d_small.p + 128)));
    }
    const E3 *off = (const E3 *)es.off.p;
    HIPCHK(ctx, hipMemsetAsync(small + 32, 0, 16, st));
    HIPCHK(ctx, hipMemcpyAsync(d_prefix, prefix.data(), prefix.size(), hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_mid, mid.data(), mid.size(), hipMemcpyHostToDevice, st));
    stage_begin(ctx, "emit_write");
    const int64_t nblk = (m + EW_T - 1) / EW_T;
    hipLaunchKernelGGL(k_emit_write, dim3((unsigned)nblk), dim3(EW_THREADS), lds, st, hv, m,
                       pos0, pos1, fo0, rlen, q, recs, off, o1, o2, write_fastq2, cap, win_stride,
                       (int32_t)ctx->corrupt_on, err);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    if (ctx->corrupt_on)
      MH_TRY(launch_cr_inplace(ctx, st, hv, m, pos0, pos1, fo0, recs, off, (uint2 *)es.crrec.p, o1, o2,
                               write_fastq2 ? 2 : 1,
                               (int32_t)(prefix.size() + mid.size()), (int32_t)rlen, cc));
    int32_t herr = 0;
    HIPCHK(ctx, hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    stage_end(ctx);
    if (herr) return arg_fail(ctx, MH_E_CAPACITY, "FASTQ record larger than the LDS staging image");
  }
  ctx->used1 += ht.b1;
  if (write_fastq2) ctx->used2 += ht.b2;
  *out_kept = ht.kept;
  *out_b1 = ht.b1;
  *out_b2 = write_fastq2 ? ht.b2 : 0;
  return MH_OK;
}

// ---- the single-pass writer's host side -----------------------------------------------------------------------
using EfKernel = void (*)(TArgs, QHead);
static EfKernel ef_kernel(int cr, bool two) {
  return cr == 2 ? (two ? k_emit_fused<2, 4, 2, 3> : k_emit_fused<1, 8, 2, 3>)
                 : (two ? k_emit_fused<2, 4, 0, 3> : k_emit_fused<1, 8, 0, 3>);
}
static int32_t ndig_host(int64_t v) {
  int32_t d = 1;
  for (; v >= 10; v /= 10) d++;
  return d;
}

int32_t emit_unit_async(mh_ctx *ctx, const Hap &h, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, bool *queued) {
  *queued = false;
  auto tit = ctx->tsets.find(ctx->cur_tpl);
  if (tit == ctx->tsets.end() || !tit->second.valid)
    return arg_fail(ctx, MH_E_STATE, "no templates: call mh_sample_templates / mh_use_templates first");
  const TplSet &tp = tit->second;
  const int64_t m = tp.n, rlen = tp.rlen;
  const int32_t nf = write_fastq2 ? 2 : 1;
  const std::string prefix = std::string("@") + serial_stub + ":";
  const std::string mid = std::string("|") + chrom + "|" + std::to_string(cpy);
  // what the single-pass writer covers (the rest takes emit_reads: the LDS-image writer, long names, reads past
  // the windows the splice bounded, the in-place corruption)
  if (ctx->emit_lds_only || ctx->emit_two_pass || !h.bound_valid || m >= (int64_t)UINT32_MAX) return MH_OK;
  int w = 0;
  while (w < PB_NW && PB_W[w] < rlen) w++;
  QHead qh{};
  if (w == PB_NW || prefix.size() + mid.size() > sizeof(qh.w)) return MH_OK;
  const bool cr_rows = ctx->corrupt_on && cr_rows_lds(nf, rlen, ctx->corrupt_n_bq);
  if (ctx->corrupt_on && (!cr_rows || rlen > ctx->corrupt_max_bp)) return MH_OK;
  // a read's qname part: '|' s '|' POS '|' rlen '|' + its nodes' CIGAR and v_list bytes (the splice's bound) + '|'
  const int32_t part_b = 3 + std::max(ndig_host(h.pos_max), 2) + 1 + ndig_host(rlen) + 1 + 1 + h.part_w[w];
  const int32_t hslot = 2 * part_b + 1;   // both reads' parts + '\n'
  const int32_t win_stride = (int32_t)(((rlen + 31) / 16) * 16);
  const int32_t head = (int32_t)(((prefix.size() + mid.size() + 10 + 16) + 15) / 16 * 16);
  const int32_t hrow = (hslot + 15) / 16 * 16;
  const int32_t qstride = head + hrow + 32 + ED_QPAD;
  const size_t lds_d = ed_lds_bytes(win_stride, qstride, rlen, nf, cr_rows);
  if (win_stride > 16 * 3 * ED_GMAX || lds_d > 64 * 1024) return MH_OK;
  // the default: the measure pass and the tile scan queued on the main stream, the writer on the writer stream, the
  // unit's offsets and totals passed on the device (no readback); mh_set_emit_mode(3): the single-pass writer
  const bool single = ctx->emit_single;
  if (!single && m > 0 && ctx->eset[ctx->eset_i].prepared) return MH_OK;   // (a prepared unit holds the next set)
  *queued = true;
  if ((int64_t)ctx->lazy.size() >= mh_ctx::LZ_SLOTS) MH_TRY(lazy_resolve(ctx));   // (the result slots are full)
  if (m == 0) {
    ctx->lazy.push_back(mh_ctx::LazyUnit{-1, ctx->lazy_gen, {0, 0, 0}});
    return MH_OK;
  }
  if (!ctx->h_lazy) {
    if (hipHostMalloc((void **)&ctx->h_lazy, 64 * (size_t)mh_ctx::LZ_SLOTS,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      ctx->h_lazy = nullptr;
      return arg_fail(ctx, MH_E_OOM, "pinned host memory");
    }
    void *d = nullptr;
    HIPCHK(ctx, hipHostGetDevicePointer(&d, ctx->h_lazy, 0));
    ctx->d_lazy = (int64_t *)d;
  }
  MH_TRY(ensure(ctx, ctx->d_cur, 32 * (size_t)(mh_ctx::LZ_SLOTS + 1)));
  // arenas: room for the chain's upper bound (every record at the bound: the longest qname part twice, both reads)
  if (!ctx->chain_open) {
    ctx->used_ub1 = ctx->used1;
    ctx->used_ub2 = ctx->used2;
  }
  const int64_t rec_b = (int64_t)(prefix.size() + mid.size()) + ndig_host(m) + hslot + 2 * rlen + 5;
  const int64_t add = m * rec_b;
  // a growth reserves for the rest of the sampled batch too (its units' draws bound their templates), by an eighth
  // more, not by half: one reallocation per batch size instead of one every few units, and no superseded arenas
  // piling up in the device block cache
  ctx->batch_left = std::max<int64_t>(0, ctx->batch_left - tp.n_draws);
  const int64_t rest = ctx->batch_left * rec_b;
  if ((int64_t)ctx->out1.cap < ctx->used_ub1 + add + 64)
    MH_TRY(ensure_keep(ctx, ctx->out1, ctx->used_ub1 + add + rest + 64, ctx->used_ub1, 3));
  if (write_fastq2 && (int64_t)ctx->out2.cap < ctx->used_ub2 + add + 64)
    MH_TRY(ensure_keep(ctx, ctx->out2, ctx->used_ub2 + add + rest + 64, ctx->used_ub2, 3));
  const int64_t ntiles = (m + ED_T - 1) / ED_T;
  const size_t lb_need = 64 + 48 * (size_t)ntiles + 64;
  int32_t set = -1;
  if (single) {
    MH_TRY(ensure(ctx, ctx->fused_lb, lb_need));
  } else {
    set = ctx->eset_i;
    EmitSet &es = ctx->eset[set];
    ctx->eset_i = (ctx->eset_i + 1) % mh_ctx::N_ESET;
    if (m > ctx->eset_max_m) ctx->eset_max_m = m;
    const int64_t mm = ctx->eset_max_m, mt = (mm + ED_T - 1) / ED_T;
    MH_TRY(ensure(ctx, es.recs, sizeof(Rec) * mm));
    MH_TRY(ensure(ctx, es.tsum, sizeof(int4) * (size_t)mt));
    MH_TRY(ensure(ctx, es.tpre, sizeof(E3) * (size_t)mt));
    MH_TRY(ensure(ctx, es.stat, 64));
    MH_TRY(ensure(ctx, ctx->scan_partials, scan_lb_scratch_bytes<E3>(ntiles)));
  }
  CorruptCfg cc{0, nullptr, nullptr, 0, 0, 0, 0, 0, 0};
  if (cr_rows) {
    cc = corrupt_cfg(ctx, unit_key, 0);
    MH_TRY(cr_rows_alloc(ctx, m, nf, rlen));
  }
  // (every allocation above may drain the writers; from here on nothing does)
  const std::string pm = prefix + mid;
  std::memcpy(qh.w, pm.data(), pm.size());
  qh.lp = (int32_t)prefix.size();
  qh.lm = (int32_t)mid.size();
  const int64_t seq = ctx->lazy_seq;
  const int32_t rslot = (int32_t)(seq % mh_ctx::LZ_SLOTS);
  int64_t *d_cur = (int64_t *)ctx->d_cur.p;
  hipStream_t ws = ctx->wstream;
  uint32_t tbase = 0, epoch = 0;
  if (single) HIPCHK(ctx, lb_reserve(ws, ctx->fused_lb.p, lb_need, (uint32_t)ntiles, &tbase, &epoch));
  TArgs A{};
  A.h = view_of(h);
  A.m = m;
  A.pos0 = (const int64_t *)tp.pos0.p;
  A.pos1 = (const int64_t *)tp.pos1.p;
  A.fo0 = (const int8_t *)tp.fo0.p;
  A.arena[0] = (char *)ctx->out1.p;
  A.arena[1] = (char *)ctx->out2.p;
  A.used[0] = ctx->used1;
  A.used[1] = ctx->used2;
  A.cnt_base = 0;
  A.rlen = (int32_t)rlen;
  A.win_stride = win_stride;
  A.head = head;
  A.qstride = qstride;
  A.nb = 1;
  A.lb = single ? (uint64_t *)ctx->fused_lb.p : nullptr;
  A.ntiles = ntiles;
  A.tbase = tbase;
  A.epoch = epoch;
  A.fault = scan_fault_device();
  A.cur_in = ctx->chain_open ? d_cur + 4 * (seq % (mh_ctx::LZ_SLOTS + 1)) : nullptr;
  A.cur_out = d_cur + 4 * ((seq + 1) % (mh_ctx::LZ_SLOTS + 1));
  A.res = ctx->d_lazy + 8 * rslot;
  A.cap[0] = (int64_t)ctx->out1.cap;
  A.cap[1] = write_fastq2 ? (int64_t)ctx->out2.cap : 0;
  A.hcap = hrow;
  // the writer waits for what the main stream has queued (this unit's templates: its sampling tail was joined there
  // by tpl_resolve; its measure pass and tile scan), not for any host readback
  stage_begin(ctx, "emit");
  if (!single) {
    EmitSet &es = ctx->eset[set];
    hipStream_t st = ctx->stream;
    if (es.busy) HIPCHK(ctx, hipStreamWaitEvent(st, es.done, 0));   // the writer that last read the set
    char *stat = (char *)es.stat.p;   // (its maxima are not read: the splice's bound sizes the rows)
    stage_begin(ctx, "emit_measure");
    hipLaunchKernelGGL(k_emit_measure, dim3(grid_for(m, 256, INT32_MAX)), dim3(256), 0, st, A.h, m, A.pos0, A.pos1,
                       A.fo0, rlen, QFixed{nullptr, nullptr, qh.lp, qh.lm}, (int32_t)ctx->corrupt_on,
                       (Rec *)es.recs.p, (int4 *)es.tsum.p, (int32_t *)(stat + 32),
                       tp.has_n0 ? (const int32_t *)tp.n0.p : nullptr);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
    stage_begin(ctx, "emit_scan");
    HIPCHK(ctx, device_scan_sum<E3>(st, ntiles, LoadTile{(const int4 *)es.tsum.p, ntiles},
                                    StoreTile{(E3 *)es.tpre.p}, ctx->scan_partials.p, (E3 *)stat));
    stage_end(ctx);
    A.recs = (const Rec *)es.recs.p;
    A.tpre = (const E3 *)es.tpre.p;
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev_ready, ctx->stream));
  HIPCHK(ctx, hipStreamWaitEvent(ws, ctx->ev_ready, 0));
  ctx->stage_stream = ws;
  if (cr_rows) MH_TRY(cr_rows_prepare(ctx, ws, m, nf, (int32_t)rlen, cc, A));
  stage_begin(ctx, "emit_write");
  hipLaunchKernelGGL(single ? ef_kernel(cr_rows ? 2 : 0, write_fastq2 != 0) : ew_kernel(cr_rows ? 2 : 0, write_fastq2),
                     dim3((unsigned)ntiles), dim3(ED_THREADS), lds_d, ws, A, qh);
  HIPCHK(ctx, hipGetLastError());
  stage_end(ctx);
  stage_end(ctx);   // "emit"
  ctx->stage_stream = nullptr;
  if (!single) {
    HIPCHK(ctx, hipEventRecord(ctx->eset[set].done, ws));
    ctx->eset[set].busy = true;
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev_writer, ws));
  MH_TRY(mark_used(ctx, h.used, h.used_set));     // the haplotype and the templates stay live until then
  MH_TRY(mark_used(ctx, tp.used, tp.used_set));
  ctx->writer_pending = true;
  ctx->chain_open = true;
  ctx->used_ub1 += add;
  if (write_fastq2) ctx->used_ub2 += add;
  ctx->lazy_seq = seq + 1;
  ctx->lazy.push_back(mh_ctx::LazyUnit{rslot, ctx->lazy_gen, {0, 0, 0}});
  return MH_OK;
}

int32_t lazy_resolve(mh_ctx *ctx) {
  if (ctx->lazy.empty()) return MH_OK;
  const int32_t rc = sync_writers(ctx);   // (SYNCCHK: a look-back timeout or a bound the writer found wrong fails here)
  if (rc != MH_OK) {   // the queued units' totals and ends are not to be trusted: dropped with the chain
    ctx->lazy.clear();
    ctx->chain_open = false;
    return rc;
  }
  const volatile int64_t *r = ctx->h_lazy;
  for (const auto &u : ctx->lazy) {
    int64_t k = 0, b1 = 0, b2 = 0;
    if (u.slot < 0) {
      k = u.known[0];
      b1 = u.known[1];
      b2 = u.known[2];
    } else {
      const volatile int64_t *q = r + 8 * u.slot;
      k = q[0];
      b1 = q[1];
      b2 = q[2];
      if (u.gen == ctx->lazy_gen) {   // the chain's ends move the arenas
        ctx->used1 = q[3];
        ctx->used2 = q[4];
      }
    }
    ctx->lazy_done.push_back(k);
    ctx->lazy_done.push_back(b1);
    ctx->lazy_done.push_back(b2);
  }
  ctx->lazy.clear();
  ctx->chain_open = false;
  return MH_OK;
}

int32_t read_batch(mh_ctx *ctx, const Hap &h, const int64_t *p, const int64_t *l, int64_t n, int64_t *out_pos,
                   int64_t *out_n0, int64_t *out_n1, char *cigar, int64_t cigar_cap, int64_t *cigar_off,
                   int64_t *cigar_used, char *vlist, int64_t vlist_cap, int64_t *vlist_off, int64_t *vlist_used,
                   char *seq, int64_t seq_cap, int64_t *seq_off, int64_t *seq_used) {
  hipStream_t st = ctx->stream;
  if (n <= 0) {
    *cigar_used = *vlist_used = *seq_used = 0;
    if (cigar_off) cigar_off[0] = 0;
    if (vlist_off) vlist_off[0] = 0;
    if (seq_off) seq_off[0] = 0;
    return MH_OK;
  }
  DevBuf b;
  size_t sz = 8 * (size_t)n * (2 + 3 + 3 + 3) + 64;
  HIPCHK(ctx, hipMalloc(&b.p, sz));
  int64_t *dp = (int64_t *)b.p, *dl = dp + n, *dpos = dl + n, *dn0 = dpos + n, *dn1 = dn0 + n, *lens = dn1 + n,
          *offs = lens + 3 * n;
  int32_t *derr = (int32_t *)(offs + 3 * n);
  HapView hv = view_of(h);
  int32_t herr = 0;
  std::vector<int64_t> hl(3 * n), ho(3 * n);
  int32_t rc = MH_OK;
  char *dtxt = nullptr;
  do {
    if (hipMemcpyAsync(dp, p, 8 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dl, l, 8 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(derr, 0, 4, st) != hipSuccess) {
      rc = hip_fail(ctx, hipGetLastError(), "read_batch upload", __FILE__, __LINE__);
      break;
    }
    hipLaunchKernelGGL(k_rb_measure, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, hv, n, dp, dl, dpos, dn0,
                       dn1, lens, derr);
    if (hipMemcpyAsync(hl.data(), lens, 24 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      rc = hip_fail(ctx, hipGetLastError(), "read_batch measure", __FILE__, __LINE__);
      break;
    }
    if (herr) {
      rc = arg_fail(ctx, MH_E_ARG, "read start before the first node (p < p_min) or non-positive length");
      break;
    }
    int64_t acc[3] = {0, 0, 0};
    for (int64_t i = 0; i < n; i++)
      for (int k = 0; k < 3; k++) {
        ho[3 * i + k] = acc[k];
        acc[k] += hl[3 * i + k];
      }
    *cigar_used = acc[0];
    *vlist_used = acc[1];
    *seq_used = acc[2];
    if (acc[0] > cigar_cap || acc[1] > vlist_cap || acc[2] > seq_cap) {
      rc = arg_fail(ctx, MH_E_CAPACITY, "read_batch text buffers too small");
      break;
    }
    for (int64_t i = 0; i < n; i++) {
      cigar_off[i] = ho[3 * i];
      vlist_off[i] = ho[3 * i + 1];
      seq_off[i] = ho[3 * i + 2];
    }
    cigar_off[n] = acc[0];
    vlist_off[n] = acc[1];
    seq_off[n] = acc[2];
    int64_t tot = acc[0] + acc[1] + acc[2] + 3;
    if (hipMalloc(&dtxt, tot) != hipSuccess) {
      rc = arg_fail(ctx, MH_E_OOM, "read_batch text");
      break;
    }
    char *dc = dtxt, *dv = dtxt + acc[0] + 1, *ds = dv + acc[1] + 1;
    if (hipMemcpyAsync(offs, ho.data(), 24 * n, hipMemcpyHostToDevice, st) != hipSuccess) {
      rc = hip_fail(ctx, hipGetLastError(), "read_batch offsets", __FILE__, __LINE__);
      break;
    }
    hipLaunchKernelGGL(k_rb_write, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, st, hv, n, dp, dl, offs, dc, dv,
                       ds);
    if ((acc[0] && hipMemcpyAsync(cigar, dc, acc[0], hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (acc[1] && hipMemcpyAsync(vlist, dv, acc[1], hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (acc[2] && hipMemcpyAsync(seq, ds, acc[2], hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipMemcpyAsync(out_pos, dpos, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(out_n0, dn0, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(out_n1, dn1, 8 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      rc = hip_fail(ctx, hipGetLastError(), "read_batch write", __FILE__, __LINE__);
      break;
    }
  } while (0);
  if (dtxt) (void)hipFree(dtxt);
  (void)hipFree(b.p);
  return rc;
}

}  // namespace mh
