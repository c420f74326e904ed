// mh_splice.hip — haplotype splice on the device (reference rpc.create_node_list, mitty/simulation/rpc.py:38-116).
//
// The reference walks the variant list with two cursors (samp_pos, ref_pos) and skips a variant whose position is
// before the ref cursor left by the last ACCEPTED variant (rpc.py:55) — a sequential chain.  Here:
//   1. max-scan of variant ends  -> "anchor" = pos >= every earlier end, accepted whatever happened before;
//   2. k_resolve                 -> one thread per anchor walks its (short) run of non-anchors sequentially;
//   3. max-scan of accepted ends -> ref cursor before each variant (accepted ends are strictly increasing);
//   4. sum-scan of (nodes, sample length) -> every node's index and ps, written straight from the scan's Store;
//   5. packed nodes + buckets    -> Node16 copy and the node-search bucket table;
//   6. k_hap_fill                -> haplotype bytes (hap[k] = base at sample position p_min + k) by output position
//                                   from the resident contig / alt pool; k_hap_rc the reverse complement;
//   7. N-run extraction          -> sorted [start, end) runs of 'N' so the N-filter never re-reads bases.
// Node arrays are SoA in HBM: keys (search key, ps+1 for 'D' as rpc.py:127), ps, pr, op, oplen.

#include <cstring>

#include "mh_device.h"
#include "mh_internal.h"
#include "mh_scan.h"
#include "mh_sort.h"

namespace mh {

namespace {

constexpr int64_t ALT_FLAG = (int64_t)1 << 62;

__device__ __forceinline__ int64_t var_end(int64_t pos, uint8_t op, int64_t oplen) {
  return pos + 1 + (op == 'D' ? oplen : 0);
}

struct LoadEnd {
  const int64_t *pos; const uint8_t *op; const int64_t *oplen;
  __device__ int64_t operator()(int64_t i) const { return var_end(pos[i], op[i], oplen[i]); }
};
struct StoreAnchor {
  const int64_t *pos; uint8_t *anchor; int64_t rs;
  __device__ void operator()(int64_t i, int64_t, int64_t excl) const {
    int64_t m = excl > rs ? excl : rs;
    anchor[i] = pos[i] >= m;
  }
};

__global__ void k_resolve(int64_t n, const int64_t *pos, const uint8_t *op, const int64_t *oplen,
                          const uint8_t *anchor, uint8_t *accepted, int64_t rs) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t cur;
  int64_t k;
  if (anchor[i]) {
    accepted[i] = 1;
    cur = var_end(pos[i], op[i], oplen[i]);
    k = i + 1;
  } else if (i == 0) {
    cur = rs;
    k = 0;
  } else {
    return;
  }
  for (; k < n && !anchor[k]; k++) {
    uint8_t a = pos[k] >= cur;
    accepted[k] = a;
    if (a) cur = var_end(pos[k], op[k], oplen[k]);
  }
}

struct LoadAccEnd {
  const int64_t *pos; const uint8_t *op; const int64_t *oplen; const uint8_t *accepted; int64_t rs;
  __device__ int64_t operator()(int64_t i) const { return accepted[i] ? var_end(pos[i], op[i], oplen[i]) : rs; }
};
struct StoreRefBefore {
  int64_t *ref_before; int64_t rs;
  __device__ void operator()(int64_t i, int64_t, int64_t excl) const { ref_before[i] = excl > rs ? excl : rs; }
};

struct NS {
  int64_t nodes, samp;
  __device__ NS operator+(const NS &o) const { return NS{nodes + o.nodes, samp + o.samp}; }
};

struct LoadNS {
  const int64_t *pos; const uint8_t *op; const int64_t *oplen; const uint8_t *accepted; const int64_t *ref_before;
  __device__ NS operator()(int64_t i) const {
    if (!accepted[i]) return NS{0, 0};
    uint8_t o = op[i];
    int64_t delta = (o == 'X') ? pos[i] - ref_before[i] : pos[i] + 1 - ref_before[i];
    int64_t eq = delta > 0 ? 1 : 0;
    int64_t sl = (delta > 0 ? delta : 0) + (o == 'X' ? 1 : (o == 'I' ? oplen[i] : 0));
    return NS{eq + 1, sl};
  }
};

}  // namespace

// The nodes one variant adds from the two cursors (rb = ref_pos, sp = samp_pos; rs = ref_start_pos): rpc.py:66-116's
// snp / insertion / deletion (op selects the rule).  An optional '=' node up to the variant (through its first base
// for 'I' / 'D'), then the variant's node.  src: the '=' node's offset into the region's reference bytes, the
// 'X' / 'I' node's offset into the variant's alt bytes, -1 for 'D'.  Shared by the device splice (StoreNodes) and
// the host entry mh_expand_variant (the plugin API's per-variant helpers).
__host__ __device__ int expand_variant(uint8_t o, int64_t vp, int64_t oplen, int64_t rb, int64_t sp, int64_t rs,
                                       VarNode out[2], int64_t *sp_next, int64_t *rp_next) {
  int n = 0;
  const int64_t delta = (o == 'X') ? vp - rb : vp + 1 - rb;
  int64_t pr_x = rb;
  if (delta > 0) {
    out[n++] = VarNode{sp, rb, delta, rb - rs, (uint8_t)'='};
    sp += delta;
    pr_x = vp;
  }
  if (o == 'X') {
    out[n++] = VarNode{sp, pr_x, 1, 0, (uint8_t)'X'};
    *rp_next = pr_x + 1;
    *sp_next = sp + 1;
  } else if (o == 'I') {
    out[n++] = VarNode{sp, vp + 1, oplen, 1, (uint8_t)'I'};
    *rp_next = vp + 1;
    *sp_next = sp + oplen;
  } else {
    out[n++] = VarNode{sp - 1, vp + 1 + oplen, oplen, -1, (uint8_t)'D'};
    *rp_next = vp + 1 + oplen;
    *sp_next = sp;
  }
  return n;
}

namespace {

struct StoreNodes {
  const int64_t *pos; const uint8_t *op; const int64_t *oplen; const uint8_t *accepted; const int64_t *ref_before;
  const int64_t *alt_off; const int64_t *alt_len;
  int64_t *keys, *ps, *pr, *nl, *src; uint8_t *nop;
  int64_t rs, ref_len; int32_t *err;
  __device__ void operator()(int64_t i, NS, NS excl) const {
    if (!accepted[i]) return;
    const uint8_t o = op[i];
    VarNode v[2];
    int64_t sn, rn;
    const int nn = expand_variant(o, pos[i], oplen[i], ref_before[i], rs + excl.samp, rs, v, &sn, &rn);
    for (int j = 0; j < nn; j++) {
      const int64_t k = excl.nodes + j;
      keys[k] = v[j].op == 'D' ? v[j].ps + 1 : v[j].ps;   // the search key (rpc.py:127)
      ps[k] = v[j].ps; pr[k] = v[j].pr; nop[k] = v[j].op; nl[k] = v[j].oplen;
      if (v[j].op == '=') {
        src[k] = v[j].src;
        if (v[j].src + v[j].oplen > ref_len) atomicOr(err, 1);
      } else if (v[j].op == 'D') {
        src[k] = -1;
      } else {
        src[k] = ALT_FLAG | (alt_off[i] + v[j].src);
        if (alt_len[i] - v[j].src != (v[j].op == 'X' ? 1 : oplen[i])) atomicOr(err, 2);
      }
    }
  }
};

__global__ void k_trailing(int64_t k, int64_t sp, int64_t rp, int64_t rs, int64_t len, int64_t *keys, int64_t *ps,
                           int64_t *pr, int64_t *nl, int64_t *src, uint8_t *nop) {
  keys[k] = sp; ps[k] = sp; pr[k] = rp; nop[k] = '='; nl[k] = len; src[k] = rp - rs;
}

// Haplotype bytes by output position: thread i writes hap[16i, 16i+16).  The node holding sample position x is the
// last node whose key is <= x (the bucket table narrows the search, as in emission); 'D' nodes hold no bytes
// (their key equals the next node's).  Bytes no node covers (possible only before the first node's bytes) are 0.
constexpr int FILL_NODES = 512;   // nodes of one workgroup's span staged in LDS (more: searched in global memory)
constexpr int FILL_Q = 4;         // 16-byte chunks per thread (lane-strided: stores stay coalesced)
constexpr int64_t FILL_SPAN = 256 * 16 * FILL_Q;

// One 16-byte chunk of the haplotype at output offset o0 (sample position x0): node search, then the bytes.
__device__ __forceinline__ void hap_fill_chunk(int64_t o0, int64_t hap_len, int64_t p_min, int64_t n_nodes,
                                               const Node16 *nd, const int64_t *src, const int32_t *bkt,
                                               int64_t n_bkt, const uint8_t *contig, const uint8_t *alt_pool,
                                               uint8_t *hap, bool staged, int64_t lo, int64_t cnt,
                                               const Node16 *s_nd, const int64_t *s_src) {
  const int64_t x0 = p_min + o0;
  int64_t k;   // the last node whose key is <= x0 (-1: none)
  bool global = !staged;
  if (staged) {
    int64_t a = 0, b = cnt;
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (s_nd[mid].key() <= x0) a = mid + 1; else b = mid;
    }
    k = lo + a - 1;
    global = a == 0 && lo > 0;   // below the staged range (not expected): search globally
  }
  if (global) {
    int64_t kb = (x0 - p_min) >> NODE_BKT_SHIFT;
    if (kb >= n_bkt) kb = n_bkt - 1;
    int64_t l2 = bkt[kb], h2 = kb + 1 < n_bkt ? bkt[kb + 1] : n_nodes;
    while (l2 < h2) {
      const int64_t mid = (l2 + h2) >> 1;
      if (nd[mid].key() <= x0) l2 = mid + 1; else h2 = mid;
    }
    k = l2 - 1;
  }
  auto node_at = [&](int64_t q) -> Node16 { return staged && q >= lo && q < lo + cnt ? s_nd[q - lo] : nd[q]; };
  auto src_at = [&](int64_t q) -> int64_t { return staged && q >= lo && q < lo + cnt ? s_src[q - lo] : src[q]; };
  int64_t nk = 0, ne = 0;
  const uint8_t *sp = nullptr;
  if (k >= 0) {
    const Node16 n = node_at(k);
    nk = n.ps();
    ne = nk + (n.code() == 3 ? 0 : n.oplen());
    const int64_t s = src_at(k);
    sp = (s & ALT_FLAG) ? alt_pool + (s & ~ALT_FLAG) : contig + s;
  }
  // the usual case: all 16 bytes inside one node's bytes (no later node starts within them)
  const int64_t kn = k + 1 < n_nodes ? node_at(k + 1).key() : INT64_MAX;
  if (k >= 0 && o0 + 16 <= hap_len && kn > x0 + 15 && x0 >= nk && x0 + 16 <= ne) {
    *(uint4 *)(hap + o0) = load16_unaligned(sp + (x0 - nk));
    return;
  }
  // a chunk meeting several nodes: each node's bytes in it from one 16-byte load, shifted into place
  typedef unsigned __int128 u128;
  const int64_t xe = x0 + (o0 + 16 <= hap_len ? 16 : hap_len - o0);   // end of the chunk's positions
  u128 acc = 0;
  for (int guard = 0; guard < 40; guard++) {   // at most 16 byte-holding nodes (+ 'D' nodes) meet 16 positions
    if (k >= 0) {
      const int64_t a = x0 > nk ? x0 : nk, e = xe < ne ? xe : ne;
      if (e > a) {
        const uint4 v = load16_unaligned(sp + (a - nk));
        u128 V = ((u128)(((uint64_t)v.w << 32) | v.z) << 64) | (((uint64_t)v.y << 32) | v.x);
        const int off = (int)(a - x0), len = (int)(e - a);   // 0 <= off, off + len <= 16
        const u128 m = len >= 16 ? ~(u128)0 : (((u128)1 << (8 * len)) - 1);
        acc |= (V & m) << (8 * off);
      }
    }
    const int64_t kn2 = k + 1 < n_nodes ? node_at(k + 1).key() : INT64_MAX;
    if (kn2 >= xe) break;
    k++;
    const Node16 n = node_at(k);
    nk = n.ps();
    ne = nk + (n.code() == 3 ? 0 : n.oplen());
    const int64_t s = src_at(k);
    sp = (s & ALT_FLAG) ? alt_pool + (s & ~ALT_FLAG) : contig + s;
  }
  const uint64_t lo64 = (uint64_t)acc, hi64 = (uint64_t)(acc >> 64);
  *(uint4 *)(hap + o0) = make_uint4((uint32_t)lo64, (uint32_t)(lo64 >> 32), (uint32_t)hi64, (uint32_t)(hi64 >> 32));
}

// A workgroup fills FILL_SPAN bytes; its nodes (from the last one keyed below its first bucket to the first one
// past its last bucket) are staged in LDS first, so every chunk's search is an LDS binary search.
// ends: the splice's {ps of the first node, ...} (k_splice_ends) and err its error word: a spliced node list with an
// error is not filled (its sources may point anywhere); the host reports the error after its one synchronisation
__global__ void __launch_bounds__(256) k_hap_fill(int64_t hap_len, const int64_t *ends, const int32_t *err,
                                                  int64_t n_nodes, const Node16 *nd,
                                                  const int64_t *src, const int32_t *bkt, int64_t n_bkt,
                                                  const uint8_t *contig, const uint8_t *alt_pool, uint8_t *hap) {
  if (*err) return;
  const int64_t p_min = ends[0];
  __shared__ Node16 s_nd[FILL_NODES];
  __shared__ int64_t s_src[FILL_NODES];
  __shared__ int64_t s_lo, s_hi;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * FILL_SPAN;
  if (tid == 0) {
    int64_t kb0 = b0 >> NODE_BKT_SHIFT, kb1 = ((b0 + FILL_SPAN - 1) >> NODE_BKT_SHIFT) + 1;
    if (kb0 >= n_bkt) kb0 = n_bkt - 1;
    const int64_t lo = bkt[kb0] - 1, hi = kb1 < n_bkt ? (int64_t)bkt[kb1] + 1 : n_nodes;
    s_lo = lo < 0 ? 0 : lo;
    s_hi = hi > n_nodes ? n_nodes : hi;
  }
  __syncthreads();
  const int64_t lo = s_lo, cnt = s_hi - s_lo;
  const bool staged = cnt <= FILL_NODES;   // workgroup-uniform
  if (staged) {
    for (int i = tid; i < cnt; i += 256) {
      s_nd[i] = nd[lo + i];
      s_src[i] = src[lo + i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < FILL_Q; q++) {
    const int64_t o0 = b0 + (int64_t)(q * 256 + tid) * 16;
    if (o0 < hap_len)
      hap_fill_chunk(o0, hap_len, p_min, n_nodes, nd, src, bkt, n_bkt, contig, alt_pool, hap, staged, lo, cnt, s_nd,
                     s_src);
  }
}

// ---- N runs ---------------------------------------------------------------------------------------------------
// A run starts at position k if hap[k]=='N' and hap[k-1] != 'N', and ends (exclusive) at k if hap[k-1]=='N' and
// (k == len or hap[k] != 'N').  'N' found with SWAR over aligned 16-byte loads (the haplotype buffer is padded).
__device__ __forceinline__ uint32_t n_bits4(uint32_t w) {
  const uint32_t t = w ^ 0x4E4E4E4Eu;                                    // zero byte where 'N'
  const uint32_t nz = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;             // bit 7 of each byte: byte != 0
  const uint32_t z = ~nz & 0x80808080u;
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}
// One pass over the haplotype for the run boundaries, 64 positions per thread: boundaries are rare, so each is
// appended to an unsorted list through an atomic counter (cap entries kept, all counted); sorted afterwards.
// Both N-run boundary lists of a haplotype (blockIdx.x: 0 starts, 1 ends; n distinct positions each, n <= NR_LDS)
// sorted in LDS by one workgroup (bitonic over the next power of two, padded with 0xffffffff) and widened to the i64
// lists the measure pass searches: one launch instead of two radix sorts' dozen (a genome has ~50 haplotypes per step,
// each with a few dozen N runs).
constexpr int NR_LDS = 8192;
__global__ void __launch_bounds__(1024) k_nrun_sort_small(const uint32_t *us, const uint32_t *ue, int64_t n,
                                                          int64_t *os, int64_t *oe) {
  __shared__ uint32_t v[NR_LDS];
  const uint32_t *a = blockIdx.x ? ue : us;
  int64_t *o = blockIdx.x ? oe : os;
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = threadIdx.x; i < np; i += blockDim.x) v[i] = i < n ? a[i] : 0xffffffffu;
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = v[i], y = v[l];
          if (((i & k) == 0) == (x > y)) {
            v[i] = y;
            v[l] = x;
          }
        }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < n; i += blockDim.x) o[i] = v[i];
}

// ps of the first node, ps and oplen of the last, into out[0..2] (one readback with the splice's error word)
__global__ void k_splice_ends(const int64_t *ps, const int64_t *nl, int64_t n_nodes, int64_t *out) {
  if (threadIdx.x == 0) {
    out[0] = ps[0];
    out[1] = ps[n_nodes - 1];
    out[2] = nl[n_nodes - 1];
  }
}

__global__ void __launch_bounds__(256) k_widen_u32(const uint32_t *a, int64_t n, int64_t *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a[i];
}

// (positions as u32: the caller refuses haplotypes of 2^32 - 1 bases or more)
__global__ void __launch_bounds__(256) k_nrun_find(const uint8_t *hap, int64_t len, int64_t cap, uint32_t *rs,
                                                   uint32_t *re, unsigned long long *cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t k0 = c * 64;
  if (k0 > len) return;
  uint64_t nm = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 v = *(const uint4 *)(hap + k0 + 16 * q);   // the buffer is padded past len
    const uint64_t m = n_bits4(v.x) | (n_bits4(v.y) << 4) | (n_bits4(v.z) << 8) | (n_bits4(v.w) << 12);
    nm |= m << (16 * q);
  }
  const int64_t valid = len - k0;                            // positions >= len are not 'N'
  if (valid < 64) nm &= (1ull << valid) - 1ull;
  const uint64_t prev = (k0 > 0 && hap[k0 - 1] == 'N') ? 1ull : 0ull;
  const uint64_t sh = (nm << 1) | prev;                       // bit i: hap[k0 + i - 1] == 'N'
  uint64_t pos = ~0ull;                                       // positions k0 + i <= len
  if (valid < 63) pos = (1ull << (valid + 1)) - 1ull;
  uint64_t st = nm & ~sh & pos, en = sh & ~nm & pos;
  while (st) {
    const unsigned long long i = atomicAdd(cnt, 1ull);
    if ((int64_t)i < cap) rs[i] = (uint32_t)(k0 + __builtin_ctzll(st));
    st &= st - 1;
  }
  while (en) {
    const unsigned long long i = atomicAdd(cnt + 1, 1ull);
    if ((int64_t)i < cap) re[i] = (uint32_t)(k0 + __builtin_ctzll(en));
    en &= en - 1;
  }
}

// Reverse complement of the haplotype (readgenerate.py:56,205-206: str.maketrans('ATCGN', 'TAGCN') then [::-1]):
// rc[i] = comp(hap[hap_len - 1 - i]); mate-1 reads are then forward ranges of rc.  16 output bytes per thread.
__global__ void __launch_bounds__(256) k_hap_rc(const uint8_t *hap, int64_t hap_len, uint8_t *rc) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i0 >= hap_len) return;
  if (i0 + 16 <= hap_len) {   // rc[i0, i0 + 16) = complement of hap[hap_len - 16 - i0, hap_len - i0), reversed
    const uint4 v = load16_unaligned(hap + (hap_len - 16 - i0));
    *(uint4 *)(rc + i0) = make_uint4(comp4(__builtin_bswap32(v.w)), comp4(__builtin_bswap32(v.z)),
                                     comp4(__builtin_bswap32(v.y)), comp4(__builtin_bswap32(v.x)));
    return;
  }
  uint32_t w[4] = {0, 0, 0, 0};
  for (int k = 0; k < 16 && i0 + k < hap_len; k++)
    w[k >> 2] |= (uint32_t)hap[hap_len - 1 - (i0 + k)] << (8 * (k & 3));
  *(uint4 *)(rc + i0) = make_uint4(comp4(w[0]), comp4(w[1]), comp4(w[2]), comp4(w[3]));
}

// AoS copy of the node arrays for the emission kernels' random lookups (field ranges checked on the host).
__global__ void __launch_bounds__(256) k_node_pack(int64_t n, const int64_t *ps, const int64_t *pr,
                                                   const int64_t *oplen, const uint8_t *op, Node16 *nd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t o = op[i];
  const uint64_t code = o == 'X' ? 1u : o == 'I' ? 2u : o == 'D' ? 3u : 0u;
  const uint64_t a = (uint64_t)ps[i], b = (uint64_t)pr[i], l = (uint64_t)oplen[i];
  nd[i] = Node16{(a & 0xffffffffffull) | code << 40 | (l & 0x3fffffull) << 42, (b & 0xffffffffffull) | (l >> 22) << 40};
}

__device__ __forceinline__ int32_t pb_ndig(int64_t v) {   // (no 64-bit division: it is a long VALU routine)
  int32_t d = 1;
  for (int64_t p = 10; v >= p && d < 18; p *= 10) d++;
  return d;
}
// Bytes node n adds to a read's qname part under window W (rpc.py:146-147): its CIGAR count and op — a count is
// min(p + l - ps, oplen) - max(0, p - ps) <= min(oplen, l), a deletion's is its length — and, for a variant, its size
// in v_list (X: 0, I: +oplen, D: -oplen) with a comma.
__device__ __forceinline__ int32_t pb_node_cost(const Node16 &n, int32_t W) {
  const int c = n.code();
  const int64_t ol = n.oplen();
  const int32_t cnt = pb_ndig(c == 3 ? ol : (ol < W ? ol : W)) + 1;
  return cnt + (c == 0 ? 0 : c == 1 ? 2 : c == 2 ? pb_ndig(ol) + 1 : pb_ndig(ol) + 2);
}

// The qname-part bound of the single-pass writer (k_emit_fused).  A read at p whose start node is j (key_j <= p <
// key_{j+1}) ends in the last node with key <= p + rlen - 1 < key_{j+1} + rlen - 1 (rpc.py:119-130), so its nodes'
// bytes are at most node j's plus those of every node k > j with key_k <= key_{j+1} + W - 2, W >= rlen; a read inside
// an insertion (rpc.py:152-156) writes '>' off ':' l 'I' instead of its count.  Per window the maximum over j, and the
// largest POS (p - ps + pr < pr + oplen), into out_w[PB_NW] / *out_pos (zeroed).
__global__ void __launch_bounds__(256) k_part_bound(const Node16 *nd, int64_t n, int32_t *out_w,
                                                    unsigned long long *out_pos) {
  __shared__ int32_t s_w[4][PB_NW];
  __shared__ unsigned long long s_p[4];
  int32_t best[PB_NW];
  unsigned long long pm = 0;
#pragma unroll
  for (int w = 0; w < PB_NW; w++) best[w] = 0;
  // (a grid-stride loop over few workgroups, one atomic per workgroup and window: one per wave, ~10 k waves on the
  // same nine words, serialised at the memory side and took ~0.26 ms per chr1 haplotype)
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const Node16 a = nd[j];
    const int64_t ol = a.oplen();
    int32_t c[PB_NW];
#pragma unroll
    for (int w = 0; w < PB_NW; w++) {
      c[w] = pb_node_cost(a, PB_W[w]);
      if (a.code() == 2) {   // (special: the count replaced by '>' off ':' l 'I', off < oplen, l <= W)
        const int32_t sp = 3 + pb_ndig(ol) + pb_ndig(PB_W[w]) + pb_ndig(ol) + 1;
        if (sp > c[w]) c[w] = sp;
      }
    }
    if (j + 1 < n) {
      const int64_t base = nd[j + 1].key();
      for (int64_t k = j + 1; k < n; k++) {
        const Node16 b = nd[k];
        const int64_t key = b.key();
        if (key > base + PB_W[PB_NW - 1] - 2) break;
#pragma unroll
        for (int w = 0; w < PB_NW; w++)
          if (key <= base + PB_W[w] - 2) c[w] += pb_node_cost(b, PB_W[w]);
      }
    }
#pragma unroll
    for (int w = 0; w < PB_NW; w++) best[w] = c[w] > best[w] ? c[w] : best[w];
    const unsigned long long e = (unsigned long long)(a.pr() + (ol > 1 ? ol : 1));
    pm = e > pm ? e : pm;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
#pragma unroll
    for (int w = 0; w < PB_NW; w++) {
      const int32_t o = __shfl_xor(best[w], d, 64);
      best[w] = o > best[w] ? o : best[w];
    }
    const unsigned long long o = __shfl_xor(pm, d, 64);
    pm = o > pm ? o : pm;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int w = 0; w < PB_NW; w++) s_w[wv][w] = best[w];
    s_p[wv] = pm;
  }
  __syncthreads();
  if (threadIdx.x < PB_NW) {
    int32_t m = 0;
    for (int k = 0; k < 4; k++) m = s_w[k][threadIdx.x] > m ? s_w[k][threadIdx.x] : m;
    atomicMax(out_w + threadIdx.x, m);
  } else if (threadIdx.x == PB_NW) {
    unsigned long long m = 0;
    for (int k = 0; k < 4; k++) m = s_p[k] > m ? s_p[k] : m;
    atomicMax(out_pos, m);
  }
}

// Node-search buckets: bkt[k] = first node whose key is >= p_min + (k << NODE_BKT_SHIFT) (lower_bound), so the
// searchsorted of rpc.get_begin_end_nodes (rpc.py:127-130) only scans the few keys of one bucket.
__global__ void __launch_bounds__(256) k_node_buckets(const int64_t *keys, int64_t n, const int64_t *ends,
                                                      int64_t n_bkt, int32_t *bkt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n_bkt) return;
  const int64_t p_min = ends[0];   // (k_splice_ends)
  const int64_t x = p_min + (k << NODE_BKT_SHIFT);
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < x) lo = mid + 1; else hi = mid;
  }
  bkt[k] = (int32_t)lo;
}

}  // namespace

int32_t var_upload(mh_ctx *ctx, VarSet &v, const int64_t *v_pos, const uint8_t *v_op, const int64_t *v_oplen,
                   const int64_t *v_alt_off, const int64_t *v_alt_len, const char *alt_pool, int64_t alt_pool_len,
                   int64_t n_var) {
  for (int64_t i = 0; i < n_var; i++)
    if (v_op[i] != 'X' && v_op[i] != 'I' && v_op[i] != 'D')
      return arg_fail(ctx, MH_E_COMPLEX_VARIANT, "Complex variants present in VCF. Please filter or refactor these.");
  for (int64_t i = 0; i < n_var; i++)
    if (v_alt_off[i] < 0 || v_alt_len[i] < 0 || v_alt_off[i] + v_alt_len[i] > alt_pool_len)
      return arg_fail(ctx, MH_E_ARG, "variant alt bytes outside alt_pool");
  hipStream_t st = ctx->stream;
  const int64_t nv = n_var > 0 ? n_var : 1;
  MH_TRY(ensure(ctx, v.pos, 8 * nv));
  MH_TRY(ensure(ctx, v.op, nv));
  MH_TRY(ensure(ctx, v.oplen, 8 * nv));
  MH_TRY(ensure(ctx, v.aoff, 8 * nv));
  MH_TRY(ensure(ctx, v.alen, 8 * nv));
  MH_TRY(ensure(ctx, v.pool, alt_pool_len > 0 ? alt_pool_len : 1));
  if (n_var > 0) {
    HIPCHK(ctx, hipMemcpyAsync(v.pos.p, v_pos, 8 * n_var, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(v.op.p, v_op, n_var, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(v.oplen.p, v_oplen, 8 * n_var, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(v.aoff.p, v_alt_off, 8 * n_var, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(v.alen.p, v_alt_len, 8 * n_var, hipMemcpyHostToDevice, st));
  }
  if (alt_pool_len > 0) HIPCHK(ctx, hipMemcpyAsync(v.pool.p, alt_pool, alt_pool_len, hipMemcpyHostToDevice, st));
  // pageable sources: the copies have read them once the stream reaches here
  SYNCCHK(ctx, hipStreamSynchronize(st));
  v.n = n_var;
  v.pool_len = alt_pool_len;
  return MH_OK;
}

void release_vars(VarSet &v) {
  release(v.pos); release(v.op); release(v.oplen); release(v.aoff); release(v.alen); release(v.pool);
  v.n = v.pool_len = 0;
}

int32_t splice_build(mh_ctx *ctx, Hap &h, const Contig &c, int64_t rs, const VarSet &v, int lane) {
  // lane 1 (mh_build_haplotypes_vset's second copy, on a host thread of its own): the second stream and its own
  // scratch, no stage timing; lane 2 (mh_prefetch_haplotypes_vset's thread): the prefetch stream and its own scratch
  const bool l1 = lane != 0;
  hipStream_t st = lane == 2 ? ctx->pstream : l1 ? ctx->stream2 : ctx->stream;
  DevBuf *sl = lane == 2 ? ctx->sl3 : ctx->sl2;
  DevBuf &b_anchor = l1 ? sl[0] : ctx->s[6], &b_acc = l1 ? sl[1] : ctx->s[7];
  DevBuf &b_refb = l1 ? sl[2] : ctx->s[8], &b_nsrc = l1 ? sl[3] : ctx->s[9];
  DevBuf &b_small = l1 ? sl[4] : ctx->d_small, &b_part = l1 ? sl[5] : ctx->scan_partials;
  DevBuf &b_nrun = l1 ? sl[6] : ctx->nrun_tmp, &b_perm = l1 ? sl[7] : ctx->perm_tmp;
  auto stage_begin = [&](mh_ctx *cx, const char *name) {
    if (!l1) ::mh::stage_begin(cx, name);
  };
  auto stage_end = [&](mh_ctx *cx) {
    if (!l1) ::mh::stage_end(cx);
  };
  int64_t *hs_base = lane == 2 ? ctx->h_small3 : pinned_small(ctx);
  if (!hs_base) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  int64_t *const hs_lane = hs_base + (lane == 1 ? 256 : 0);
  const int64_t n_var = v.n;
  const int64_t nv = n_var > 0 ? n_var : 1;
  const int64_t node_cap = 2 * n_var + 1;
  h.bound_valid = false;

  stage_begin(ctx, "splice");
  const int64_t *d_pos = (const int64_t *)v.pos.p, *d_oplen = (const int64_t *)v.oplen.p;
  const int64_t *d_aoff = (const int64_t *)v.aoff.p, *d_alen = (const int64_t *)v.alen.p;
  const uint8_t *d_op = (const uint8_t *)v.op.p, *d_pool = (const uint8_t *)v.pool.p;

  // --- scratch: anchor(6) accepted(7) ref_before(8) node src(9) small(d_small) -----------------------------
  MH_TRY(ensure(ctx, b_anchor, nv));
  MH_TRY(ensure(ctx, b_acc, nv));
  MH_TRY(ensure(ctx, b_refb, 8 * nv));
  MH_TRY(ensure(ctx, b_nsrc, 8 * node_cap));
  MH_TRY(ensure(ctx, b_small, 256));
  MH_TRY(ensure(ctx, b_part, 32 * scan_partials_count(node_cap > nv ? node_cap : nv) + 64));
  uint8_t *anchor = (uint8_t *)b_anchor.p, *accepted = (uint8_t *)b_acc.p;
  int64_t *ref_before = (int64_t *)b_refb.p, *nsrc = (int64_t *)b_nsrc.p;
  char *small = (char *)b_small.p;
  int64_t *tot_i64 = (int64_t *)small;           // [0]
  NS *tot_ns = (NS *)(small + 16);                // [16..32)
  int32_t *err = (int32_t *)(small + 64);
  HIPCHK(ctx, hipMemsetAsync(small, 0, 256, st));

  MH_TRY(ensure(ctx, h.keys, 8 * node_cap));
  MH_TRY(ensure(ctx, h.ps, 8 * node_cap));
  MH_TRY(ensure(ctx, h.pr, 8 * node_cap));
  MH_TRY(ensure(ctx, h.oplen, 8 * node_cap));
  MH_TRY(ensure(ctx, h.op, node_cap));

  int64_t *keys = (int64_t *)h.keys.p, *ps = (int64_t *)h.ps.p, *pr = (int64_t *)h.pr.p, *nl = (int64_t *)h.oplen.p;
  uint8_t *nop = (uint8_t *)h.op.p;

  int64_t final_ref = rs;
  NS tot{0, 0};
  if (n_var > 0) {
    HIPCHK(ctx, device_scan<int64_t>(st, n_var, LoadEnd{d_pos, d_op, d_oplen}, StoreAnchor{d_pos, anchor, rs}, OpMax{},
                                     INT64_MIN, (int64_t *)b_part.p, tot_i64));
    HIPCHK(ctx, hipMemsetAsync(accepted, 0, n_var, st));
    hipLaunchKernelGGL(k_resolve, dim3(grid_for(n_var, 256)), dim3(256), 0, st, n_var, d_pos, d_op, d_oplen, anchor,
                       accepted, rs);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, device_scan<int64_t>(st, n_var, LoadAccEnd{d_pos, d_op, d_oplen, accepted, rs},
                                     StoreRefBefore{ref_before, rs}, OpMax{}, INT64_MIN,
                                     (int64_t *)b_part.p, tot_i64));
    HIPCHK(ctx, device_scan<NS>(st, n_var, LoadNS{d_pos, d_op, d_oplen, accepted, ref_before},
                                StoreNodes{d_pos, d_op, d_oplen, accepted, ref_before, d_aoff, d_alen, keys, ps, pr, nl,
                                           nsrc, nop, rs, c.len, err},
                                OpSum{}, NS{0, 0}, (NS *)b_part.p, tot_ns));
    // one readback into pinned memory: tot_i64 at small + 0, tot_ns at small + 16
    int64_t *hs = hs_lane;
    HIPCHK(ctx, hipMemcpyAsync(hs, small, 32, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    final_ref = hs[0];
    if (final_ref < rs) final_ref = rs;
    tot = NS{hs[2], hs[3]};
  }
  int64_t n_nodes = tot.nodes, samp_end = rs + tot.samp, hap_len = tot.samp;
  int64_t offset = final_ref - rs;
  if (offset <= c.len) {                                   // trailing '=' node, rpc.py:59-61
    int64_t len = c.len - offset;
    hipLaunchKernelGGL(k_trailing, dim3(1), dim3(1), 0, st, n_nodes, samp_end, final_ref, rs, len, keys, ps, pr, nl,
                       nsrc, nop);
    HIPCHK(ctx, hipGetLastError());
    n_nodes++;
    hap_len += len;
  }
  // p_min / p_max (readgenerate.py:192): ps of the first node; ps + oplen of the last — gathered beside the error
  // word by one thread and read back in one copy (each small copy is a blit launch of its own)
  int64_t *hs = hs_lane;
  hipLaunchKernelGGL(k_splice_ends, dim3(1), dim3(64), 0, st, (const int64_t *)ps, (const int64_t *)nl, n_nodes,
                     (int64_t *)(small + 96));
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipMemcpyAsync(hs + 8, small + 64, 64, hipMemcpyDeviceToHost, st));   // err at + 64, ends at + 96
  // (read after the N-run count's synchronisation below: the kernels in between take p_min from the device and
  // skip an erroneous splice)
  const int64_t *d_ends = (const int64_t *)(small + 96);
  int64_t p_min = 0, p_last = 0, nl_last = 0;

  // --- haplotype bytes ---------------------------------------------------------------------------------------
  if (hap_len >= ((int64_t)1 << 32) - 1) {   // (the N-run boundaries are sorted as u32 positions)
    stage_end(ctx);
    return arg_fail(ctx, MH_E_ARG, "haplotype of 2^32 - 1 bases or more");
  }
  MH_TRY(ensure(ctx, h.hap, hap_len + 1024));   // emission gathers whole 16-byte chunks past the last base
  // --- node-search buckets and the AoS node copy (the byte fill below and emission search through them) --------
  {
    // Node16 holds positions below 2^40 and lengths below 2^46: ps <= rs + hap_len, pr <= rs + contig length
    if (rs < 0 || rs + hap_len + c.len >= ((int64_t)1 << 40)) {
      stage_end(ctx);
      return arg_fail(ctx, MH_E_ARG, "region coordinates beyond 2^40");
    }
    MH_TRY(ensure(ctx, h.nd, sizeof(Node16) * (n_nodes + 1)));
    hipLaunchKernelGGL(k_node_pack, dim3(grid_for(n_nodes, 256, INT32_MAX)), dim3(256), 0, st, n_nodes,
                       (const int64_t *)h.ps.p, (const int64_t *)h.pr.p, (const int64_t *)h.oplen.p,
                       (const uint8_t *)h.op.p, (Node16 *)h.nd.p);
    HIPCHK(ctx, hipGetLastError());
    const int64_t n_bkt = ((hap_len + 2048) >> NODE_BKT_SHIFT) + 1;   // keys reach at most p_min + hap_len + 1
    MH_TRY(ensure(ctx, h.bkt, 4 * (n_bkt + 2)));
    hipLaunchKernelGGL(k_node_buckets, dim3(grid_for(n_bkt + 1, 256, INT32_MAX)), dim3(256), 0, st,
                       (const int64_t *)h.keys.p, n_nodes, d_ends, n_bkt, (int32_t *)h.bkt.p);
    HIPCHK(ctx, hipGetLastError());
    h.n_bkt = n_bkt;
    // the single-pass writer's qname-part bounds, read back with the N-run counts below (small + 160 / + 192)
    if (n_nodes > 0) {
      hipLaunchKernelGGL(k_part_bound, dim3(grid_for(n_nodes, 256, 512)), dim3(256), 0, st,
                         (const Node16 *)h.nd.p, n_nodes, (int32_t *)(small + 160),
                         (unsigned long long *)(small + 192));
      HIPCHK(ctx, hipGetLastError());
    }
  }
  if (hap_len > 0) {
    stage_begin(ctx, "splice_hap_copy");
    hipLaunchKernelGGL(k_hap_fill, dim3((unsigned)((hap_len + FILL_SPAN - 1) / FILL_SPAN)), dim3(256), 0, st, hap_len,
                       d_ends, (const int32_t *)err, n_nodes, (const Node16 *)h.nd.p, (const int64_t *)nsrc, (const int32_t *)h.bkt.p,
                       h.n_bkt, (const uint8_t *)c.seq.p, d_pool, (uint8_t *)h.hap.p);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  }
  // --- reverse complement (mate-1 reads) --------------------------------------------------------------------
  MH_TRY(ensure(ctx, h.rc, hap_len + 1024));
  if (hap_len > 0) {
    stage_begin(ctx, "splice_hap_rc");
    hipLaunchKernelGGL(k_hap_rc, dim3(grid_for((hap_len + 15) / 16, 256, INT32_MAX)), dim3(256), 0, st,
                       (const uint8_t *)h.hap.p, hap_len, (uint8_t *)h.rc.p);
    HIPCHK(ctx, hipGetLastError());
    stage_end(ctx);
  }
  // --- N runs: boundaries appended by k_nrun_find, then sorted ----------------------------------------------
  {
    unsigned long long *cnt = (unsigned long long *)(small + 128);
    int64_t cap = std::max<int64_t>(4096, (int64_t)(h.nrun_s.cap / 8) - 1);   // (nrun scratch: b_nrun)
    unsigned long long hc[2] = {0, 0};
    for (int attempt = 0; attempt < 2; attempt++) {
      MH_TRY(ensure(ctx, b_nrun, 16 * (size_t)cap + 64));
      uint32_t *us = (uint32_t *)b_nrun.p, *ue = us + cap;
      if (attempt) HIPCHK(ctx, hipMemsetAsync(cnt, 0, 16, st));   // (the first time: zeroed with `small`)
      const int64_t nel = hap_len / 64 + 1;
      hipLaunchKernelGGL(k_nrun_find, dim3(grid_for(nel, 256, INT32_MAX)), dim3(256), 0, st, (const uint8_t *)h.hap.p,
                         hap_len, cap, us, ue, cnt);
      HIPCHK(ctx, hipGetLastError());
      // the counts (small + 128) and k_part_bound's results (small + 160 .. 200) -> hs + 16 .. 25
      HIPCHK(ctx, hipMemcpyAsync(hs + 16, cnt, 72, hipMemcpyDeviceToHost, st));
      SYNCCHK(ctx, hipStreamSynchronize(st));
      if (attempt == 0) {   // the splice's error word and node ends, read back before the haplotype bytes
        const int32_t herr = (int32_t)(hs[8] & 0xffffffff);
        if (herr) {
          stage_end(ctx);
          return arg_fail(ctx, MH_E_ARG, herr & 1 ? "variant beyond the end of the fetched reference region"
                                                  : "SNP/INS alt length inconsistent with its op");
        }
        p_min = hs[12];
        p_last = hs[13];
        nl_last = hs[14];
        std::memcpy(h.part_w, hs + 20, sizeof(h.part_w));
        h.pos_max = hs[24];
        h.bound_valid = true;
      }
      hc[0] = (unsigned long long)hs[16];
      hc[1] = (unsigned long long)hs[17];
      if ((int64_t)hc[0] <= cap && (int64_t)hc[1] <= cap) break;
      cap = (int64_t)std::max(hc[0], hc[1]);   // more boundaries than room: once more with room for all
    }
    const int64_t nr = (int64_t)hc[0];
    if ((int64_t)hc[1] != nr) {
      stage_end(ctx);
      return arg_fail(ctx, MH_E_STATE, "N-run starts and ends do not pair");
    }
    h.n_runs = nr;
    MH_TRY(ensure(ctx, h.nrun_s, 8 * (nr + 1)));
    MH_TRY(ensure(ctx, h.nrun_e, 8 * (nr + 1)));
    if (nr > 0 && nr <= NR_LDS) {
      hipLaunchKernelGGL(k_nrun_sort_small, dim3(2), dim3(1024), 0, st, (const uint32_t *)b_nrun.p,
                         (const uint32_t *)b_nrun.p + cap, nr, (int64_t *)h.nrun_s.p, (int64_t *)h.nrun_e.p);
      HIPCHK(ctx, hipGetLastError());
    } else if (nr > 0) {
      // both boundary lists sorted by the library's LSD sort (mh_sort.h; the values, element indices, unused),
      // then widened to the i64 lists the measure pass searches
      unsigned bits = 1;
      while (bits < 32 && ((int64_t)1 << bits) <= hap_len) bits++;
      const uint32_t *us = (const uint32_t *)b_nrun.p, *ue = us + cap;
      size_t tmp = 0;
      HIPCHK(ctx, lsd_sort_pairs_iota(nullptr, tmp, us, nullptr, nullptr, nr, bits, st));
      const size_t kb = (8 * (size_t)nr + 255) & ~(size_t)255;
      MH_TRY(ensure(ctx, b_perm, tmp + 2 * kb + 256));
      uint32_t *sk = (uint32_t *)b_perm.p, *sv = (uint32_t *)((char *)b_perm.p + kb);
      void *stmp = (char *)b_perm.p + 2 * kb;
      for (int e = 0; e < 2; e++) {
        HIPCHK(ctx, lsd_sort_pairs_iota(stmp, tmp, e ? ue : us, sk, sv, nr, bits, st));
        hipLaunchKernelGGL(k_widen_u32, dim3(grid_for(nr, 256, 65535)), dim3(256), 0, st, (const uint32_t *)sk, nr,
                           (int64_t *)(e ? h.nrun_e.p : h.nrun_s.p));
        HIPCHK(ctx, hipGetLastError());
      }
    }
  }
  stage_end(ctx);

  h.n_nodes = n_nodes;
  h.p_min = p_min;
  h.p_max = p_last + nl_last;
  h.hap_len = hap_len;
  h.ref_start_pos = rs;
  h.valid = true;
  return MH_OK;
}

}  // namespace mh
