// mh_deflate.hip — BGZF compression of device buffers on the GPU (`.gz` FASTQ output;
// reference readgenerate.py:233-253 writes through pysam / htslib, whose BGZF is zlib deflate in 0xff00-byte
// blocks).  The host deflate pool (mh_bgzf.cpp) does ~1.5 GB/s on 16 cores; a chr1 job is 17.4 GB of FASTQ.
//
// One 512-thread workgroup per BGZF block (up to 0xff00 input bytes, staged in LDS).  Its eight waves each compress
// one eighth of the block as a deflate block of their own (dynamic Huffman codes from that slice's symbols,
// matches inside the slice): wave w < 7 ends its block with an empty stored block (a sync flush, 5 bytes) so the
// next slice's bits start on a byte boundary, and the slices' bytes simply concatenate; wave 7's block is final.
//   parse   greedy LZ77 over the slice, 256 positions per step: every position is looked up (a 2^11-entry hash of
//           the next four bytes, holding positions of earlier steps, and the run candidate at distance 1) and its
//           match extended up to 32 bytes; a walk over the positions takes every match the step's positions start
//           (literals between them; a match of 32+ bytes is extended by the whole wave, up to 258), then the
//           positions passed are hashed in;
//   pass 1  the parse, counting symbol frequencies;
//   codes   lane 0: length-limited Huffman lengths (15 bits; 7 for the code-length code), canonical codes, the
//           dynamic header (mh_deflate.h, host-testable);
//   pass 2  pass 1's tokens (kept per wave in global memory: each step's position masks and its matches), each
//           step's codes placed by wave prefix sums of their bit lengths into an LDS staging strip, whole words
//           flushed to the slice's region of the block's slot;
//   CRC-32  every thread a 132-byte segment (slicing by 4), scaled to the block's end by compile-time powers of x,
//           XOR-reduced.
// A block whose codes would not fit a BGZF block, or not be smaller than its bytes, is stored instead.
// k_bgzf_pack then writes the blocks (gzip header with the BC field, the slices' bytes, CRC32, ISIZE) at offsets
// from a scan of their sizes.
#include "mh_deflate.h"
#include "mh_device.h"
#include "mh_internal.h"
#include "mh_scan.h"

namespace mh {

namespace {

using namespace df;

constexpr int DF_WAVES = 8;
constexpr int DF_THREADS = 64 * DF_WAVES;
constexpr int SLICE = (BLOCK + DF_WAVES - 1) / DF_WAVES;   // 8160 input bytes per wave
constexpr int HBITS = 11;
constexpr int REGION = 9216;                // a slice's output bytes in the slot (more: the block is stored)
constexpr int SLOT = DF_WAVES * REGION;
constexpr int DF_NP = 4;                    // parse positions per lane and step (a step covers 256 positions;
                                            // 512 measured slower on BAM records: 0.30 vs 0.26 s, round 4)
// pass 1's tokens, kept for pass 2 (global memory, per wave): per step its end and position masks (TSW words), then
// the matches packed (length | distance << 9).  A step covers >= 256 positions but the last, a match >= 7 bytes.
constexpr int TSW = 1 + 4 * DF_NP;
constexpr int TOK_STEPS = (SLICE + 64 * DF_NP - 1) / (64 * DF_NP) + 1;
constexpr int TOK_MATCHES = SLICE / 7 + 1;
constexpr int TOK_WORDS = ((TOK_STEPS * TSW + TOK_MATCHES) + 63) / 64 * 64;
// staging words: a step's codes (at most 256 literals of <= 15 bits: a match of <= 48 bits stands for >= 7
// positions), a carried word, slack
constexpr int STAGE = (64 * DF_NP * 15 + 31) / 32 + 8;

struct CodeScratch {                        // while the codes are built (the hash table is idle then)
  uint32_t keys[512], A[NLIT];
  int32_t count[32];
  HeaderScratch H;
};
struct PackedCodes {                        // pass 2 (the hash table is idle then): code | length << 16
  uint32_t l[NLIT], d[NDIST];
};
struct WaveLds {
  union {
    uint32_t ht[1 << HBITS];                // hash: position + 1 of the latest earlier position (atomicMax)
    CodeScratch cs;
    PackedCodes pk;
  };
  uint32_t lf[NLIT], dfq[NDIST];
  uint8_t llen[NLIT], dlen[NDIST];
  uint16_t lcode[NLIT], dcode[NDIST];
  uint32_t stage[STAGE];
  uint32_t hw[96];                          // the dynamic header's bits, as words
};
static_assert(sizeof(CodeScratch) <= sizeof(uint32_t) * (1 << HBITS), "code scratch inside the hash table");
static_assert(sizeof(PackedCodes) <= sizeof(uint32_t) * (1 << HBITS), "packed codes inside the hash table");

struct BlockLds {
  uint8_t in[BLOCK + 64];                   // the block's input, zero-padded
  uint32_t crc_tab[4][256];                 // slicing-by-4 tables: byte i followed by k zero bytes
  uint32_t crcw[DF_WAVES], crc_tail, crc;   // per-wave XOR of the scaled segment CRCs; the partial segment's; result
  int32_t stored;
  WaveLds w[DF_WAVES];
};
static_assert(sizeof(BlockLds) <= 160 * 1024, "LDS");
static_assert(CRC_NSEG <= DF_THREADS, "a CRC segment per thread");

__constant__ CrcPowers kCrcPow = make_crc_powers();

// DF_PROF (calibration builds only: make prof): per-phase shader-clock sums of every wave's lane 0, read back by
// mh_df_prof (scripts/calib_deflate.py).  Slots: 0 staging, 1 CRC, 2 parse, 3 count, 4 keep, 5 hash-in, 6 pass-2
// set-up (and the pass-1 tail), 7 token load, 8 encode, 9 end of block; 10 parse steps, 11 matches, 12 waves with a
// slice; 13 literal/length codes, 14 distance codes, 15 header.
#ifdef DF_PROF
__device__ unsigned long long df_prof[16];
struct DfProf {
  uint64_t t, a[16];
  __device__ void mark(int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    a[i] += now - t;
    t = now;
  }
};
#define DFP_BEGIN                          \
  DfProf P_;                               \
  for (int i_ = 0; i_ < 16; i_++) P_.a[i_] = 0; \
  P_.t = __builtin_amdgcn_s_memtime()
#define DFP(i) P_.mark(i)
#define DFP_ADD(i, v) P_.a[i] += (uint64_t)(v)
#define DFP_END \
  if (lane == 0) \
    for (int i_ = 0; i_ < 16; i_++) atomicAdd(&df_prof[i_], (unsigned long long)P_.a[i_])
#else
#define DFP_BEGIN
#define DFP(i)
#define DFP_ADD(i, v)
#define DFP_END
#endif

struct DfBlockInfo {
  int32_t n;           // input bytes
  int32_t stored;      // 1: stored block (the slices' regions unused)
  uint32_t crc;
  int32_t len[DF_WAVES];   // bytes of each slice's deflate data
};

__device__ __forceinline__ uint32_t load4(const uint8_t *b, int x) {   // bytes x .. x+3 of an LDS array
  const uint32_t *q = (const uint32_t *)(b + (x & ~3));
  return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(x & 3));
}
__device__ __forceinline__ uint32_t hash4(uint32_t w) { return (w * 2654435761u) >> (32 - HBITS); }
static_assert(MIN_MATCH == 7, "words7: a match is checked as two overlapping 4-byte words");

// Wave-wide ascending sort of n <= 320 keys in LDS (bitonic over the next power of two, padded with ~0u).
__device__ void wave_sort(uint32_t *k, int n, int lane) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = n + lane; i < P; i += 64) k[i] = 0xffffffffu;
  __builtin_amdgcn_s_waitcnt(0xc07f);   // (lgkmcnt(0)) the padding is in place
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < P / 2; i += 64) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t a = k[lo], b = k[hi];
        if ((a > b) == up) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
}

// Canonical codes of one alphabet from its lengths, wave-wide: the count of each length by ballots, then each
// symbol's rank among the earlier symbols of its length (per-length counts in registers: loops over the 15 lengths
// unrolled)
__device__ void wave_canonical(const uint8_t *len, int n, uint16_t *code, int lane) {
  uint32_t cnt[16], next[16], run[16];
#pragma unroll
  for (int b = 0; b < 16; b++) cnt[b] = run[b] = 0;
  for (int s0 = 0; s0 < n; s0 += 64) {
    const int l = s0 + lane < n ? len[s0 + lane] : 0;
#pragma unroll
    for (int b = 1; b < 16; b++) cnt[b] += (uint32_t)__popcll(__ballot(l == b));
  }
  uint32_t c = 0;
  next[0] = 0;
#pragma unroll
  for (int b = 1; b < 16; b++) {
    c = (c + cnt[b - 1]) << 1;
    next[b] = c;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int s0 = 0; s0 < n; s0 += 64) {
    const int l = s0 + lane < n ? len[s0 + lane] : 0;
    uint32_t cd = 0;
#pragma unroll
    for (int b = 1; b < 16; b++) {
      const uint64_t bal = __ballot(l == b);
      if (l == b) cd = next[b] + run[b] + (uint32_t)__popcll(bal & below);
      run[b] += (uint32_t)__popcll(bal);
    }
    if (s0 + lane < n) code[s0 + lane] = l ? (uint16_t)(__builtin_bitreverse32(cd) >> (32 - l)) : (uint16_t)0;
  }
}

// Code lengths of one alphabet from the wave's frequencies (keys sorted by the whole wave, the lengths on lane 0,
// the codes wave-wide).
__device__ void wave_huffman(const uint32_t *f, int n, int limit, uint8_t *len, uint16_t *code, uint32_t *keys,
                             uint32_t *A, int32_t *count, int lane) {
  // keys of the used symbols, compacted in symbol order by a wave prefix count
  int base = 0;
  for (int s0 = 0; s0 < n; s0 += 64) {
    const int s = s0 + lane;
    const bool used = s < n && f[s] != 0;
    const uint64_t bal = __ballot(used);
    if (used) keys[base + __popcll(bal & ((1ull << lane) - 1))] = (f[s] << 9) | (uint32_t)s;
    if (s < n) len[s] = 0;
    base += __popcll(bal);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  wave_sort(keys, base, lane);
  if (lane == 0) huffman_from_sorted(keys, base, limit, len, A, count);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  wave_canonical(len, n, code, lane);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// One step of the parse at `cur` (wave-uniform) covers DF_NP x 64 positions (lane l holds positions cur + 64 h + l,
// h < DF_NP): every position looks for a match (cand: an earlier position), then a greedy walk over the positions
// (wave-uniform, one iteration per match) picks the tokens: literals up to the next position with a match, that
// match — extended by the whole wave, 64 bytes per round, up to MAX_MATCH — and on after its end.  So a step takes
// every match its positions start (records with many short matches, e.g. BAM, took one step per match), and a
// step of literals covers 256 bytes (random FASTQ bases are literals).  The later positions' candidates were looked
// up before this step's earlier positions were hashed in: the tokens differ from a position-by-position greedy
// parse, never in validity (every match is verified); the host restatement (tests/deflate_host.cpp) deflates the
// golden FASTQ to the same ratio in 3.6x fewer steps than one match per step.  (Each position extending its own
// candidate before the walk cost three times the time on runs of matches: round 4, `scripts/bgzf_rate.py`.)
struct Step {
  int next;                          // the position after the step's last token
  uint64_t lit[DF_NP], ms[DF_NP];    // positions 64 h + lane holding a literal / starting a match
  int mlen[DF_NP], mdist[DF_NP];     // this lane's matches (ms positions)
};
// what pass 1 keeps of a step's positions for its hash inserts and counts (no second look at the bytes)
struct StepPos {
  uint32_t hv[DF_NP];                // hash of the position's first four bytes (valid positions)
  uint32_t lb[DF_NP];                // the position's byte
};

// bytes x .. x+3 and x+3 .. x+6 from three aligned words (the slice starts 4-byte aligned)
__device__ __forceinline__ void words7(const uint32_t *wd, int x, uint32_t &w, uint32_t &w3) {
  const int i = x >> 2, o = x & 3;
  const uint32_t q0 = wd[i], q1 = wd[i + 1], q2 = wd[i + 2];
  w = __builtin_amdgcn_alignbyte(q1, q0, (uint32_t)o);
  w3 = o ? __builtin_amdgcn_alignbyte(q2, q1, (uint32_t)(o - 1)) : __builtin_amdgcn_alignbyte(q1, q0, 3u);
}

__device__ __forceinline__ Step parse_step(const uint8_t *s, int S, int cur, const uint32_t *ht, int lane,
                                           StepPos &sp) {
  const uint32_t *wd = (const uint32_t *)s;
  int cand[DF_NP], len[DF_NP];
  uint64_t M[DF_NP];
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    const int p = cur + 64 * h + lane;
    int c = -1;
    uint32_t hv = 0, lb = 0;
    if (p + MIN_MATCH <= S) {
      uint32_t w, w3;
      words7(wd, p, w, w3);   // bytes p .. p+6 (two overlapping words)
      lb = w & 0xffu;
      hv = hash4(w);
      // a run (distance 1): bytes p-1 .. p+6 all equal
      if (p >= 1 && w == lb * 0x01010101u && w3 == w && s[p - 1] == lb) {
        c = p - 1;
      } else {
        const int j = (int)ht[hv] - 1;                // a position of an earlier step (< cur <= p)
        if (j >= 0) {
          uint32_t cw, cw3;
          words7(wd, j, cw, cw3);
          if (cw == w && cw3 == w3) c = j;
        }
      }
    } else if (p < S) {
      lb = s[p];
    }
    sp.hv[h] = hv;
    sp.lb[h] = lb;
    cand[h] = c;
    len[h] = 0;
    M[h] = __ballot(c >= 0);
  }
  const int NW = 64 * DF_NP;
  const int W = S - cur < NW ? S - cur : NW;
  Step st;
#pragma unroll
  for (int h = 0; h < DF_NP; h++) st.lit[h] = st.ms[h] = 0;
  // (the walk's state is wave-uniform: readfirstlane keeps it in scalar registers)
  int x = 0;
  for (;;) {   // wave-uniform greedy walk: x = the position of the next token
    int m = NW;
#pragma unroll
    for (int h = 0; h < DF_NP; h++)
      if (m == NW && x < 64 * (h + 1)) {
        const uint64_t r = x > 64 * h ? M[h] & (~0ull << (x - 64 * h)) : M[h];
        if (r) m = 64 * h + __builtin_ctzll(r);
      }
    m = __builtin_amdgcn_readfirstlane(m);
    const int me = m < W ? m : W;
#pragma unroll
    for (int h = 0; h < DF_NP; h++) {   // literals [x, me)
      const int a = x > 64 * h ? x - 64 * h : 0, b = me < 64 * (h + 1) ? me - 64 * h : 64;
      if (b > a) st.lit[h] |= (b - a >= 64 ? ~0ull : ((1ull << (b - a)) - 1ull)) << a;
    }
    if (m >= W) {
      st.next = cur + W;
      break;
    }
    const int hm = m >> 6, l = m & 63;
    int jc = 0;
#pragma unroll
    for (int h = 0; h < DF_NP; h++)
      if (h == hm) {
        st.ms[h] |= 1ull << l;
        jc = __builtin_amdgcn_readlane(cand[h], l);
      }
    // the match extended by the whole wave, 64 bytes per round (up to MAX_MATCH)
    const int q = cur + m;
    const int cap = S - q < MAX_MATCH ? S - q : MAX_MATCH;
    int L = MIN_MATCH;
    for (;;) {
      const int k = L + lane;
      const bool eq = k < cap && s[q + k] == s[jc + k];
      const uint64_t ne = ~__ballot(eq);
      const int run = ne ? __builtin_ctzll(ne) : 64;
      L += run;
      if (run < 64 || L >= cap) break;
    }
    if (L > cap) L = cap;
    L = __builtin_amdgcn_readfirstlane(L);
#pragma unroll
    for (int h = 0; h < DF_NP; h++)
      if (h == hm && lane == l) len[h] = L;
    x = __builtin_amdgcn_readfirstlane(m + L);
    if (x >= W) {
      st.next = cur + x;
      break;
    }
  }
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    st.mlen[h] = len[h];
    st.mdist[h] = cur + 64 * h + lane - cand[h];
  }
  return st;
}

// the step's positions cur .. next-1 into the hash table (the hashes parse_step computed; positions past the step's
// window, inside its last match, hashed here); lanes colliding on one entry keep the latest position (atomicMax), so
// the table does not depend on the order of the inserts
__device__ __forceinline__ void hash_in(const uint8_t *s, int S, int cur, int next, const StepPos &sp, uint32_t *ht,
                                        int lane) {
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    const int p = cur + 64 * h + lane;
    if (p < next && p + HASH_BYTES <= S)
      atomicMax(&ht[p + MIN_MATCH <= S ? sp.hv[h] : hash4(load4(s, p))], (uint32_t)(p + 1));
  }
  for (int k = cur + 64 * DF_NP + lane; k < next; k += 64)
    if (k + HASH_BYTES <= S) atomicMax(&ht[hash4(load4(s, k))], (uint32_t)(k + 1));
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// the symbols of one step, pass 1: literal and match frequencies (LDS atomics, one per token position)
__device__ __forceinline__ void count_step(const Step &st, const StepPos &sp, WaveLds &W, int lane) {
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    if ((st.lit[h] >> lane) & 1ull) atomicAdd(&W.lf[sp.lb[h]], 1u);
    if ((st.ms[h] >> lane) & 1ull) {
      atomicAdd(&W.lf[257 + len_code(st.mlen[h])], 1u);
      atomicAdd(&W.dfq[dist_code(st.mdist[h])], 1u);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// The wave's bit writer over its region (words): the staging strip holds the words from `wbase` on; stage[0] is
// partial (the bits below bitpos % 32).
struct BitWave {
  uint32_t *region;    // the slice's output region (global)
  int64_t bitpos;      // bits written
  bool overflow;
};

// OR one code (v, n) into the staging strip at bit offset r
__device__ __forceinline__ void stage_or(uint32_t *stage, uint64_t v, int n, int r) {
  if (!n) return;
  const int wi = r >> 5, sh = r & 31;
  atomicOr(&stage[wi], (uint32_t)(v << sh));
  const uint64_t hi = sh ? v >> (32 - sh) : v >> 32;
  if (hi) atomicOr(&stage[wi + 1], (uint32_t)hi);
  const uint64_t hi2 = sh ? (v >> (64 - sh)) : 0;
  if (sh && (sh + n) > 64 && hi2) atomicOr(&stage[wi + 2], (uint32_t)hi2);
}

// the strip's completed words to the region after `total` more bits, the partial one carried
__device__ __forceinline__ void flush_bits(BitWave &bw, uint32_t *stage, int total, int lane) {
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int64_t end = bw.bitpos + total;
  const int full = (int)((end >> 5) - (bw.bitpos >> 5));   // words completed by this step
  const int64_t w0 = bw.bitpos >> 5;
  if ((end >> 3) + 8 > REGION) bw.overflow = true;
  if (!bw.overflow)
    for (int k = lane; k < full; k += 64) bw.region[w0 + k] = stage[k];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const uint32_t carry = stage[full];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  for (int k = lane; k <= full + 2 && k < STAGE; k += 64) stage[k] = k == 0 ? carry : 0u;   // (the words used)
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  bw.bitpos = end;
}

// put each lane's (v, n) (n <= 57 bits: v < 2^n) in lane order after bitpos
__device__ __forceinline__ void put_bits(BitWave &bw, uint32_t *stage, uint64_t v, int n, int lane) {
  int total;
  const int excl = wave_sum_incl(n, total) - n;   // the bits before this lane's
  stage_or(stage, v, n, (int)(bw.bitpos & 31) + excl);
  flush_bits(bw, stage, total, lane);
}

// the codes of one step, pass 2: every token position's code (a literal's, or a match's length and distance codes
// with their extra bits: <= 48 bits), placed in position order (h, then lane)
__device__ __forceinline__ void encode_step(const uint8_t *s, int cur, const Step &st, WaveLds &W, BitWave &bw,
                                            int lane) {
  int before = (int)(bw.bitpos & 31);
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    uint64_t v = 0;
    int n = 0;
    if ((st.lit[h] >> lane) & 1ull) {
      const uint32_t c = W.pk.l[s[cur + 64 * h + lane]];
      v = c & 0xffffu;
      n = (int)(c >> 16);
    } else if ((st.ms[h] >> lane) & 1ull) {
      const int ml = st.mlen[h], md = st.mdist[h];
      const int lc = len_code(ml), dc = dist_code(md);
      const int le = len_extra(lc), de = dist_extra(dc);
      const uint32_t lk = W.pk.l[257 + lc], dk = W.pk.d[dc];
      v = lk & 0xffffu;
      n = (int)(lk >> 16);
      v |= (uint64_t)(ml - len_base(lc)) << n;
      n += le;
      v |= (uint64_t)(dk & 0xffffu) << n;
      n += (int)(dk >> 16);
      v |= (uint64_t)(md - dist_base(dc)) << n;
      n += de;
    }
    int tot;
    const int excl = wave_sum_incl(n, tot) - n;
    stage_or(W.stage, v, n, before + excl);
    before += tot;
  }
  flush_bits(bw, W.stage, before - (int)(bw.bitpos & 31), lane);
}

// pass 1: a step's tokens into the wave's token area (step record, then its matches in position order)
__device__ __forceinline__ void keep_step(uint32_t *tok, int step, int *nm, const Step &st, int lane) {
  uint32_t v = (uint32_t)st.next;
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    if (lane == 1 + 2 * h) v = (uint32_t)st.lit[h];
    if (lane == 2 + 2 * h) v = (uint32_t)(st.lit[h] >> 32);
    if (lane == 1 + 2 * DF_NP + 2 * h) v = (uint32_t)st.ms[h];
    if (lane == 2 + 2 * DF_NP + 2 * h) v = (uint32_t)(st.ms[h] >> 32);
  }
  if (lane < TSW) tok[step * TSW + lane] = v;
  uint32_t *mt = tok + TOK_STEPS * TSW;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int base = *nm;
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    if ((st.ms[h] >> lane) & 1ull)
      mt[base + __popcll(st.ms[h] & below)] = (uint32_t)st.mlen[h] | ((uint32_t)st.mdist[h] << 9);
    base += __popcll(st.ms[h]);
  }
  *nm = base;
}

// pass 2: a step's record word (lane l: word l of the step record), loaded a step ahead
__device__ __forceinline__ uint32_t load_rec(const uint32_t *tok, int step, int lane) {
  return tok[step * TSW + (lane < TSW ? lane : 0)];
}
// pass 2: the step from its record, its matches loaded from the token area (vector loads: the words pass 1 stored)
__device__ __forceinline__ Step load_step(const uint32_t *tok, uint32_t rv, int *nm, int lane) {
  Step st;
  st.next = __builtin_amdgcn_readlane((int)rv, 0);
  const uint32_t *mt = tok + TOK_STEPS * TSW;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int base = *nm;
#pragma unroll
  for (int h = 0; h < DF_NP; h++) {
    st.lit[h] = (uint32_t)__builtin_amdgcn_readlane((int)rv, 1 + 2 * h) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rv, 2 + 2 * h) << 32);
    st.ms[h] = (uint32_t)__builtin_amdgcn_readlane((int)rv, 1 + 2 * DF_NP + 2 * h) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rv, 2 + 2 * DF_NP + 2 * h) << 32);
    uint32_t m = 0;
    if ((st.ms[h] >> lane) & 1ull) m = mt[base + __popcll(st.ms[h] & below)];
    st.mlen[h] = (int)(m & 511u);
    st.mdist[h] = (int)(m >> 9);
    base += __popcll(st.ms[h]);
  }
  *nm = base;
  return st;
}

__global__ void __launch_bounds__(DF_THREADS) k_bgzf_blocks(const uint8_t *in, int64_t n_in, int64_t b0, int64_t nb,
                                                            uint8_t *slots, DfBlockInfo *info, uint32_t *tokens) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  BlockLds &L = *(BlockLds *)smem_raw;
  // (wave: readfirstlane tells the compiler it is uniform, so the slice bounds and the whole parse walk are scalar;
  // derived from threadIdx.x it is taken as divergent and the walk runs as exec-masked vector code)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b = b0 + blockIdx.x;
  if (blockIdx.x >= nb) return;
  DFP_BEGIN;
  const int64_t start = b * BLOCK;
  const int n = (int)(n_in - start < BLOCK ? n_in - start : BLOCK);
  // stage the block (16-byte loads when the block starts 16-byte aligned, bytes otherwise) and the CRC table
  const uint8_t *src = in + start;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    for (int i = tid; i < (BLOCK + 64) / 16; i += DF_THREADS) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (16 * i + 16 <= n) {
        v = reinterpret_cast<const uint4 *>(src)[i];
      } else if (16 * i < n) {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int k = 0; 16 * i + k < n; k++) w[k >> 2] |= (uint32_t)src[16 * i + k] << (8 * (k & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      reinterpret_cast<uint4 *>(L.in)[i] = v;
    }
  } else {
    for (int i = tid; i < BLOCK + 64; i += DF_THREADS) L.in[i] = i < n ? src[i] : 0;
  }
  for (int i = tid; i < 4 * 256; i += DF_THREADS) {   // table k: byte i & 255, then k zero bytes
    uint32_t c = (uint32_t)(i & 255);
    for (int k = 0; k < 8 * (1 + (i >> 8)); k++) c = c & 1 ? (c >> 1) ^ CRC_POLY : c >> 1;
    L.crc_tab[i >> 8][i & 255] = c;
  }
  if (tid == 0) {
    L.stored = 0;
    L.crc_tail = 0;
  }
  __syncthreads();
  DFP(0);
  // CRC-32 by segments (mh_deflate.h crc32_segments): thread t's raw CRC of bytes [132 t, 132 t + 132), four bytes
  // per step (slicing by 4), scaled by the compile-time power for its distance to the block's end; an XOR reduction
  {
    const int q = n / CRC_SEG, r = n - q * CRC_SEG;
    const int a = tid * CRC_SEG;
    uint32_t c = 0;
    if (a < n) {
      const int e = a + CRC_SEG < n ? a + CRC_SEG : n;
      const uint32_t *w = (const uint32_t *)(L.in + a);   // (a: a multiple of 4)
      const int nw = (e - a) >> 2;
      for (int k = 0; k < nw; k++) {
        c ^= w[k];
        c = L.crc_tab[3][c & 255u] ^ L.crc_tab[2][(c >> 8) & 255u] ^ L.crc_tab[1][(c >> 16) & 255u] ^
            L.crc_tab[0][c >> 24];
      }
      for (int k = a + 4 * nw; k < e; k++) c = crc_raw_byte(c, L.in[k], L.crc_tab[0]);
      if (tid < q) {
        c = crc_multmodp(kCrcPow.seg[q - 1 - tid], c);
      } else {
        L.crc_tail = c;   // the partial segment (thread q, when r > 0): not scaled
        c = 0;
      }
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o, 64);
    if (lane == 0) L.crcw[wave] = c;
    __syncthreads();
    if (tid == 0) {
      uint32_t x = 0;
      for (int k = 0; k < DF_WAVES; k++) x ^= L.crcw[k];
      const uint32_t raw = crc_multmodp(kCrcPow.byte[r], x) ^ L.crc_tail;
      L.crc = ~(crc_multmodp(crc_multmodp(kCrcPow.seg[q], kCrcPow.byte[r]), 0xffffffffu) ^ raw);
    }
  }
  DFP(1);
  // the wave's slice
  WaveLds &W = L.w[wave];
  const int s0 = wave * SLICE;
  const int S = s0 >= n ? 0 : (n - s0 < SLICE ? n - s0 : SLICE);
  const uint8_t *s = L.in + s0;
  const bool last = s0 + SLICE >= n;   // the final deflate block (later waves have empty slices)
  uint32_t *region = (uint32_t *)(slots + (size_t)blockIdx.x * SLOT + (size_t)wave * REGION);
  uint32_t *tok = tokens + ((size_t)blockIdx.x * DF_WAVES + wave) * TOK_WORDS;
  int32_t out_len = 0;
  if (S > 0) {
    // pass 1: frequencies
    for (int i = lane; i < (1 << HBITS); i += 64) W.ht[i] = 0;
    for (int i = lane; i < NLIT; i += 64) W.lf[i] = 0;
    for (int i = lane; i < NDIST; i += 64) W.dfq[i] = 0;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    int n_step = 0, n_match = 0;
    for (int cur = 0; cur < S;) {
      StepPos sp;
      const Step st = parse_step(s, S, cur, W.ht, lane, sp);
      DFP(2);
      count_step(st, sp, W, lane);
      DFP(3);
      keep_step(tok, n_step++, &n_match, st, lane);
      DFP(4);
      hash_in(s, S, cur, st.next, sp, W.ht, lane);
      DFP(5);
      cur = __builtin_amdgcn_readfirstlane(st.next);
    }
    DFP_ADD(10, n_step);
    DFP_ADD(11, n_match);
    DFP_ADD(12, 1);
    if (lane == 0) W.lf[256] = 1;   // end of block (a slice without matches: HDIST 1, one unused distance code)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // codes
    DFP(6);
    wave_huffman(W.lf, NLIT, 15, W.llen, W.lcode, W.cs.keys, W.cs.A, W.cs.count, lane);
    DFP(13);
    wave_huffman(W.dfq, NDIST, 15, W.dlen, W.dcode, W.cs.keys, W.cs.A, W.cs.count, lane);
    DFP(14);
    // the header bits into hw (lane 0)
    int hbits = 0;
    if (lane == 0) {
      BitSink bs{(uint8_t *)W.hw, 0, 0, 0};
      bs.put(last ? 1u : 0u, 1);
      bs.put(2u, 2);
      write_dynamic_header(bs, W.llen, W.dlen, W.cs.H);
      hbits = (int)(bs.pos * 8 + bs.nacc);
      if (bs.nacc) ((uint8_t *)W.hw)[bs.pos] = (uint8_t)bs.acc;   // the last partial byte
      for (int k = (int)bs.pos + (bs.nacc ? 1 : 0); k < (int)bs.pos + 8; k++) ((uint8_t *)W.hw)[k] = 0;
    }
    hbits = __shfl(hbits, 0, 64);
    DFP(15);
    for (int k = lane; k < STAGE; k += 64) W.stage[k] = 0;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    BitWave bw{region, 0, false};
    {   // the header's whole words straight to the region, its partial word into the strip
      const int full = hbits >> 5;
      for (int k = lane; k < full; k += 64) region[k] = W.hw[k];
      if (lane == 0) W.stage[0] = (hbits & 31) ? W.hw[full] & ((1u << (hbits & 31)) - 1u) : 0u;
      bw.bitpos = hbits;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    // pass 2: pass 1's tokens, encoded (no second parse); the packed codes over the idle hash table
    for (int i = lane; i < NLIT; i += 64) W.pk.l[i] = (uint32_t)W.lcode[i] | ((uint32_t)W.llen[i] << 16);
    if (lane < NDIST) W.pk.d[lane] = (uint32_t)W.dcode[lane] | ((uint32_t)W.dlen[lane] << 16);
    __builtin_amdgcn_s_waitcnt(0);   // (pass 1's token stores are done; the tables are in place)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    DFP(6);
    n_match = 0;
    // step k + 1's record and matches are loaded while step k is encoded
    Step nx = load_step(tok, load_rec(tok, 0, lane), &n_match, lane);
    uint32_t rvn = n_step > 1 ? load_rec(tok, 1, lane) : 0u;
    for (int cur = 0, k = 0; cur < S; k++) {
      const Step st = nx;
      if (k + 1 < n_step) {
        nx = load_step(tok, rvn, &n_match, lane);
        if (k + 2 < n_step) rvn = load_rec(tok, k + 2, lane);
      }
      DFP(7);
      encode_step(s, cur, st, W, bw, lane);
      DFP(8);
      cur = st.next;
    }
    // end of block; then either the final padding or a sync flush (empty stored block) to a byte boundary
    put_bits(bw, W.stage, lane == 0 ? (uint64_t)W.lcode[256] : 0ull, lane == 0 ? W.llen[256] : 0, lane);
    if (!last) {
      put_bits(bw, W.stage, 0ull, lane == 0 ? 3 : 0, lane);               // BFINAL 0, BTYPE 00
      const int pad = (int)((8 - (bw.bitpos & 7)) & 7);
      put_bits(bw, W.stage, 0ull, lane == 0 ? pad : 0, lane);
      put_bits(bw, W.stage, lane == 0 ? 0xffff0000ull : 0ull, lane == 0 ? 32 : 0, lane);   // LEN 0, NLEN ~0
    }
    const int pad = (int)((8 - (bw.bitpos & 7)) & 7);
    put_bits(bw, W.stage, 0ull, lane == 0 ? pad : 0, lane);
    // the partial last word
    if (lane == 0 && !bw.overflow && (bw.bitpos & 31)) bw.region[bw.bitpos >> 5] = W.stage[0];
    out_len = (int32_t)(bw.bitpos >> 3);
    if (bw.overflow) out_len = -1;
  }
  if (lane == 0 && out_len < 0) atomicOr(&L.stored, 1);
  __syncthreads();
  if (lane == 0) info[blockIdx.x].len[wave] = out_len < 0 ? 0 : out_len;
  __syncthreads();
  if (tid == 0) {
    DfBlockInfo &I = info[blockIdx.x];
    I.n = n;
    I.crc = L.crc;
    int64_t tot = 0;
    for (int w = 0; w < DF_WAVES; w++) tot += I.len[w];
    // stored also when the codes would not be smaller (random bytes): the output never exceeds bgzf_device_bound
    I.stored = (L.stored || HDR + tot + TRL > MAX_BSIZE || tot >= 5 + (int64_t)n) ? 1 : 0;
  }
  DFP(9);
  DFP_END;
}

__device__ __forceinline__ int64_t block_bytes(const DfBlockInfo &I) {
  if (I.stored) return HDR + 5 + I.n + TRL;
  int64_t t = HDR + TRL;
  for (int w = 0; w < DF_WAVES; w++) t += I.len[w];
  return t;
}
struct LoadBlk {
  const DfBlockInfo *info;
  int64_t nb;
  __device__ int64_t operator()(int64_t i) const { return i < nb ? block_bytes(info[i]) : 0; }
};
struct StoreBlk {
  int64_t *off;
  __device__ void operator()(int64_t i, int64_t, int64_t excl) const { off[i] = excl; }
};

// one workgroup per block: gzip header, the slices (or the stored input), CRC32 and ISIZE at its offset
__global__ void __launch_bounds__(256) k_bgzf_pack(const uint8_t *in, int64_t b0, const uint8_t *slots,
                                                   const DfBlockInfo *info, const int64_t *off, uint8_t *out) {
  const DfBlockInfo &I = info[blockIdx.x];
  uint8_t *d = out + off[blockIdx.x];
  const int tid = threadIdx.x;
  const int64_t bs = block_bytes(I);
  if (tid < HDR) {
    static constexpr uint8_t H0[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
    d[tid] = tid < 16 ? H0[tid] : (uint8_t)((bs - 1) >> (8 * (tid - 16)));
  }
  int64_t o = HDR;
  if (I.stored) {
    if (tid == 0) {
      d[o] = 1;   // BFINAL 1, BTYPE 00
      d[o + 1] = (uint8_t)I.n;
      d[o + 2] = (uint8_t)(I.n >> 8);
      d[o + 3] = (uint8_t)~I.n;
      d[o + 4] = (uint8_t)(~I.n >> 8);
    }
    const uint8_t *src = in + (b0 + blockIdx.x) * (int64_t)BLOCK;
    for (int i = tid; i < I.n; i += 256) d[o + 5 + i] = src[i];
    o += 5 + I.n;
  } else {
    for (int w = 0; w < DF_WAVES; w++) {
      const uint8_t *src = slots + (size_t)blockIdx.x * SLOT + (size_t)w * REGION;
      for (int i = tid; i < I.len[w]; i += 256) d[o + i] = src[i];
      o += I.len[w];
    }
  }
  if (tid < 8) d[o + tid] = (uint8_t)((tid < 4 ? I.crc : (uint32_t)I.n) >> (8 * (tid & 3)));
}

}  // namespace

int32_t bgzf_device(mh_ctx *ctx, hipStream_t st, const uint8_t *d_in, int64_t n, uint8_t *d_out, int64_t cap,
                    int64_t *used, std::vector<int64_t> *boff, const std::function<void(int64_t, int64_t)> *on_piece) {
  *used = 0;
  const int64_t nb_all = (n + BLOCK - 1) / BLOCK;
  if (boff) boff->assign((size_t)nb_all + 1, 0);
  // blocks per launch (slots: CH x 72 KiB); no more than the input has, so a small window (a bounded BAM store's)
  // does not allocate the scratch of 8192 blocks
  const int64_t CH = std::max<int64_t>(1, std::min<int64_t>(8192, nb_all));
  MH_TRY(ensure(ctx, ctx->gz_slots, (size_t)CH * SLOT + 64));
  MH_TRY(ensure(ctx, ctx->gz_tok, sizeof(uint32_t) * (size_t)CH * DF_WAVES * TOK_WORDS + 64));
  MH_TRY(ensure(ctx, ctx->gz_info, sizeof(DfBlockInfo) * (size_t)CH + 64));
  MH_TRY(ensure(ctx, ctx->gz_off, sizeof(int64_t) * (size_t)(CH + 1) + 64));
  MH_TRY(ensure(ctx, ctx->gz_scan, scan_lb_scratch_bytes<int64_t>(CH + 1)));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int64_t *tot = (int64_t *)((char *)ctx->d_small.p + 3072);
  int64_t *hs = pinned_small(ctx);
  if (!hs) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  const size_t lds = sizeof(BlockLds);
  int64_t w = 0;
  for (int64_t b0 = 0; b0 < nb_all; b0 += CH) {
    const int64_t nb = nb_all - b0 < CH ? nb_all - b0 : CH;
    hipLaunchKernelGGL(k_bgzf_blocks, dim3((unsigned)nb), dim3(DF_THREADS), lds, st, d_in, n, b0, nb,
                       (uint8_t *)ctx->gz_slots.p, (DfBlockInfo *)ctx->gz_info.p, (uint32_t *)ctx->gz_tok.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, device_scan_sum<int64_t>(st, nb, LoadBlk{(const DfBlockInfo *)ctx->gz_info.p, nb},
                                         StoreBlk{(int64_t *)ctx->gz_off.p}, ctx->gz_scan.p, tot));
    HIPCHK(ctx, hipMemcpyAsync(hs + 32, tot, 8, hipMemcpyDeviceToHost, st));
    if (boff) HIPCHK(ctx, hipMemcpyAsync(boff->data() + b0, ctx->gz_off.p, 8 * (size_t)nb, hipMemcpyDeviceToHost, st));
    SYNCCHK(ctx, hipStreamSynchronize(st));
    const int64_t bytes = hs[32];
    if (boff)
      for (int64_t i = 0; i < nb; i++) (*boff)[b0 + i] += w;
    if (w + bytes > cap) return arg_fail(ctx, MH_E_CAPACITY, "BGZF output buffer too small");
    hipLaunchKernelGGL(k_bgzf_pack, dim3((unsigned)nb), dim3(256), 0, st, d_in, b0,
                       (const uint8_t *)ctx->gz_slots.p, (const DfBlockInfo *)ctx->gz_info.p,
                       (const int64_t *)ctx->gz_off.p, d_out + w);
    HIPCHK(ctx, hipGetLastError());
    if (on_piece) (*on_piece)(w, bytes);
    w += bytes;
  }
  SYNCCHK(ctx, hipStreamSynchronize(st));
  *used = w;
  if (boff) (*boff)[nb_all] = w;
  return MH_OK;
}

#ifdef DF_PROF
extern "C" int mh_df_prof(unsigned long long *out) {   // the sums since the last call (then zeroed)
  unsigned long long z[16] = {0};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(df_prof), sizeof(z)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(df_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

// worst-case output bytes for n input bytes (every block stored)
int64_t bgzf_device_bound(int64_t n) { return n + ((n + BLOCK - 1) / BLOCK + 1) * (HDR + 5 + TRL) + 64; }

}  // namespace mh

