// mh_internal.h — shared definitions for libmitty_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <unordered_map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mitty_hip.h"

namespace mh {

// ---------------------------------------------------------------------------------------------------------------
// Error handling: every HIP call is checked; failures set ctx->err and return MH_E_HIP up the stack.
// ---------------------------------------------------------------------------------------------------------------
struct Status {
  int32_t code = MH_OK;
  std::string msg;
};

#define MH_TRY(expr)                        \
  do {                                      \
    int32_t _rc = (expr);                   \
    if (_rc != MH_OK) return _rc;           \
  } while (0)

// A grow-only device buffer.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

// Haplotype (one chromosome copy of one BED region) resident on the device.  SURVEY.md §8(a) A9.
// Sample coordinates are the reference's 1-based `ps`; hap[k] is the base at sample position p_min + k.
// One node in 16 bytes (emission's random node lookups are one 16-byte load instead of five SoA arrays):
//   a = ps | op code << 40 | (oplen mod 2^22) << 42,   b = pr | (oplen >> 22) << 40
// op codes 0 '=', 1 'X', 2 'I', 3 'D'; positions < 2^40, oplen < 2^46 (k_node_pack flags anything larger).
struct Node16 {
  uint64_t a, b;
  __host__ __device__ int64_t ps() const { return (int64_t)(a & 0xffffffffffull); }
  __host__ __device__ int64_t pr() const { return (int64_t)(b & 0xffffffffffull); }
  __host__ __device__ int code() const { return (int)((a >> 40) & 3u); }
  __host__ __device__ uint8_t op() const { return (uint8_t)(0x4449583Du >> (8 * code())); }   // '=' 'X' 'I' 'D'
  __host__ __device__ int64_t oplen() const { return (int64_t)((a >> 42) | ((b >> 40) << 22)); }
  __host__ __device__ int64_t key() const { return ps() + (code() == 3); }   // 'D': ps + 1 (rpc.py:41-45)
};

// One node produced by a variant (expand_variant, mh_splice.hip): src = offset into the region's reference bytes
// ('='), into the variant's alt bytes ('X' / 'I'), or -1 ('D').
struct VarNode {
  int64_t ps, pr, oplen, src;
  uint8_t op;
};
__host__ __device__ int expand_variant(uint8_t o, int64_t vp, int64_t oplen, int64_t rb, int64_t sp, int64_t rs,
                                       VarNode out[2], int64_t *sp_next, int64_t *rp_next);

constexpr int NODE_BKT_SHIFT = 8;   // 256 bp per node-search bucket (~0.7 nodes per bucket at 1.3 variants/kbp)

// A haplotype's node search (searchsorted(keys, x, 'right'), rpc.py:127-130) for the sampling side: the geometric
// cumsum's store finds each draw's start node while the positions are still in sorted order (neighbouring draws, the
// same buckets: cached), and packs it into the position's top bits (TS_NODE_SHIFT), so the shuffle carries it for free
// and the measure pass starts from it instead of searching in shuffled order.  nd == nullptr: no node index.
constexpr int TS_NODE_SHIFT = 40;                                  // positions < 2^40 (Node16's own bound)
constexpr int64_t TS_POS_MASK = ((int64_t)1 << TS_NODE_SHIFT) - 1;
struct NodeIdx {
  const Node16 *nd = nullptr;
  const int32_t *bkt = nullptr;
  int64_t n_bkt = 0, n_nodes = 0, p_min = 0;
};
__device__ __forceinline__ int64_t node_idx_upper(const NodeIdx &h, int64_t x) {
  int64_t k = (x - h.p_min) >> NODE_BKT_SHIFT, lo = 0, hi = h.n_nodes;
  if (k >= 0) {
    if (k >= h.n_bkt) k = h.n_bkt - 1;
    lo = h.bkt[k];
    hi = k + 1 < h.n_bkt ? h.bkt[k + 1] : h.n_nodes;
  }
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (h.nd[mid].key() <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
struct Hap;
inline NodeIdx node_idx_of(const Hap &h);
// the packed word: position | (start node + 1) << TS_NODE_SHIFT (0: none)
__device__ __forceinline__ int64_t ts_pack(const NodeIdx &h, int64_t v) {
  if (!h.nd || v < 0 || v > TS_POS_MASK || h.n_nodes >= ((int64_t)1 << (63 - TS_NODE_SHIFT)) - 1) return v;
  return v | node_idx_upper(h, v) << TS_NODE_SHIFT;   // (upper_bound = start node + 1)
}

// Read windows the splice bounds a read's qname part for (k_part_bound): the single-pass writer sizes its qname rows
// and reserves arena bytes from the bound of the smallest window >= rlen, before any template is measured.
constexpr int PB_NW = 4;   // (eight windows cost 35 us per chr1 haplotype, rebuilt every step)
constexpr int32_t PB_W[PB_NW] = {100, 150, 250, 321};

// The next sampling batch's word streams, generated on the prefetch stream into their own buffer (prefetch_words);
// sample_head takes the buffer when its batch has the same units (seeds, spans) and p
struct PrefetchedWords {
  bool valid = false;
  double p = 0.0;
  std::vector<uint64_t> seeds;
  std::vector<int64_t> p_min, p_max;
  int64_t words_total = 0;
  DevBuf buf, jobs;
};

struct Hap {
  bool valid = false;
  mutable hipEvent_t used = nullptr;   // after the last FASTQ writer that reads it (writer stream)
  mutable bool used_set = false;
  DevBuf hap, rc, keys, ps, pr, op, oplen, nrun_s, nrun_e;   // rc: reverse complement of hap (mate-1 reads)
  DevBuf nd;    // Node16 copy of the node arrays
  DevBuf bkt;   // node search buckets: bkt[k] = first node with key >= p_min + k * 2^NODE_BKT_SHIFT
  int64_t n_bkt = 0;
  int64_t n_nodes = 0, n_runs = 0, p_min = 0, p_max = 0, hap_len = 0, ref_start_pos = 0;
  // k_part_bound: per window PB_W[w], the most bytes the nodes of one read add to its qname part (counts, ops,
  // variant sizes); the largest POS a read can have
  bool bound_valid = false;
  int32_t part_w[PB_NW] = {0};
  int64_t pos_max = 0;
  bool prefetched = false;   // built by mh_prefetch_haplotypes_vset, not yet joined (join_prefetch)
};
inline NodeIdx node_idx_of(const Hap &h) {
  NodeIdx n;
  if (h.valid && h.n_nodes > 0 && h.nd.p && h.bkt.p) {
    n.nd = (const Node16 *)h.nd.p;
    n.bkt = (const int32_t *)h.bkt.p;
    n.n_bkt = h.n_bkt;
    n.n_nodes = h.n_nodes;
    n.p_min = h.p_min;
  }
  return n;
}

// One work unit's templates (illumina.generate_reads output), device-resident.
// mh_emit_prepare's results for a template set: the measure pass and record offsets already in buffer set `set`
struct E3h {
  int64_t kept, b1, b2;
};
struct EmitPrep {
  bool valid = false;
  int32_t set = -1, slot = -1;
  int64_t t_begin = 0, t_end = 0, cnt_base = 0;
  std::string prefix, mid;
  bool direct = true;
  E3h ht{0, 0, 0};
  int32_t hm4[4] = {0, 0, 0, 0};
  bool deferred = false;       // ht / hm4 still in the set's pinned readback (wait on its rb event)
};

struct TplSet {
  DevBuf fo0, pos0, pos1;
  DevBuf n0;                           // int32 per template: mate 0's start node (-1: unknown), when has_n0
  bool has_n0 = false;
  mutable EmitPrep prep;
  mutable hipEvent_t used = nullptr;   // after the last FASTQ writer that reads it (writer stream)
  mutable bool used_set = false;
  int64_t n = 0;
  int64_t n_draws = 0;   // the unit's template draws (n <= n_draws), known when sampling is queued
  int32_t rlen = 0;
  bool valid = false;
  int32_t pend = -1;   // unit index in ctx->tail_state while the batch's asynchronous tail has not been resolved
};

struct Contig {
  DevBuf seq;
  int64_t len = 0;
};

// One chromosome copy's variants, device-resident (the splice's input): 1-based pos, op 'X'/'I'/'D', oplen, alt
// bytes pool[aoff .. +alen).
struct VarSet {
  DevBuf pos, op, oplen, aoff, alen, pool;
  int64_t n = 0, pool_len = 0;
};

// God-aligner record store (mh_bam.hip): parsed FASTQ -> BAM records, resident until mh_bam_write.
struct BamStore {
  bool refs_set = false;
  std::vector<std::string> ref_names;
  std::vector<int64_t> ref_len;
  DevBuf names, name_off;      // @SQ names on the device (concatenated + offsets)
  DevBuf in1, in2;             // staged host FASTQ chunks
  DevBuf nl1, nl2;             // newline positions of the current input
  DevBuf tpl;                  // per-template parse results
  DevBuf roff, recs;           // record offsets [n_rec + 1] / bytes (input order)
  DevBuf key, val, info;       // sort key, record index, BAI info per record
  DevBuf key2, val2, sort_tmp, soff, srecs, sinfo;   // sorted
  DevBuf bai_lin, bai_runs, bai_out;                  // the BAI's device plan (mh_bam.hip bam_bai_plan)
  // ranks (configs[4] on N GPUs): each record's global input index (tie), which orders equal keys when records
  // arrive from several ranks (use_tie); the range partition's scratch and packed segments (mh_bam_partition)
  DevBuf tie, tie2, tval, tkey;
  DevBuf part_dest, part_dk, part_ord, part_soff, part_start, part_seg, part_split, part_tmp, send;
  bool use_tie = false;
  int64_t send_bytes = 0;
  int64_t n_rec = 0, bytes = 0;
  int32_t n_files = 0;
  bool sorted = false;         // soff/sinfo (and srecs unless spilled) hold the current store in coordinate order
  bool direct = false;         // ... written there straight from the parse (no input-order copy in recs yet)
  // Bounded HBM (mh_bam_set_capacity): the records' bytes beyond `cap` leave HBM.  The store's input-order prefix
  // [0, spilled) lives in host blocks; recs holds [spilled, bytes).  Keys, offsets and BAI info of every record stay
  // in HBM (~36 B per record), so the coordinate sort is one device sort of the keys; the sorted byte stream is
  // assembled on the host window by window and deflated on the device (mh_bam_write_gpu) or the host.
  int64_t cap = 0;             // record bytes held in HBM before a spill (0: no limit)
  struct HostBlock {
    uint8_t *p;
    int64_t b0, b1;            // the store's input-order bytes [b0, b1)
    bool mapped = false;       // an unlinked temporary file mapped in (spill_dir), else malloc
  };
  std::vector<HostBlock> spill;
  int64_t spilled = 0;
  std::string spill_dir;       // mh_bam_set_spill_dir: spill to files there (the page cache, not anonymous memory)
};

struct StageTime {
  const char *name;
  hipEvent_t a, b;
};

}  // namespace mh

namespace mh {
// One set of emission buffers (records, tile sums and prefixes, offsets).  Sets rotate so the FASTQ writers of earlier
// units (on the writer stream) overlap the measure passes of later ones and the next job's sampling (main stream).
struct EmitSet {
  DevBuf recs, off;            // per template: k_emit_measure's records; offsets (LDS-image writer only)
  DevBuf tsum, tpre;           // per 32-template tile: sums (kept, bytes per file) and their exclusive prefixes
  DevBuf crrec;                // corruption: per record the first base's offset and S (k_cr_recs)
  DevBuf stat;                 // the measure pass's totals (E3 at 0) and maxima (int32[4] at 32)
  int64_t *h_stat = nullptr;   // pinned: stat's readback (64 B), then the qname prefix (+64) and mid (+4160) staged
  hipEvent_t rb = nullptr;     // after that copy
  hipEvent_t done = nullptr;   // the last writer that read this set
  bool busy = false;
  bool prepared = false;       // holds a prepared unit whose writer is not queued yet
};
}  // namespace mh

struct mh_ctx {
  int fault_slot = 0;   // this context's look-back scan fault word (mh_scan.h)
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;   // second sampling lane: per-unit finish stages of odd units run here
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // FASTQ writer stream: mh_emit_reads returns once its writer is queued here; every other entry point first makes
  // the main stream wait for the last queued writer (ev_writer)
  hipStream_t wstream = nullptr;
  // a batch whose per-unit tail (chase, template lengths, compaction) is queued on stream2 without a host wait
  // (mh_sample_units_async): its template sets are resolved one by one (tpl_resolve) as they are used
  std::shared_ptr<void> tail_state;
  int64_t *h_units = nullptr, *d_units = nullptr;   // mapped host memory: per unit m, status, flag, done
  hipEvent_t ev_ready = nullptr, ev_writer = nullptr;
  bool writer_pending = false;
  // emission buffer sets in flight: a unit's measure pass refills the set the writer N_ESET units back read, so with
  // fewer sets than a batch's units the host (waiting for each unit's measure totals) is held until the batch's
  // writers are nearly done and the next batch's sampling cannot start beside them
  static constexpr int N_ESET = 16;
  mh::EmitSet eset[N_ESET];
  int64_t eset_max_m = 0;   // the most templates a unit had: every set is sized for it (no growth, no drain, later)
  int eset_i = 0;
  hipStream_t stage_stream = nullptr;   // stream the stage timing events go to (nullptr: stream)
  std::string err;
  int32_t max_cu = 256;

  std::map<int32_t, mh::Contig> contigs;
  std::map<int32_t, mh::Hap> haps;

  // template sets by id; `cur_tpl` is the one mh_emit_reads / mh_get_templates use
  std::map<int32_t, mh::TplSet> tsets;
  int32_t cur_tpl = -1;

  // MT19937 jump polynomials on the device (x^(k * SEG_WORDS) mod P, k < jump_k)
  mh::DevBuf jump_polys;
  int64_t jump_k = 0, jump_seg = 0;
  int64_t fixups = 0;   // units redone on the exact fallback path
  std::map<int32_t, mh::VarSet> vsets;   // resident variant sets (mh_upload_variants); id -1: mh_build_haplotype's
  std::vector<mh::Hap> hap_spare;   // released haplotypes' buffers, reused by the next build (no hipMalloc/hipFree)
  mh::DevBuf perm_tmp;  // radix sort scratch (permutation, N runs)
  mh::DevBuf pb[6];     // batch-wide permutation: ts, shuffled ts, global keys, sorted keys, sorted steps, heads
  mh::DevBuf pb_tmp;    // its radix sort scratch
  mh::DevBuf gz_slots, gz_info, gz_off, gz_scan, gz_out, gz_in;   // device BGZF (mh_deflate.hip)
  mh::DevBuf gz_tok;                                               // ... its pass-1 tokens per wave
  // mh_output_bgzf_pair: gz_out in two halves used by alternate calls; per half the event after its copies (stream2)
  hipEvent_t ev_gz[2] = {nullptr, nullptr};
  hipEvent_t ev_fetch[2] = {nullptr, nullptr};   // mh_output_fetch_async: per ticket, after both files' copies
  bool fetch_pending[2] = {false, false};
  int fetch_next = 0;
  bool gz_pending[2] = {false, false};
  int gz_half = 0;
  mh::DevBuf nrun_tmp;  // unsorted N-run boundaries
  mh::DevBuf dec_buf;   // chunk-parallel shuffle decode: chunk jobs, starts, counts, work list
  int64_t dec_passes = 0;   // count passes of the last chunk-parallel decode (diagnostics)

  // scratch (grow-only), reused by all stages
  mh::DevBuf s[16];
  mh::DevBuf scan_partials;
  mh::DevBuf lane2[8];   // the second lane's copies of s[4..10] and its radix-sort scratch (index 7)
  mh::DevBuf scan_partials2;
  // lanes 2 and 3 (a four-unit job's units each on a lane of their own): streams, scratch, join events
  hipStream_t xstream[2] = {nullptr, nullptr};
  mh::DevBuf xlane[2][8];
  mh::DevBuf xscan[2];
  hipEvent_t ev_xjoin[2] = {nullptr, nullptr};
  mh::DevBuf sl2[8];   // the splice's second lane: anchor, accepted, ref_before, node src, small, partials, N runs, sort
  // mh_prefetch_haplotypes_vset: the next batch's splices issued by a host thread of the context on a stream of their
  // own (the fourth: GPU_MAX_HW_QUEUES is 4) with their own scratch and pinned readback block
  hipStream_t pstream = nullptr;
  hipEvent_t ev_prefetch = nullptr;   // after the last prefetched splice
  bool prefetch_pending = false;      // some Hap has prefetched set
  std::thread pf_thread;              // the host thread issuing the prefetched splices (their readbacks wait there)
  int32_t pf_rc = 0;                  // its result
  mh::DevBuf sl3[8];
  int64_t *h_small3 = nullptr;
  mh::PrefetchedWords pf_words;       // the next batch's MT19937 word streams (prefetch_words), or none
  mh::DevBuf pinned_small;   // host-visible small readback area (hipHostMalloc)
  mh::DevBuf d_small;        // device small scalars

  // fused corruption (mh_set_corruption)
  bool corrupt_on = false;
  mh::DevBuf corrupt_cum, corrupt_phred;
  int32_t corrupt_max_bp = 0, corrupt_n_bq = 0;
  size_t corrupt_guide_off = 0;   // byte offsets inside corrupt_cum: the search guide, the Philox-mode bucket table
  size_t corrupt_bk_off = 0, corrupt_T16_off = 0, corrupt_Fp16_off = 0;   // and the u16 tables T16, Fp16
  size_t corrupt_bkf_off = 0;                                               // the row pass's fine bucket table
  uint64_t corrupt_seed = 0;
  // exact corruption stream of mh_corrupt_fastq (mh_corrupt_stream_seed / _state): 0 = Philox; 1 = the stream of
  // RandomState(cx_seed) from output cx_pos on; 2 = continuing the explicit state (cx_key, cx_kpos)
  int32_t cx_mode = 0;
  uint32_t cx_seed = 0;
  int64_t cx_pos = 0;
  uint32_t cx_key[624] = {0};
  int32_t cx_kpos = 624;
  mh::DevBuf cx_words, cx_bits, cx_start, cx_aux;

  // emission: emit_lds_only forces the LDS-image writer (A/B and fallback testing)
  bool emit_lds_only = false;
  bool decode_sequential = false;   // MH_DEC_SEQUENTIAL: block-sequential shuffle decode only
  bool force_fixup = false;         // MH_DEC_FORCE_FIXUP: every unit through the single-stream decode fix-up
  bool force_geo = false;           // MH_DEC_FORCE_GEO: every unit's geometric draws recomputed on the host

  // FASTQ arenas
  mh::DevBuf out1, out2;
  int64_t used1 = 0, used2 = 0;
  // single-pass emission (mh_emit_reads_async, k_emit_fused): units queued on the writer stream with no host wait.
  // Each writer's last tile writes the unit's totals to mapped host memory (h_lazy, LZ_SLOTS slots of 8 words) and
  // the arena ends to the device cursor ring (d_cur) the next unit's writer starts from.  While a chain is open the
  // host knows only an upper bound of the arena ends (used_ub); lazy_resolve waits for the writers and makes
  // used1/used2 exact again.  Units queued before an mh_output_reset belong to an older generation: their totals are
  // still collected, their ends no longer move the arenas.
  static constexpr int LZ_SLOTS = 4096;
  int64_t *h_lazy = nullptr, *d_lazy = nullptr;
  mh::DevBuf d_cur;                 // LZ_SLOTS + 1 cursors of 4 words: kept, end file 1, end file 2, -
  mh::DevBuf fused_lb;              // the single-pass writer's look-back scratch (writer stream)
  struct LazyUnit {
    int32_t slot;                   // h_lazy slot (-1: totals already known, in `known`)
    int64_t gen;
    int64_t known[3];
  };
  std::vector<LazyUnit> lazy;       // queued, not resolved
  std::vector<int64_t> lazy_done;   // resolved totals (3 per unit, queue order) for mh_emit_collect
  int64_t lazy_seq = 0;             // units queued on the chain so far (cursor ring position)
  int64_t lazy_gen = 0;
  bool chain_open = false;
  int64_t used_ub1 = 0, used_ub2 = 0;
  int64_t batch_left = 0;           // draws of the last sampled batch's units not emitted yet (arena reservation)
  bool emit_two_pass = false;       // mh_set_emit_mode(2): every unit through mh_emit_reads' path (host readbacks)
  bool emit_single = false;         // mh_set_emit_mode(3): the single-pass writer (k_emit_fused)
  // corruption rows (the direct writer's mode): per block 15 qualities | 2-bit codes; one set, the row pass and its
  // writer in stream order on the writer stream
  mh::DevBuf cr_rows, cr_codes;
  mh::DevBuf scan_partials_w;            // look-back scratch of the writer stream's scans
  int64_t *h_small = nullptr;            // pinned 4 KiB for small readbacks (no staged copy per value)
  uint8_t *h_bam_pin[2] = {nullptr, nullptr};   // mh_bam_write_gpu's two 64 MiB D2H slots (kept: page-locking
                                                // 128 MiB per BAM file cost ~13 ms)

  // timing
  bool timing = false;
  std::vector<mh::StageTime> stages;    // open (begun, not ended)
  std::vector<mh::StageTime> pending;   // ended, not yet resolved
  std::vector<std::pair<const char *, double>> last_times;

  // god-aligner BAM records
  mh::BamStore bam;
};

namespace mh {

int32_t hip_fail(mh_ctx *ctx, hipError_t e, const char *what, const char *file, int line);
int32_t arg_fail(mh_ctx *ctx, int32_t code, const std::string &msg);

#define HIPCHK(ctx, call)                                                     \
  do {                                                                        \
    hipError_t _e = (call);                                                   \
    if (_e != hipSuccess) return ::mh::hip_fail((ctx), _e, #call, __FILE__, __LINE__); \
  } while (0)

// A host synchronisation, then the look-back scans' fault word (mh_scan.h): a scan that timed out since the last check
// fails the call instead of its wrong offsets being used
int32_t scan_fault_fail(mh_ctx *ctx);
#define SYNCCHK(ctx, call)                                                    \
  do {                                                                        \
    HIPCHK(ctx, call);                                                        \
    if (::mh::scan_fault_pending(ctx)) return ::mh::scan_fault_fail(ctx);     \
  } while (0)
bool scan_fault_pending(const mh_ctx *ctx);

// Grow `b` to hold at least `bytes`; contents are NOT preserved.
int32_t ensure(mh_ctx *ctx, DevBuf &b, size_t bytes);
// Grow preserving the first `keep` bytes (stream-ordered copy); the new capacity is bytes + bytes >> grow_shift (and
// ensure's eighth).
int32_t ensure_keep(mh_ctx *ctx, DevBuf &b, size_t bytes, size_t keep, int32_t grow_shift = 1);
void release(DevBuf &b);
void release_hap(Hap &h);
int32_t join_writer(mh_ctx *ctx);   // main stream waits for the last queued FASTQ writer
// a resource a queued FASTQ writer reads: mark it (writer stream) / make the main stream wait before overwriting it
int32_t mark_used(mh_ctx *ctx, hipEvent_t &ev, bool &set);
int32_t wait_unused(mh_ctx *ctx, hipEvent_t ev, bool set, hipStream_t st = nullptr);   // st: ctx->stream when null
int32_t join_prefetch(mh_ctx *ctx);
// The MT19937 word streams of a sampling batch (units' spans and seeds, p; rng mode mitty) generated on `st` into
// ctx->pf_words (the prefetch thread, after the next batch's splices); skipped (no error) while the jump polynomials
// the batch needs are not resident yet
int32_t prefetch_words(mh_ctx *ctx, hipStream_t st, int32_t n_units, const int64_t *p_min, const int64_t *p_max,
                       const uint64_t *seeds, double p);   // the prefetch thread joined, the main stream after its splices

// Stage timing (HIP events on ctx->stream).
void stage_begin(mh_ctx *ctx, const char *name);
void stage_end(mh_ctx *ctx);
void stages_collect(mh_ctx *ctx);

// Launch helpers
inline unsigned grid_for(int64_t n, int threads, int64_t cap = 1 << 20) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---- subsystem entry points (host side, called from mh_api.cpp) -----------------------------------------------
int32_t var_upload(mh_ctx *ctx, VarSet &v, const int64_t *v_pos, const uint8_t *v_op, const int64_t *v_oplen,
                   const int64_t *v_alt_off, const int64_t *v_alt_len, const char *alt_pool, int64_t alt_pool_len,
                   int64_t n_var);
void release_vars(VarSet &v);
// lane 0: ctx->stream and the shared scratch; lane 1: ctx->stream2 and sl2 (a second host thread)
int32_t splice_build(mh_ctx *ctx, Hap &h, const Contig &c, int64_t ref_start_pos, const VarSet &v, int lane = 0);

// nidx: per unit its haplotype's node search (the start nodes then travel packed in the positions), or null
int32_t sample_units(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int64_t *p_min, const int64_t *p_max,
                     const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                     int32_t rng_mode, int64_t *out_n, const NodeIdx *nidx = nullptr);
int32_t sample_units_async(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int64_t *p_min,
                           const int64_t *p_max, const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen,
                           int32_t n_tlen, int32_t rng_mode, const NodeIdx *nidx = nullptr);
// a template set of an asynchronous tail: wait for its unit (host), read its count, run the rare exact fix-up, and
// order the main stream after it; no-op for a resolved set
int32_t tpl_resolve(mh_ctx *ctx, TplSet &ts);
int32_t tpl_resolve_all(mh_ctx *ctx);

// FASTQ emission of the current template set's [t_begin, t_end) (mh_emit_reads); prepare_only: the measure pass and
// record offsets only, kept for the next emit_reads of the same unit (mh_emit_prepare)
int32_t sync_writers(mh_ctx *ctx);   // the writer stream and the corruption stream drained (host wait)
int32_t bgzf_device(mh_ctx *ctx, hipStream_t st, const uint8_t *d_in, int64_t n, uint8_t *d_out, int64_t cap,
                    int64_t *used, std::vector<int64_t> *boff = nullptr,
                    const std::function<void(int64_t, int64_t)> *on_piece = nullptr);
                    // BGZF blocks of a device buffer (no EOF marker), mh_deflate.hip; boff: each block's offset in
                    // d_out (+ the end), for a BAI; on_piece(offset, bytes): a piece of d_out is queued on `st` (the
                    // caller may copy it out behind that point while the next piece deflates)
int64_t bgzf_device_bound(int64_t n);
int gpu_numa_node(int dev);   // the NUMA node of the device's PCI function (sysfs), -1 when unknown
std::mutex &host_allocs_mu();  // mh_host_alloc's node-bound registrations (address -> bytes)
std::unordered_map<void *, size_t> &host_allocs();
int64_t *pinned_small(mh_ctx *ctx);     // ctx->h_small (allocated on first use); nullptr on failure
int32_t emit_reads(mh_ctx *ctx, const Hap &h, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                   int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end, int64_t cnt_base,
                   bool prepare_only, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2);
int32_t count_kept(mh_ctx *ctx, const Hap &h, int64_t t_begin, int64_t t_end, int64_t *out_kept);
// One whole unit of the current template set through the single-pass writer, queued with no host wait (its totals
// resolved by lazy_resolve).  *queued false (MH_OK): the unit does not qualify (the caller takes the two-pass path).
int32_t emit_unit_async(mh_ctx *ctx, const Hap &h, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, bool *queued);
// Waits for the queued single-pass writers, moves their totals to lazy_done and makes used1/used2 exact.
int32_t lazy_resolve(mh_ctx *ctx);

int32_t bam_set_refs(mh_ctx *ctx, int32_t n_refs, const char *names, const int64_t *lengths);
int32_t bam_add(mh_ctx *ctx, const uint8_t *d1, int64_t len1, const uint8_t *d2, int64_t len2, int64_t max_templates,
                int64_t *used1, int64_t *used2, int64_t *templates, bool sorted_direct = false);
int32_t bam_sort(mh_ctx *ctx, const void *pa = nullptr);
int32_t bam_undirect(mh_ctx *ctx);
int32_t bam_fetch_sorted(mh_ctx *ctx, uint8_t *recs, int64_t *soff, int32_t *info);
int32_t bam_spill(mh_ctx *ctx);   // the device-resident records to a host block (input order)
int32_t bam_export(mh_ctx *ctx, int64_t r0, int64_t r1, uint8_t *recs, int64_t *roff, uint64_t *key, int32_t *info);
int32_t bam_import(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *key, const int32_t *info,
                   int64_t n, const uint64_t *tie = nullptr);
// the store's records by destination rank: dest = the number of splitters <= the record's key; packed per
// destination (bam_part_layout, input order inside each) into B.send; seg_off[d] / seg_n[d] / seg_bytes[d]
int32_t bam_partition(mh_ctx *ctx, const uint64_t *split, int32_t n_dest, uint64_t tie_base, int64_t *seg_off,
                      int64_t *seg_n, int64_t *seg_bytes);
// the raw device BAI plan of the sorted store (per run: tid << 32 | bin, first offset, end offset, records; per window
// its first record's offset or -1; per reference its window count); *ok false: outside the device plan's checks
int32_t bam_bai_raw(mh_ctx *ctx, std::vector<int64_t> &runs, std::vector<int64_t> &win, std::vector<uint32_t> &nwin,
                    std::vector<int64_t> &woff, bool *ok);
// the sorted store's byte stream [w0, w1) into dst (host), from the host blocks (every record spilled); the sorted
// order (val2), input offsets (roff) and sorted offsets (soff) as host copies (bam_host_order)
struct BamHostOrder {
  std::vector<uint32_t> val;
  std::vector<int64_t> roff, soff;
};
int32_t bam_host_order(mh_ctx *ctx, BamHostOrder &o);
void bam_assemble(const BamStore &B, const BamHostOrder &o, int64_t w0, int64_t w1, uint8_t *dst, int threads);
struct BaiPlan;
// The BAI's per-record half on the device (sorted store): chunks and linear index as positions in `offs`, the
// compact array of the data offsets they need.  *ok = false (and MH_OK) when the records are outside what the
// device plan checks (a record past its reference's length, an unsorted store): the caller then plans on the host.
int32_t bam_bai_plan(mh_ctx *ctx, BaiPlan &plan, std::vector<int64_t> &offs, bool *ok);
void bam_release(BamStore &B);
void bam_free_spill(BamStore &B);
int32_t newline_index(mh_ctx *ctx, const uint8_t *b, int64_t len, DevBuf &nl, int64_t *count);
int32_t corrupt_fastq(mh_ctx *ctx, const uint8_t *d0, int64_t len0, const uint8_t *d1, int64_t len1, int64_t t_base,
                      int64_t *used0, int64_t *used1, int64_t *templates);

int32_t read_batch(mh_ctx *ctx, const Hap &h, const int64_t *p, const int64_t *l, int64_t n, int64_t *out_pos,
                   int64_t *out_n0, int64_t *out_n1, char *cigar, int64_t cigar_cap, int64_t *cigar_off,
                   int64_t *cigar_used, char *vlist, int64_t vlist_cap, int64_t *vlist_off, int64_t *vlist_used,
                   char *seq, int64_t seq_cap, int64_t *seq_off, int64_t *seq_used);


// MT19937 word streams for exact corruption (mh_sample.hip).  mt_stream_words: outputs [first, first + count) of
// RandomState(seed) generated as whole jump-ahead segments into `out`; output `first` sits at out[*lead].
// mt_state_words: `count` outputs continuing an explicit state (numpy get_state(): raw key, pos) into out[0..).
int32_t mt_stream_words(mh_ctx *ctx, hipStream_t st, uint32_t seed, int64_t first, int64_t count, DevBuf &out,
                        DevBuf &jobs_buf, int64_t *lead);
int32_t mt_state_words(mh_ctx *ctx, hipStream_t st, const uint32_t *key624, int32_t pos, int64_t count, DevBuf &out,
                       DevBuf &key_buf);

// The corruption configuration of a launch (mh_set_corruption's tables; Philox key from the unit).
struct CorruptCfg;
CorruptCfg corrupt_cfg(const mh_ctx *ctx, uint64_t unit_key, int64_t t_base);

// Host-side MT19937 (numpy RandomState seeding), used for seed derivation and the rare exact fix-ups.
struct HostMT {
  uint32_t key[624];
  int pos;
  void seed(uint32_t s);
  uint32_t next();
  double next_double();
  uint64_t interval(uint64_t max);
};

}  // namespace mh
