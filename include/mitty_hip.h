/* mitty_hip.h — C ABI of libmitty_hip.so, the MI355X (gfx950) generate-reads engine.
 *
 * Plain C types only (pointers + sizes); no torch / HIP types cross this boundary.  Every call returns an int32
 * status (MH_OK == 0, negative = error) and leaves a message in mh_last_error(ctx).  The Python package
 * mitty_amd binds this with ctypes (mitty_amd/_native.py); INTEGRATION.md shows the binding a maintainer of the
 * reference would add.
 *
 * Which reference interface each entry point replaces (paths relative to the reference repo root):
 *   mh_upload_contig      pysam.FastaFile.fetch of a BED region          mitty/simulation/readgenerate.py:181,186
 *   mh_build_haplotype    rpc.create_node_list (+ rpc.Node)              mitty/simulation/rpc.py:5-116
 *                         fed by vcfio.split_copies/parse per copy       mitty/lib/vcfio.py:67-126
 *   mh_upload_variants    (the same copy's variant list, kept resident; mh_build_haplotype_vset splices from it)
 *   mh_sample_templates   illumina.generate_reads                        mitty/simulation/illumina.py:43-110
 *   mh_sample_units       (the same for many units: the worker pool of readgenerate.py:102-115)
 *   mh_set_templates      (the template arrays a read module returns)   mitty/simulation/illumina.py:79-110
 *   mh_get_templates      (same arrays back to the host)
 *   mh_emit_reads         read_generating_worker loop + fastq_lines      mitty/simulation/readgenerate.py:184-230
 *   mh_read_batch         rpc.get_begin_end_nodes + rpc.generate_read    mitty/simulation/rpc.py:119-160
 *   mh_expand_variant     rpc.create_nodes / snp / insertion / deletion  mitty/simulation/rpc.py:66-116
 *   mh_set_corruption     illumina.corrupt_template / corrupt_single_read mitty/simulation/illumina.py:113-162
 *   mh_set_corruption_stream  corrupt_rng = RandomState(seed) of a worker  mitty/simulation/readcorrupt.py:84
 *   mh_corrupt_fastq      readcorrupt.multi_process's reader/worker/writer  mitty/simulation/readcorrupt.py:18-118
 *   mh_work_units         readgenerate.get_data_for_workers              mitty/simulation/readgenerate.py:129-159
 *   mh_read_model_params  illumina.read_model_params                     mitty/simulation/illumina.py:12-40
 *
 * Threading: one mh_ctx per GPU and per host thread; a context owns one HIP stream and all device buffers.
 * Calls are synchronous at return (device work is ordered on the context's stream; results copied back are
 * complete).  Outputs of mh_emit_reads stay device-resident in the context's FASTQ arenas until fetched.
 */
#ifndef MITTY_HIP_H
#define MITTY_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mh_ctx mh_ctx;

enum {
  MH_OK = 0,
  MH_E_ARG = -1,              /* bad argument (ValueError in the Python facade) */
  MH_E_HIP = -2,              /* HIP runtime error */
  MH_E_OOM = -3,              /* device allocation failed */
  MH_E_CAPACITY = -4,         /* caller buffer too small: *used / *needed says how much */
  MH_E_COMPLEX_VARIANT = -5,  /* a variant that is not SNP/INS/DEL (vcfio.py:124 ValueError) */
  MH_E_SEED = -6,             /* seed outside 0..2^32-1 (illumina.py:53-54 ValueError) */
  MH_E_STATE = -7,            /* call out of order (e.g. emit before sampling) */
  MH_E_NO_DEVICE = -8         /* no HIP device */
};

enum { MH_RNG_MITTY = 0, MH_RNG_PHILOX = 1 };

/* ---- context ------------------------------------------------------------------------------------------- */
int32_t mh_version(void);
int32_t mh_device_count(int32_t *out);
int32_t mh_create(int32_t device, mh_ctx **out);
int32_t mh_destroy(mh_ctx *ctx);
const char *mh_last_error(const mh_ctx *ctx);
/* Synchronise the context's stream. */
int32_t mh_sync(mh_ctx *ctx);

/* Self-test of the look-back scans' fault report (no reference counterpart: the device offsets the scans produce —
 * FASTQ record offsets, BAM record and BGZF block offsets — must never be wrong silently).  Runs a scan whose tile 0
 * never publishes; returns MH_E_STATE when the timed-out wait was reported (the expected result), then checks that a
 * correct scan after it succeeds. */
int32_t mh_selftest_scan_fault(mh_ctx *ctx);
/* Self-test of the permutation's radix sort (mh_sort.h; the stable (target, step) sort that replaces replaying
 * illumina.py:70's shuffle): keys[0, n) (host) sorted on the device over bits [0, end_bit); keys_out / vals_out (host,
 * n each) get the sorted keys and their input indices, equal keys in input order. */
int32_t mh_selftest_sort(mh_ctx *ctx, const uint32_t *keys, int64_t n, int32_t end_bit, uint32_t *keys_out,
                         uint32_t *vals_out);

/* ---- host-side helpers that mirror the reference's scalar logic ---------------------------------------- */
int32_t mh_read_model_params(int64_t mean_rlen, double coverage, double *p, int64_t *passes);
/* Work units in the reference's shuffled order; arrays sized sum(ploidy) * passes. */
int32_t mh_work_units(uint64_t seed, const int32_t *ploidy, int64_t n_regions, int64_t passes,
                      int32_t *out_region, int32_t *out_cpy, uint32_t *out_seed, int64_t *out_n);

/* ---- reference sequence and haplotypes ----------------------------------------------------------------- */
/* Upload (or replace) contig `contig_id` — the bytes of one BED region as fetched from the FASTA. */
int32_t mh_upload_contig(mh_ctx *ctx, int32_t contig_id, const char *seq, int64_t len);
/* Splice one chromosome copy on the device: variants (1-based pos, op 'X'/'I'/'D', oplen, alt bytes in
 * alt_pool[alt_off .. +alt_len)) applied to contig `contig_id`, whose first base has 1-based coordinate
 * ref_start_pos.  Result kept in haplotype slot `slot`.  Outputs: node count, p_min, p_max (rpc/readgenerate.py:192). */
int32_t mh_build_haplotype(mh_ctx *ctx, int32_t slot, int32_t contig_id, int64_t ref_start_pos,
                           const int64_t *v_pos, const uint8_t *v_op, const int64_t *v_oplen,
                           const int64_t *v_alt_off, const int64_t *v_alt_len, const char *alt_pool,
                           int64_t alt_pool_len, int64_t n_var,
                           int64_t *out_n_nodes, int64_t *out_p_min, int64_t *out_p_max);
/* Resident variant sets: upload one copy's variants once (same arrays and checks as mh_build_haplotype), then
 * splice from the device copy as often as needed — the input stays in HBM across jobs. */
int32_t mh_upload_variants(mh_ctx *ctx, int32_t vset, const int64_t *v_pos, const uint8_t *v_op,
                           const int64_t *v_oplen, const int64_t *v_alt_off, const int64_t *v_alt_len,
                           const char *alt_pool, int64_t alt_pool_len, int64_t n_var);
int32_t mh_build_haplotype_vset(mh_ctx *ctx, int32_t slot, int32_t contig_id, int64_t ref_start_pos, int32_t vset,
                                int64_t *out_n_nodes, int64_t *out_p_min, int64_t *out_p_max);
/* Several mh_build_haplotype_vset calls at once: slots[i] from contig contig_ids[i] at ref_starts[i] with resident
 * variant set vsets[i]; two copies are spliced side by side (second stream, second host thread).  Outputs per slot. */
int32_t mh_build_haplotypes_vset(mh_ctx *ctx, int32_t n, const int32_t *slots, const int32_t *contig_ids,
                                 const int64_t *ref_starts, const int32_t *vsets, int64_t *out_n_nodes,
                                 int64_t *out_p_min, int64_t *out_p_max);
/* mh_build_haplotypes_vset for the NEXT batch while the current one is still being sampled and written: the call
 * takes the slots' buffers and returns; a host thread of the context issues the splices on a stream of their own (the
 * context's fourth, created on first use) with their own scratch, so nothing waits for the pending sampling tail
 * (mh_sample_units_async) or for queued measure passes.  Given the next batch's units (n_units > 0: each unit's
 * haplotype slot — prefetched here or live — and seed, and p as mh_sample_units takes them, rng mode mitty), the same
 * thread then generates their MT19937 word streams into a buffer of their own; mh_sample_units(_async) of a batch
 * with exactly those units, spans and p takes that buffer instead of generating them (the same words).  That thread is
 * joined, and the main stream waits for its work, before the first use of a prefetched haplotype (emission from its
 * slot) and in every entry point that resolves the sampling tail (sampling, builds, releases...), which also report a
 * failed splice.  The slots must be free (MH_E_ARG for a live slot); the haplotypes are byte-identical to a build.
 * (The reference builds each work unit's haplotype and draws its streams inside its worker, readgenerate.py:190,
 * illumina.py:43-110; this only moves that work earlier in the pipeline.) */
int32_t mh_prefetch_haplotypes_vset(mh_ctx *ctx, int32_t n, const int32_t *slots, const int32_t *contig_ids,
                                    const int64_t *ref_starts, const int32_t *vsets, int32_t n_units,
                                    const int32_t *unit_slots, const uint64_t *unit_seeds, double p);
int32_t mh_release_variants(mh_ctx *ctx, int32_t vset);
/* Copy a slot's node list back (arrays sized n_nodes; seq bytes of node k = hap[ps[k]-p_min .. +oplen) for
 * non-'D' nodes).  Any pointer may be NULL. */
int32_t mh_get_nodes(mh_ctx *ctx, int32_t slot, int64_t *ps, int64_t *pr, uint8_t *op, int64_t *oplen,
                     char *hap, int64_t hap_cap, int64_t *hap_len);
int32_t mh_release_haplotype(mh_ctx *ctx, int32_t slot);
/* The nodes ONE variant adds at cursors (samp_pos, ref_pos) of a region starting at ref_start_pos — the node rules
 * of the device splice (the same function runs inside it), exposed for the reference's per-variant helpers
 * rpc.snp / insertion / deletion (op 'X' / 'I' / 'D' selects the rule, as the helper name does).  Host-only, no
 * context.  out: up to 2 nodes x {ps, pr, op, oplen, src} (src: offset of an '=' node's bytes in the region's
 * reference, of an 'X' / 'I' node's bytes in the variant's alt allele, -1 for 'D'); *n_nodes = 1 or 2;
 * *samp_next / *ref_next: the cursors after the variant. */
int32_t mh_expand_variant(int64_t samp_pos, int64_t ref_pos, int64_t ref_start_pos, int64_t v_pos, int32_t op,
                          int64_t oplen, int64_t *out, int32_t *n_nodes, int64_t *samp_next, int64_t *ref_next);

/* ---- templates ----------------------------------------------------------------------------------------- */
/* illumina.generate_reads for haplotype `slot` (p_min/p_max from the slot).  rng_mode MH_RNG_MITTY reproduces
 * numpy's MT19937 streams bit for bit; MH_RNG_PHILOX is the counter-based fast mode. */
int32_t mh_sample_templates(mh_ctx *ctx, int32_t slot, double p, int32_t rlen, const double *cum_tlen,
                            int32_t n_tlen, uint64_t seed, int32_t rng_mode, int64_t *out_n_templates);
/* Same, for an explicit [p_min, p_max) span with no haplotype (the plugin-level generate_reads). */
int32_t mh_sample_templates_span(mh_ctx *ctx, int64_t p_min, int64_t p_max, double p, int32_t rlen,
                                 const double *cum_tlen, int32_t n_tlen, uint64_t seed, int32_t rng_mode,
                                 int64_t *out_n_templates);
/* Batched form: sample `n_units` work units at once (all their MT19937 streams are generated in parallel
 * jump-ahead segments).  Unit k uses haplotype slots[k] and seed seeds[k]; its templates are kept as template set
 * tpl_ids[k] (>= 0) until released.  out_n[k] = templates kept for unit k. */
int32_t mh_sample_units(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int32_t *slots,
                        const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                        int32_t rng_mode, int64_t *out_n);
/* mh_sample_units without the host wait at its end: each unit's last stages (its part of the permutation chase, its
 * template lengths and compaction; readgenerate.py:129-159 per unit) are queued in unit order on a second stream,
 * and the unit's template set is resolved when first used (mh_use_templates, mh_templates_count, or any entry
 * point other than the emission ones), so the first unit's FASTQ writer can start while later units still sample.
 * The same templates as mh_sample_units. */
int32_t mh_sample_units_async(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int32_t *slots,
                              const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                              int32_t rng_mode);
/* Templates kept in set tpl_id (waits for an asynchronous unit's tail). */
int32_t mh_templates_count(mh_ctx *ctx, int32_t tpl_id, int64_t *n);
/* Make template set `tpl_id` the current one (used by mh_emit_reads / mh_get_templates). */
int32_t mh_use_templates(mh_ctx *ctx, int32_t tpl_id);
int32_t mh_release_templates(mh_ctx *ctx, int32_t tpl_id);
int32_t mh_set_templates(mh_ctx *ctx, const int8_t *fo0, const int64_t *pos0, const int64_t *pos1, int64_t n,
                         int32_t rlen);
int32_t mh_get_templates(mh_ctx *ctx, int8_t *fo0, int64_t *pos0, int64_t *pos1, int64_t cap, int64_t *n);
/* Multi-GPU template sharing (a few-unit job samples each unit once, on one rank, and sends its
 * arrays to the ranks that emit slices of it).  on_device != 0: the pointers are device buffers of this context's
 * GPU (e.g. the buffers an RCCL broadcast fills); otherwise host memory.
 *   mh_templates_export  template set tpl_id -> fo0[n], pos0[n], pos1[n] (*n = its size; MH_E_CAPACITY if cap < n)
 *   mh_templates_import  template set tpl_id := the n templates in the buffers (rlen = read length) */
int32_t mh_templates_export(mh_ctx *ctx, int32_t tpl_id, int32_t on_device, int8_t *fo0, int64_t *pos0,
                            int64_t *pos1, int64_t cap, int64_t *n);
int32_t mh_templates_import(mh_ctx *ctx, int32_t tpl_id, int32_t on_device, const int8_t *fo0, const int64_t *pos0,
                            const int64_t *pos1, int64_t n, int32_t rlen);

/* ---- read emission ------------------------------------------------------------------------------------- */
/* Turn the current templates into FASTQ text for both files, appended to the device arenas.
 * serial_stub = "{sample}:{worker}:{ps}" (readgenerate.py:195).  unit_key keys the corruption stream (ignored when
 * corruption is off; pass the unit's rng_seed).  Outputs: kept templates, bytes appended. */
int32_t mh_emit_reads(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                      int32_t write_fastq2, uint64_t unit_key, int64_t *out_kept, int64_t *out_bytes1,
                      int64_t *out_bytes2);
/* The first half of mh_emit_reads for the current template set: the measure pass and record offsets, with the same
 * outputs.  The next mh_emit_reads of the same unit (same slot and names) only queues the writer, so a caller that
 * prepares a batch of units first (at most 4 at a time) queues their writers back to back and moves on.
 * out_kept, out_b1 and out_b2 may all be NULL: the call then returns without waiting for the measure pass (no host
 * round trip between a batch's passes); the totals are read back when the unit's mh_emit_reads queues its writer. */
int32_t mh_emit_prepare(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2);
/* A slice of a unit for multi-GPU sharding: emit only templates [t_begin, t_end) of the current
 * set, numbering the kept ones from cnt_base + 1 (cnt_base = templates kept before t_begin, e.g. from an all-gather
 * of mh_count_kept over the ranks' slices).  Concatenating the slices in order reproduces mh_emit_reads byte for
 * byte, corruption included (its stream is counted by the template's index in the whole unit). */
int32_t mh_emit_reads_range(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                            int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end,
                            int64_t cnt_base, int64_t *out_kept, int64_t *out_bytes1, int64_t *out_bytes2);
/* mh_emit_reads for a whole unit of the current template set, queued with no host wait (the same bytes at the same
 * arena offsets): the single-pass writer (k_emit_fused) finds each read's nodes, applies the N filter, measures and
 * numbers the records and takes every 32-template tile's arena offset from a decoupled look-back over the launch's
 * earlier tiles; the unit's end offsets pass to the next queued unit on the device.  No measure pass, no tile scan,
 * no readback between units (readgenerate.py:184-230's worker loop, whose outputs are appended in order).  Units the
 * single-pass writer does not cover (mh_set_emit_mode 1 or 2, qname heads over 96 bytes, reads over 321 bp, the
 * in-place corruption) take mh_emit_reads' path inside the call.
 *   mh_emit_collect  waits for the queued units and returns their (kept, bytes1, bytes2), 3 int64 per unit in queue
 *                    order (out NULL: *n_units only); every entry point that reads or appends to the arenas
 *                    (fetches, sizes, mh_emit_reads, BGZF, BAM, corrupt) first resolves the queued units itself. */
int32_t mh_emit_reads_async(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                            int32_t write_fastq2, uint64_t unit_key);
int32_t mh_emit_collect(mh_ctx *ctx, int64_t *out, int64_t cap, int64_t *n_units);
/* The byte sizes a slice [t_begin, t_end) of the current template set will emit (t_end < 0: the whole set), without
 * writing it: the measure pass and its totals only (kept templates, bytes per FASTQ file), no buffer set held.  The
 * multi-GPU writer (mitty_amd/distributed.py) all-reduces these to place every piece in the files before any piece is
 * written, so each piece is written as soon as it is emitted (readgenerate.py:233-253 streams its output).  The sizes
 * equal the later mh_emit_reads_range's outputs for the same arguments. */
int32_t mh_emit_measure(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end, int64_t cnt_base,
                        int64_t *out_kept, int64_t *out_b1, int64_t *out_b2);
/* Templates in [t_begin, t_end) of the current set that survive the N filter (readgenerate.py:201-204). */
int32_t mh_count_kept(mh_ctx *ctx, int32_t slot, int64_t t_begin, int64_t t_end, int64_t *out_kept);
int32_t mh_output_size(mh_ctx *ctx, int64_t *bytes1, int64_t *bytes2);
/* Copy arena bytes [offset, offset+len) of file 1 / file 2 to host (either host pointer may be NULL). */
int32_t mh_output_fetch(mh_ctx *ctx, int64_t offset1, char *fq1, int64_t len1, int64_t offset2, char *fq2,
                        int64_t len2);
/* The same copies queued (file 1 and file 2 on two streams, after the queued writers) without a host wait: the
 * bytes are in fq1 / fq2 after mh_output_fetch_wait(ticket).  Two fetches may be in flight, so the DMA engines stay
 * busy while the host writes the previous chunk (readgenerate.py:233-253's file writes).  mh_output_reset waits for
 * pending fetches. */
int32_t mh_output_fetch_async(mh_ctx *ctx, int64_t offset1, char *fq1, int64_t len1, int64_t offset2, char *fq2,
                              int64_t len2, int32_t *ticket);
int32_t mh_output_fetch_wait(mh_ctx *ctx, int32_t ticket);
int32_t mh_output_reset(mh_ctx *ctx);
/* Page-locked host memory for mh_output_fetch destinations (D2H at full link rate; the FASTQ sink writes from it). */
int32_t mh_host_alloc(int64_t bytes, void **out);
int32_t mh_host_free(void *p);
/* Device memory the library freed is kept in a process-wide cache (per device) for later requests, so a context
 * created after another closed reuses blocks allocated while device memory was unfragmented; an allocation that
 * fails empties the cache first.  This frees every cached block now (*freed_bytes: their total). */
int32_t mh_device_cache_trim(int64_t *freed_bytes);
/* Bytes of the library's device blocks in use (not in the cache), process-wide, and their peak since the last reset
 * (reset_peak != 0: the peak restarts from the current value after it is read).  Lets a caller check a bound such
 * as mh_bam_set_capacity's. */
int32_t mh_device_live_bytes(int64_t *live, int64_t *peak, int32_t reset_peak);

/* rpc.generate_read for a batch of (p, l) on haplotype `slot`: positions, start/end nodes and the text fields.
 * Text outputs are concatenated; *_off arrays (n+1 entries) index them.  MH_E_CAPACITY if a text buffer is short
 * (needed sizes returned in *cigar_used / *vlist_used / *seq_used). */
int32_t mh_read_batch(mh_ctx *ctx, int32_t slot, const int64_t *p, const int64_t *l, int64_t n,
                      int64_t *out_pos, int64_t *out_n0, int64_t *out_n1,
                      char *cigar, int64_t cigar_cap, int64_t *cigar_off, int64_t *cigar_used,
                      char *vlist, int64_t vlist_cap, int64_t *vlist_off, int64_t *vlist_used,
                      char *seq, int64_t seq_cap, int64_t *seq_off, int64_t *seq_used);

/* ---- god-aligner: perfect-alignment BAM (god_aligner.py:19-183, cli.py:183-204) ------------------------------
 * write_perfect_reads per template (god_aligner.py:153-183) on the device, then samtools sort's coordinate order
 * (stable on (tid, pos+1, is_reverse)), BGZF and a BAI (pysam.sort / pysam.index, god_aligner.py:117-131).
 *   mh_bam_set_refs     @SQ names (NUL-separated, n_refs of them) and lengths, from <fasta>.ann (parse_ann :31-40);
 *                       clears the record store
 *   mh_bam_add_fastq    host FASTQ bytes, file 2 optional (NULL = single-end): every complete template in the
 *                       buffers (at most max_templates; -1 = all) becomes 1 or 2 records.  *used1 / *used2 = bytes
 *                       consumed (whole records), so the caller carries the rest into the next call.  Read names
 *                       longer than 254 characters, chroms missing from the header and unparseable qnames are
 *                       MH_E_ARG (the reference raises in pysam / parse_qname)
 *   mh_bam_add_output   the same from this context's FASTQ arenas (mh_emit_reads output, no host round trip)
 *   mh_bam_sort         the coordinate sort alone, in HBM (samtools sort's order, god_aligner.py:117-127); done once
 *                       per store (mh_bam_write reuses it), undone by the next mh_bam_add_*
 *   mh_bam_write        sort (unless sorted), write `bam_path` (BGZF, deflate `level` 0..9 on `threads` host threads) with the
 *                       header text, and the BAI at `bai_path` (NULL = none) */
int32_t mh_bam_set_refs(mh_ctx *ctx, int32_t n_refs, const char *names, const int64_t *lengths);
int32_t mh_bam_add_fastq(mh_ctx *ctx, const char *fq1, int64_t len1, const char *fq2, int64_t len2,
                         int64_t max_templates, int64_t *used1, int64_t *used2, int64_t *templates);
int32_t mh_bam_add_output(mh_ctx *ctx, int64_t max_templates, int64_t *templates);
int32_t mh_bam_records(mh_ctx *ctx, int64_t *n_records, int64_t *bytes);
int32_t mh_bam_sort(mh_ctx *ctx);
int32_t mh_bam_write(mh_ctx *ctx, const char *bam_path, const char *header_text, int64_t header_len, int32_t level,
                     int32_t threads, const char *bai_path, int64_t *out_records, int64_t *out_bytes);
int32_t mh_bam_reset(mh_ctx *ctx);
/* Bounded HBM for the record store (the reference's `samtools sort -m 2G` spills to temporary files,
 * god_aligner.py:100-116): once the records held in HBM would pass `bytes` (0 = no limit, the default; an allocation
 * that fails spills too), they move to host memory in input order.  Keys, offsets and BAI info of every record stay
 * in HBM, so the coordinate sort is still one device sort; mh_bam_write / _gpu assemble the sorted stream on the
 * host window by window (the GPU writer deflates each window on the device).  The file is byte-identical to the
 * unbounded store's.  mh_bam_spilled: bytes and host blocks spilled so far. */
int32_t mh_bam_set_capacity(mh_ctx *ctx, int64_t bytes);
/* Spilled records to unlinked temporary files in `dir` (mapped: the page cache holds them, and the kernel may write
 * them back under memory pressure — samtools sort's temporary files) instead of anonymous host memory; NULL or ""
 * = host memory (the default). */
int32_t mh_bam_set_spill_dir(mh_ctx *ctx, const char *dir);
int32_t mh_bam_spilled(mh_ctx *ctx, int64_t *bytes, int64_t *blocks);
/* Store pieces across ranks (configs[4] on N GPUs: each rank builds the BAM records of its FASTQ pieces, rank 0's
 * store takes them in piece order and sorts and writes once — the reference's pysam.cat of the workers' fragments
 * before one sort, god_aligner.py:63-68,100-108).  mh_bam_export copies records [r0, r1) of the store in input order:
 * their bytes, the r1 - r0 + 1 record offsets (absolute), the sort keys and the BAI info (4 x int32 per record); any
 * pointer may be host or device memory, or NULL to skip.  mh_bam_import appends n records given the same way
 * (offsets with any base); ties in the coordinate order keep the import order. */
int32_t mh_bam_export(mh_ctx *ctx, int64_t r0, int64_t r1, uint8_t *recs, int64_t *roff, uint64_t *keys,
                      int32_t *info);
int32_t mh_bam_import(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *keys, const int32_t *info,
                      int64_t n);
/* mh_bam_write_gpu: mh_bam_write with the record blocks deflated on the device (mh_deflate.hip: dynamic-Huffman BGZF
 *   blocks of the sorted store in HBM, 0xff00 input bytes each, the header's block deflated on the host at level 6):
 *   only the compressed bytes cross PCIe.  Replaces the same pysam.sort / pysam.index pair (god_aligner.py:117-131);
 *   the file decompresses to the same BAM stream, the BAI indexes its own virtual offsets.  *out_file_bytes = the
 *   BAM file's size. */
int32_t mh_bam_write_gpu(mh_ctx *ctx, const char *bam_path, const char *header_text, int64_t header_len,
                         const char *bai_path, int64_t *out_records, int64_t *out_bytes, int64_t *out_file_bytes);
/* ---- configs[4] across ranks: one coordinate range per rank (god_aligner.py:63-68,100-116: its workers' fragments,
 * `samtools sort -m 2G -@N`'s external merge and pysam.index, without a single merging process) ------------------
 *   mh_bam_partition       the store's records (one FASTQ piece's) by destination rank: dest = the number of the
 *                          n_dest - 1 ascending `splitters` <= the record's sort key.  Packed into a library buffer,
 *                          one segment per destination at seg_off[d] (n_dest + 1 entries), each laid out as records
 *                          (seg_bytes[d], 8-aligned), seg_n[d] + 1 record offsets from the segment's records, seg_n[d]
 *                          sort keys, seg_n[d] BAI infos (4 x int32), seg_n[d] ties (tie_base + the record's input
 *                          index: the global input order); input order inside each segment
 *   mh_bam_partition_fetch the packed segments to `out` (host or device memory, >= seg_off[n_dest] bytes)
 *   mh_bam_import_tie      mh_bam_import with each record's tie: equal sort keys are ordered by tie, so pieces may
 *                          arrive in any order (every import of the store gives ties, or none does)
 *   mh_bam_sorted_head     the first `len` bytes of the sorted record stream (host memory)
 *   mh_bam_write_part      the sorted stream from byte `skip`, then `tail` (host bytes: the head of the next ranks'
 *                          ranges), deflated on the device into 0xff00-byte BGZF blocks and written to `path`: the
 *                          header's block(s) first when header_len >= 0, the EOF marker when `eof`.  *out_blocks data
 *                          blocks starting at *out_data_pos in the file, *out_bytes = the file's size; boff (>= blocks
 *                          + 1 entries, or NULL) = each block's offset from *out_data_pos.  With skip = the bytes that
 *                          complete the previous rank's last block, the parts concatenated are the one-rank file.
 *   mh_bam_bai_runs        the BAI's raw plan of the sorted store (two calls: NULL arrays for the sizes): per run of
 *                          consecutive records in one bin, (tid << 32 | bin, first record's data offset, end offset,
 *                          records); per 16 kbp window of every reference (n_win in all) its first overlapping record's
 *                          data offset or -1; per reference its window count.  Ranks' plans join into one BAI. */
int32_t mh_bam_partition(mh_ctx *ctx, const uint64_t *splitters, int32_t n_dest, uint64_t tie_base, int64_t *seg_off,
                         int64_t *seg_n, int64_t *seg_bytes);
int32_t mh_bam_partition_fetch(mh_ctx *ctx, void *out, int64_t cap);
int32_t mh_bam_import_tie(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *keys,
                          const int32_t *info, const uint64_t *ties, int64_t n);
int32_t mh_bam_sorted_head(mh_ctx *ctx, int64_t len, uint8_t *out);
int32_t mh_bam_write_part(mh_ctx *ctx, const char *path, const char *header_text, int64_t header_len, int64_t skip,
                          const uint8_t *tail, int64_t tail_len, int32_t eof, int64_t *out_blocks, int64_t *out_data_pos,
                          int64_t *out_bytes, int64_t *boff, int64_t boff_cap);
int32_t mh_bam_bai_runs(mh_ctx *ctx, int64_t *n_runs, int64_t *runs, int64_t runs_cap, int64_t *n_win, int64_t *win,
                        int64_t win_cap, int64_t *ref_nwin);

/* ---- VCF ingest (vcfio.load_variant_file / split_copies / parse, vcfio.py:51-126) ------
 * Host-only (no device): mh_vcf_open parses a plain or bgzipped VCF for one sample; mh_vcf_region runs the BED
 * region query (htslib overlap: pos0 < end and pos0 + rlen > start0) and splits the records per copy, returning
 * ploidy and per-copy counts (n_var[c], alt_bytes[c] for c < cap); mh_vcf_copy copies one copy's SoA out
 * (the layout mh_build_haplotype takes).  Complex variants -> MH_E_COMPLEX_VARIANT, an unknown sample -> MH_E_ARG
 * (the reference raises ValueError for both); mh_vcf_error has the message. */
typedef struct mh_vcf mh_vcf;
int32_t mh_vcf_open(const char *path, const char *sample, mh_vcf **out);
const char *mh_vcf_error(const mh_vcf *v);
int32_t mh_vcf_close(mh_vcf *v);
int32_t mh_vcf_region(mh_vcf *v, const char *chrom, int64_t start0, int64_t end, int32_t *ploidy, int64_t *n_var,
                      int64_t *alt_bytes, int32_t cap);
int32_t mh_vcf_copy(mh_vcf *v, int32_t cpy, int64_t *pos, uint8_t *op, int64_t *oplen, int64_t *alt_off,
                    int64_t *alt_len, char *alt_pool);
/* filter-variants (vcfio.prepare_variant_file, vcfio.py:129-168; cli.py:20-35): for each of the n_regions BED
 * regions in order (chroms NUL-separated, start0/end per region), the region's records (the mh_vcf_region overlap
 * query; a record in two regions is written twice, as the reference writes it) except complex ones — rlen > 1 and
 * one of the sample's genotype alleles longer than 1 and different from REF (vcfio.py:139-146) — written to
 * out_path with the first 9 columns and the sample's column (BGZF-compressed on `threads` threads when bgzf != 0).
 * Header: the input's meta lines and the #CHROM line cut to the sample.  A missing allele on a multi-base record is
 * MH_E_ARG (the reference raises TypeError there).  err (err_cap bytes) receives the message on failure. */
int32_t mh_vcf_filter(const char *in_path, const char *sample, int32_t n_regions, const char *chroms,
                      const int64_t *start0, const int64_t *end, const char *out_path, int32_t bgzf, int32_t threads,
                      int64_t *n_written, int64_t *n_filtered, char *err, int32_t err_cap);

/* ---- FASTA reader (pysam.FastaFile for the generate-reads front end, readgenerate.py:181,186) -------------------
 * Host-only: plain or gzip/bgzip FASTA; contig name = the header's first word; bytes as stored.  names: contigs to
 * keep, NUL-separated and ended by an empty name (NULL = all).  mh_fasta_contig's pointers stay valid until
 * mh_fasta_close. */
typedef struct mh_fasta mh_fasta;
int32_t mh_fasta_open(const char *path, const char *names, mh_fasta **out);
const char *mh_fasta_error(const mh_fasta *f);
int32_t mh_fasta_count(const mh_fasta *f, int32_t *n);
int32_t mh_fasta_contig(const mh_fasta *f, int32_t i, const char **name, const char **seq, int64_t *len);
/* Contig i's sequence bytes (mh_fasta_contig's len of them) into dst, joined by threads from the mapped file (a
 * plain regular file) or copied (gzip input, FIFOs); without the library's own copy of the sequence. */
int32_t mh_fasta_copy(const mh_fasta *f, int32_t i, char *dst);
int32_t mh_fasta_close(mh_fasta *f);

/* ---- compressed FASTQ sink: host-side BGZF (gzip-compatible members of <= 65280 input
 * bytes, deflated on `threads` threads).  MH_E_CAPACITY if `cap` is short (*used = bytes needed).  mh_bgzf_eof
 * writes the 28-byte end-of-file marker block.  No context or device needed. */
int32_t mh_bgzf_compress(const char *in, int64_t len, int32_t level, int32_t threads, char *out, int64_t cap,
                         int64_t *used);
int32_t mh_bgzf_eof(char *out28);
/* The same BGZF framing deflated on the GPU (mh_deflate.hip: a workgroup per block, greedy LZ77 + dynamic Huffman
 * per eighth of a block).  Output decompresses to the input (the bytes differ from zlib's).  No EOF marker.
 *   mh_bgzf_compress_device  device buffer -> device buffer (cap bytes; MH_E_CAPACITY when short)
 *   mh_bgzf_compress_gpu     host buffer -> host buffer through the context's staging
 *   mh_output_bgzf           FASTQ arena `file` (0, 1) -> host buffer (out NULL: *used = the size only)
 *   mh_output_bgzf_range     bytes [offset, offset + len) of arena `file` -> host buffer: chunked D2H through small
 *                            page-locked buffers; offsets at multiples of 0xff00 give the members one call over the
 *                            whole arena gives */
int32_t mh_bgzf_compress_device(mh_ctx *ctx, const void *d_in, int64_t len, void *d_out, int64_t cap,
                                int64_t *used);
int32_t mh_bgzf_compress_gpu(mh_ctx *ctx, const char *in, int64_t len, char *out, int64_t cap, int64_t *used);
int32_t mh_output_bgzf(mh_ctx *ctx, int32_t file, char *out, int64_t cap, int64_t *used);
int32_t mh_output_bgzf_range(mh_ctx *ctx, int32_t file, int64_t offset, int64_t len, char *out, int64_t cap,
                             int64_t *used);
/* Both arenas' bytes [offset, offset + n_f) deflated (file 1, then file 2) with each file's compressed bytes copied
 * to out_f on a second stream behind its deflate: returns once the deflates are done (used_f = compressed bytes),
 * the copies still in flight; mh_output_bgzf_wait(ticket) waits for them (before out_f is read or reused).  Two
 * calls may be outstanding (the device buffer has two halves): the pipelined form of mh_output_bgzf_range for the
 * `.gz` sinks (readgenerate.py:233-253's writes), one range's copies overlapping the next range's deflate. */
int32_t mh_output_bgzf_pair(mh_ctx *ctx, int64_t offset, int64_t n1, int64_t n2, char *out1, int64_t cap1,
                            char *out2, int64_t cap2, int64_t *used1, int64_t *used2, int32_t *ticket);
int32_t mh_output_bgzf_wait(mh_ctx *ctx, int32_t ticket);

/* ---- corrupt-reads over existing FASTQ (readcorrupt.multi_process, readcorrupt.py:18-118; cli.py:144-157) -----
 * The complete templates of the host buffers (file 2 optional) are corrupted with the model set by
 * mh_set_corruption (must be enabled) and appended to the FASTQ arenas as '@{file-1 name}\n{seq}\n+\n{bq}\n' per
 * file (readcorrupt.py:112-114).  t_base = index of the buffers' first template in the whole input (the Philox
 * counter), *used1 / *used2 = bytes consumed, *templates = templates done. */
int32_t mh_corrupt_fastq(mh_ctx *ctx, const char *fq1, int64_t len1, const char *fq2, int64_t len2, int64_t t_base,
                         int64_t *used1, int64_t *used2, int64_t *templates);

/* ---- corruption -------------------------------------------------------------------------------------- */
/* Configure the empirical-BQ corruption (illumina.corrupt_template, illumina.py:113-162) that mh_emit_reads then
 * applies while it writes each record, and that mh_corrupt_fastq applies to existing FASTQ: per base
 * bq = min(searchsorted(cum_bq[file][n], U1), 93) over the f64 table, the base replaced by one of the other three
 * ('NNN' for non-ACGT) when U2 < phred_p[bq], quality chr(bq + 33) instead of '~'.  U1, U2 are 53-bit doubles
 * built as numpy's rand() builds them.  Their words come from Philox4x32-10 keyed by (seed, unit_key): ONE draw per
 * three bases, counter (template, file << 16 | base / 3).  Base base % 3 = k of the triple takes word k — its high
 * 16 bits are the top of U1, its low 16 bits the top of U2 — and the fourth word holds the three bases' replacement
 * choices (bits 10k .. 10k + 9: c % 3; c = 1023 is redrawn from the base's own draw (template, file << 16 | 0x8000 |
 * base)).  The low 37 bits of U1 and U2 come from the base's draw (template, file << 16 | 0x4000 | base), which the
 * device takes only when the 16-bit prefix ties a table threshold's prefix (the f64 comparison then decides).
 * tests/philox_ref.py restates this stream in numpy.  The output does not depend on GPU count or launch geometry.
 * cum_bq:
 * f64[2][max_bp][n_bq]; phred_p: f64[100] (pass the reference's own 10 ** (-arange(100) / 10)).  enable = 0 turns
 * it off. */
int32_t mh_set_corruption(mh_ctx *ctx, int32_t enable, const double *cum_bq, int32_t max_bp, int32_t n_bq,
                          const double *phred_p, uint64_t seed);
/* Word source of mh_corrupt_fastq (fused emission always uses Philox).  MH_RNG_PHILOX: as above (default).
 * MH_RNG_MITTY: the reference's exact single-worker stream (readcorrupt.py:84 with processes=1) — one MT19937 stream
 * consumed template by template, mate 0 then mate 1, per mate rand(n), rand(n), randint(0, 3, n)
 * (illumina.py:151-153); key624 = NULL starts RandomState(seed) at its first word, otherwise the stream continues
 * the explicit state (key624, pos) as numpy's RandomState.get_state() gives it.  Later mh_corrupt_fastq calls carry
 * on from where the previous one stopped. */
int32_t mh_set_corruption_stream(mh_ctx *ctx, int32_t rng_mode, uint64_t seed, const uint32_t *key624, int32_t pos);
/* The exact stream's current state (key624 / pos may be NULL) and, for a seeded stream, the words consumed so far
 * (-1 for an explicit-state stream): RandomState.set_state(('MT19937', key, pos, 0, 0.0)) continues it. */
int32_t mh_get_corruption_stream(mh_ctx *ctx, uint32_t *key624, int32_t *pos, int64_t *words);

/* ---- timing / profiling hooks ------------------------------------------------------------------------- */
/* Per-stage device time of the most recent mh_emit_reads / mh_sample_templates / mh_build_haplotype calls,
 * measured with HIP events on the context's stream (milliseconds); names are static strings. */
int32_t mh_stage_times(mh_ctx *ctx, const char **names, double *ms, int32_t cap, int32_t *n);
int32_t mh_enable_timing(mh_ctx *ctx, int32_t on);

/* ---- diagnostics --------------------------------------------------------------------------------------- */
/* Host computation of the MT19937 window (x_J .. x_{J+623}, untempered) of the stream seeded with `seed`, via the
 * jump polynomial x^J mod P — the same math the device segments use (tests compare it with the plain recurrence). */
int32_t mh_mt_window_at(uint32_t seed, uint64_t offset, uint32_t *out624);
/* Emission kernel choice: 0 = default (mh_emit_reads_async: the single-pass writer where it applies; otherwise and
 * for mh_emit_reads the measure pass + direct tile writer, falling back to the LDS-image writer for sample names or
 * records too long for its LDS layout), 1 = LDS-image writer always, 2 = never the single-pass writer (the measure
 * pass + direct tile writer: the two-pass path, for tests and A/B). */
int32_t mh_set_emit_mode(mh_ctx *ctx, int32_t mode);
/* Fisher-Yates swap-index decode and its exact fallbacks, a bit set (0 = the default):
 *   MH_DEC_SEQUENTIAL  the block-sequential decode always (by default it runs only when the chunk-parallel decode's
 *                      starts do not reach their fixed point);
 *   MH_DEC_FORCE_FIXUP every unit redone by the single-stream decode + per-unit permutation fix-up (by default only a
 *                      unit whose decode ran out of words);
 *   MH_DEC_FORCE_GEO   every unit redone with every geometric draw recomputed by the host libm (by default only the
 *                      draws whose quotient lies within 1e-12 of an integer, illumina.py:66-76).
 * The forcing bits exist so the tests can pin these rare paths against the oracle; they never change the output. */
#define MH_DEC_SEQUENTIAL 1
#define MH_DEC_FORCE_FIXUP 2
#define MH_DEC_FORCE_GEO 4
int32_t mh_set_decode_mode(mh_ctx *ctx, int32_t mode);
/* Units the context redid on the exact sequential fallback path (decode out of words / near-integer quotient). */
int32_t mh_fixup_count(mh_ctx *ctx, int64_t *n);

#ifdef __cplusplus
}
#endif
#endif
