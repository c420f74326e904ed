/* mitty_oracle.h — CPU restatement of the reference generate-reads path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle: a literal, scalar C restatement of alenzhao/Mitty's algorithm, used only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product (mitty_amd + libmitty_hip.so)
 * never links or calls it.  Parity is pinned against golden vectors captured from the reference itself
 * (tests/golden/make_golden.py).
 *
 * Reference citations (paths relative to the reference repo root):
 *   MT19937 + numpy legacy distributions: numpy RandomState (third-party), SURVEY.md Appendix A.1
 *   read_model_params      mitty/simulation/illumina.py:12-40
 *   get_data_for_workers   mitty/simulation/readgenerate.py:129-159
 *   create_node_list       mitty/simulation/rpc.py:38-116
 *   get_begin_end_nodes    mitty/simulation/rpc.py:119-130
 *   generate_read          mitty/simulation/rpc.py:133-160
 *   generate_reads (templates) mitty/simulation/illumina.py:43-110
 *   read_generating_worker mitty/simulation/readgenerate.py:167-218
 *   fastq_lines            mitty/simulation/readgenerate.py:222-230
 *   corrupt_single_read    mitty/simulation/illumina.py:140-162
 */
#ifndef MITTY_ORACLE_H
#define MITTY_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint32_t key[624]; int pos; } mo_mt;

void     mo_mt_seed(mo_mt *s, uint32_t seed);
uint32_t mo_mt_next(mo_mt *s);
double   mo_mt_double(mo_mt *s);
uint64_t mo_mt_interval(mo_mt *s, uint64_t max);
int64_t  mo_mt_geometric(mo_mt *s, double p);
/* fill helpers for vector tests */
void mo_mt_words(uint32_t seed, uint32_t *out, int64_t n);

void mo_read_model_params(int64_t mean_rlen, double coverage, double *p, int64_t *passes);

/* Work units: returns count; out arrays sized sum(ploidy)*passes. */
int64_t mo_work_units(uint32_t seed, const int32_t *ploidy, int64_t n_regions, int64_t passes,
                      int32_t *out_region, int32_t *out_cpy, uint32_t *out_seed);

/* Node list.  Variants: 1-based pos, op in {'X','I','D'}, oplen, alt bytes in alt_pool[alt_off .. +alt_len).
 * Output node arrays must have room for 2*n_var+1 entries.  seq of node k: src[k]==0 -> ref_seq, ==1 -> alt_pool,
 * at seq_off[k], length seq_len[k].  Returns node count. */
int64_t mo_create_node_list(const char *ref_seq, int64_t ref_len, int64_t ref_start_pos,
                            const int64_t *v_pos, const char *v_op, const int64_t *v_oplen,
                            const int64_t *v_alt_off, const int64_t *v_alt_len, int64_t n_var,
                            int64_t *ps, int64_t *pr, char *op, int64_t *oplen,
                            uint8_t *src, int64_t *seq_off, int64_t *seq_len);

/* Templates (illumina.generate_reads).  Returns m (kept) or -1 on a bad seed.  Arrays sized by
 * mo_template_capacity(). */
int64_t mo_template_capacity(int64_t p_min, int64_t p_max, double p);
int64_t mo_generate_templates(double p, int64_t rlen, const double *cum_tlen, int64_t n_tlen,
                              int64_t p_min, int64_t p_max, uint64_t seed,
                              int8_t *fo0, int64_t *pos0, int64_t *pos1);

/* One work unit end to end (node list -> templates -> reads -> FASTQ text).  The outputs are malloc'ed and
 * returned through out1/out2 (free with mo_free).  Returns kept template count, or -1 on a bad seed. */
int64_t mo_generate_unit(const char *ref_seq, int64_t ref_len, int64_t region_start0,
                         const int64_t *v_pos, const char *v_op, const int64_t *v_oplen,
                         const int64_t *v_alt_off, const int64_t *v_alt_len, const char *alt_pool, int64_t n_var,
                         double p, int64_t rlen, const double *cum_tlen, int64_t n_tlen, uint32_t rng_seed,
                         const char *serial_stub, const char *chrom, int64_t cpy,
                         char **out1, int64_t *len1, char **out2, int64_t *len2);

/* Exact-MT corruption of one read (corrupt_single_read).  cum_bq: the mate's (max_bp x n_bq) table, row-major.
 * phred_p: 100-entry table computed by the caller as numpy does.  out_seq/out_qual sized n. */
void mo_corrupt_read(mo_mt *s, const char *seq, int64_t n, const double *cum_bq, int64_t n_bq,
                     const double *phred_p, char *out_seq, char *out_qual);
/* Corrupt a whole FASTQ pair stream (readcorrupt.multi_process, processes=1).  Inputs are parallel arrays of
 * template sequences; output text malloc'ed. */
int64_t mo_corrupt_fastq(uint32_t seed, int64_t n_tpl, const char *const *names, const char *const *seq1,
                         const char *const *seq2, const int64_t *len1, const int64_t *len2,
                         const double *cum_bq, int64_t max_bp, int64_t n_bq, const double *phred_p,
                         char **out1, int64_t *olen1, char **out2, int64_t *olen2);

void mo_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
