/* mitty_oracle.c — CPU restatement of the reference generate-reads / corrupt-reads path.
 *
 * TEST INFRASTRUCTURE ONLY (see mitty_oracle.h).  Deliberately literal and scalar: every function follows the
 * reference line by line so that it can be checked by reading the two side by side; speed is not a goal.
 * Parity is pinned by tests/test_oracle_golden.py against vectors captured from the reference itself.
 */
#include "mitty_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------------------------
 * MT19937 (numpy RandomState legacy seeding: mt19937_seed == init_genrand) and the legacy distributions.
 * SURVEY.md Appendix A.1.
 * ---------------------------------------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397

void mo_mt_seed(mo_mt *s, uint32_t seed) {
  s->key[0] = seed;
  for (int i = 1; i < MT_N; i++)
    s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
  s->pos = MT_N;
}

static void mt_twist(mo_mt *s) {
  uint32_t *mt = s->key, y;
  int i;
  for (i = 0; i < MT_N - MT_M; i++) {
    y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
    mt[i] = mt[i + MT_M] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  for (; i < MT_N - 1; i++) {
    y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
    mt[i] = mt[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
  mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  s->pos = 0;
}

uint32_t mo_mt_next(mo_mt *s) {
  if (s->pos == MT_N) mt_twist(s);
  uint32_t y = s->key[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double mo_mt_double(mo_mt *s) {
  int32_t a = (int32_t)(mo_mt_next(s) >> 5), b = (int32_t)(mo_mt_next(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* numpy random_interval(max): smallest all-ones mask >= max, rejection. */
uint64_t mo_mt_interval(mo_mt *s, uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = max, value;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  if (max <= 0xffffffffull) {
    while ((value = (mo_mt_next(s) & mask)) > max) {}
  } else {
    while ((value = ((((uint64_t)mo_mt_next(s)) << 32 | mo_mt_next(s)) & mask)) > max) {}
  }
  return value;
}

/* numpy legacy_random_geometric: p >= 1/3 -> search, else inversion ceil(log1p(-U) / log(1 - p)).
 * (The log1p/log pairing was pinned against numpy with crafted MT states; see tests/golden/rng.json.) */
int64_t mo_mt_geometric(mo_mt *s, double p) {
  if (p >= 0.333333333333333333333333) {
    double U = mo_mt_double(s), sum = p, prod = p, q = 1.0 - p;
    int64_t X = 1;
    while (U > sum) { prod *= q; sum += prod; X++; }
    return X;
  }
  return (int64_t)ceil(log1p(-mo_mt_double(s)) / log(1.0 - p));
}

void mo_mt_words(uint32_t seed, uint32_t *out, int64_t n) {
  mo_mt s;
  mo_mt_seed(&s, seed);
  for (int64_t i = 0; i < n; i++) out[i] = mo_mt_next(&s);
}

/* ------------------------------------------------------------------------------------------------------------
 * illumina.read_model_params (mitty/simulation/illumina.py:12-40)
 * ---------------------------------------------------------------------------------------------------------- */
void mo_read_model_params(int64_t mean_rlen, double coverage, double *p_out, int64_t *passes_out) {
  double p = 1.0;
  int64_t passes = 1;
  while (p > 0.1) {
    passes *= 2;
    p = 0.5 * coverage / (double)(2 * mean_rlen * passes);
  }
  *p_out = p;
  *passes_out = passes;
}

/* ------------------------------------------------------------------------------------------------------------
 * readgenerate.get_data_for_workers (mitty/simulation/readgenerate.py:129-159)
 * ---------------------------------------------------------------------------------------------------------- */
int64_t mo_work_units(uint32_t seed, const int32_t *ploidy, int64_t n_regions, int64_t passes,
                      int32_t *out_region, int32_t *out_cpy, uint32_t *out_seed) {
  mo_mt s;
  mo_mt_seed(&s, seed);
  uint32_t shuffle_seed = (uint32_t)mo_mt_interval(&s, 0xfffffffeull);
  int64_t n = 0;
  for (int64_t r = 0; r < n_regions; r++)
    for (int32_t c = 0; c < ploidy[r]; c++)
      for (int64_t k = 0; k < passes; k++) {
        out_region[n] = (int32_t)r;
        out_cpy[n] = c;
        out_seed[n] = (uint32_t)mo_mt_interval(&s, 0xfffffffeull);
        n++;
      }
  mo_mt sh;
  mo_mt_seed(&sh, shuffle_seed);
  for (int64_t i = n - 1; i >= 1; i--) {
    int64_t j = (int64_t)mo_mt_interval(&sh, (uint64_t)i);
    int32_t tr = out_region[i]; out_region[i] = out_region[j]; out_region[j] = tr;
    int32_t tc = out_cpy[i]; out_cpy[i] = out_cpy[j]; out_cpy[j] = tc;
    uint32_t ts = out_seed[i]; out_seed[i] = out_seed[j]; out_seed[j] = ts;
  }
  return n;
}

/* ------------------------------------------------------------------------------------------------------------
 * rpc.create_node_list + snp/insertion/deletion (mitty/simulation/rpc.py:38-116)
 * ---------------------------------------------------------------------------------------------------------- */
static void py_slice(int64_t len, int64_t a, int64_t b, int64_t *off, int64_t *n) {
  if (a < 0) a += len; if (a < 0) a = 0; if (a > len) a = len;
  if (b < 0) b += len; if (b < 0) b = 0; if (b > len) b = len;
  *off = a;
  *n = b > a ? b - a : 0;
}

typedef struct {
  int64_t *ps, *pr, *oplen, *seq_off, *seq_len;
  char *op;
  uint8_t *src;
  int64_t n;
} nodes_t;

static void add_node(nodes_t *nd, int64_t ps, int64_t pr, char op, int64_t oplen, uint8_t src, int64_t off,
                     int64_t len) {
  int64_t k = nd->n++;
  nd->ps[k] = ps; nd->pr[k] = pr; nd->op[k] = op; nd->oplen[k] = oplen;
  nd->src[k] = src; nd->seq_off[k] = off; nd->seq_len[k] = len;
}

int64_t mo_create_node_list(const char *ref_seq, int64_t ref_len, int64_t ref_start_pos,
                            const int64_t *v_pos, const char *v_op, const int64_t *v_oplen,
                            const int64_t *v_alt_off, const int64_t *v_alt_len, int64_t n_var,
                            int64_t *ps, int64_t *pr, char *op, int64_t *oplen,
                            uint8_t *src, int64_t *seq_off, int64_t *seq_len) {
  (void)ref_seq;
  nodes_t nd = {ps, pr, oplen, seq_off, seq_len, op, src, 0};
  int64_t samp_pos = ref_start_pos, ref_pos = ref_start_pos, rs = ref_start_pos, off, n;
  for (int64_t i = 0; i < n_var; i++) {
    int64_t vp = v_pos[i];
    if (vp < ref_pos) continue;                                  /* rpc.py:55 */
    if (v_op[i] == 'X') {                                        /* rpc.py:75-87 */
      int64_t delta = vp - ref_pos;
      if (delta > 0) {
        py_slice(ref_len, ref_pos - rs, vp - rs, &off, &n);
        add_node(&nd, samp_pos, ref_pos, '=', delta, 0, off, n);
        ref_pos = vp;
        samp_pos += delta;
      }
      add_node(&nd, samp_pos, ref_pos, 'X', 1, 1, v_alt_off[i], v_alt_len[i]);
      ref_pos += 1;
      samp_pos += 1;
    } else if (v_op[i] == 'I') {                                 /* rpc.py:90-102 */
      int64_t delta = vp + 1 - ref_pos;
      if (delta > 0) {
        py_slice(ref_len, ref_pos - rs, vp + 1 - rs, &off, &n);
        add_node(&nd, samp_pos, ref_pos, '=', delta, 0, off, n);
        samp_pos += delta;
      }
      ref_pos = vp + 1;
      /* v.alt[1:] */
      int64_t al = v_alt_len[i] > 0 ? v_alt_len[i] - 1 : 0;
      add_node(&nd, samp_pos, ref_pos, 'I', v_oplen[i], 1, v_alt_off[i] + 1, al);
      samp_pos += v_oplen[i];
    } else {                                                     /* rpc.py:105-116 */
      int64_t delta = vp + 1 - ref_pos;
      if (delta > 0) {
        py_slice(ref_len, ref_pos - rs, vp + 1 - rs, &off, &n);
        add_node(&nd, samp_pos, ref_pos, '=', delta, 0, off, n);
        samp_pos += delta;
      }
      ref_pos = vp + 1 + v_oplen[i];
      add_node(&nd, samp_pos - 1, ref_pos, 'D', v_oplen[i], 0, 0, 0);
    }
  }
  int64_t offset = ref_pos - rs;                                 /* rpc.py:59-61 */
  if (offset <= ref_len) {
    py_slice(ref_len, offset, ref_len, &off, &n);
    add_node(&nd, samp_pos, ref_pos, '=', ref_len - offset, 0, off, n);
  }
  return nd.n;
}

/* ------------------------------------------------------------------------------------------------------------
 * illumina.generate_reads / _templates_for_region / _reads_for_template_in_region (illumina.py:43-110)
 * ---------------------------------------------------------------------------------------------------------- */
static int64_t est_block_size(int64_t p_min, int64_t p_max, double p) {
  return (int64_t)((double)(p_max - p_min) * p * 1.2);   /* int((p_max - p_min) * p * 1.2) */
}

int64_t mo_template_capacity(int64_t p_min, int64_t p_max, double p) {
  int64_t n = est_block_size(p_min, p_max, p);
  return n > 0 ? n : 0;
}

static int64_t searchsorted_left_f64(const double *a, int64_t n, double x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

int64_t mo_generate_templates(double p, int64_t rlen, const double *cum_tlen, int64_t n_tlen,
                              int64_t p_min, int64_t p_max, uint64_t seed,
                              int8_t *fo0, int64_t *pos0, int64_t *pos1) {
  if (seed > 0xffffffffull) return -1;                             /* illumina.py:53-54 */
  mo_mt sr, tloc, tlen, shuf, fo;
  mo_mt_seed(&sr, (uint32_t)seed);
  uint32_t s0 = (uint32_t)mo_mt_interval(&sr, 0xfffffffeull), s1 = (uint32_t)mo_mt_interval(&sr, 0xfffffffeull);
  uint32_t s2 = (uint32_t)mo_mt_interval(&sr, 0xfffffffeull), s3 = (uint32_t)mo_mt_interval(&sr, 0xfffffffeull);
  mo_mt_seed(&tloc, s0); mo_mt_seed(&tlen, s1); mo_mt_seed(&shuf, s2); mo_mt_seed(&fo, s3);

  int64_t n = mo_template_capacity(p_min, p_max, p);
  int64_t *ts = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
  int64_t acc = 0;
  for (int64_t k = 0; k < n; k++) {                                 /* geometric(p, n).cumsum() + p_min + 1 */
    acc += mo_mt_geometric(&tloc, p);
    ts[k] = acc + p_min + 1;
  }
  for (int64_t i = n - 1; i >= 1; i--) {                            /* shuffle_rng.shuffle(ts) */
    int64_t j = (int64_t)mo_mt_interval(&shuf, (uint64_t)i);
    int64_t t = ts[i]; ts[i] = ts[j]; ts[j] = t;
  }
  int64_t m = 0;
  for (int64_t k = 0; k < n; k++) {                                 /* tl = searchsorted(cum_tlen, rand(n)) */
    int64_t tl = searchsorted_left_f64(cum_tlen, n_tlen, mo_mt_double(&tlen));
    if (tl < rlen) tl = rlen;                                       /* tl.clip(rlen) */
    int64_t te = ts[k] + tl;
    if (te < p_max) {                                               /* idx = te < p_max */
      pos0[m] = ts[k];
      pos1[m] = te - rlen;                                          /* r1p = te - rlen */
      m++;
    }
  }
  uint32_t buf = 0;                                                 /* randint(2, size=m, dtype='i1') */
  int bcnt = 0;
  for (int64_t k = 0; k < m; k++) {
    if (bcnt == 0) { buf = mo_mt_next(&fo); bcnt = 3; } else { buf >>= 8; bcnt--; }
    fo0[k] = (int8_t)(buf & 1u);
  }
  free(ts);
  return m;
}

/* ------------------------------------------------------------------------------------------------------------
 * Growable byte buffer
 * ---------------------------------------------------------------------------------------------------------- */
typedef struct { char *p; int64_t n, cap; } sbuf;

static void sb_reserve(sbuf *b, int64_t extra) {
  if (b->n + extra + 1 > b->cap) {
    int64_t c = b->cap ? b->cap : 4096;
    while (c < b->n + extra + 1) c *= 2;
    b->p = (char *)realloc(b->p, (size_t)c);
    b->cap = c;
  }
}
static void sb_put(sbuf *b, const char *s, int64_t n) { sb_reserve(b, n); memcpy(b->p + b->n, s, (size_t)n); b->n += n; }
static void sb_str(sbuf *b, const char *s) { sb_put(b, s, (int64_t)strlen(s)); }
static void sb_int(sbuf *b, int64_t v) { char t[32]; int k = snprintf(t, sizeof t, "%lld", (long long)v); sb_put(b, t, k); }
static void sb_chr(sbuf *b, char c) { sb_put(b, &c, 1); }

/* ------------------------------------------------------------------------------------------------------------
 * rpc.get_begin_end_nodes (rpc.py:119-130) + rpc.generate_read (rpc.py:133-160)
 * ---------------------------------------------------------------------------------------------------------- */
static int64_t searchsorted_right_u64(const uint64_t *keys, int64_t n, int64_t x) {
  /* numpy compares uint64 keys with int64 values through float64; exact for |values| < 2^53. */
  double xd = (double)x;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if ((double)keys[mid] <= xd) lo = mid + 1; else hi = mid;
  }
  return lo;
}

typedef struct {
  int64_t pos;
  sbuf cigar, vlist, seq;
} read_t;

static void generate_read(const nodes_t *nd, const char *ref_seq, const char *alt_pool, int64_t p, int64_t l,
                          int64_t n0, int64_t n1, read_t *r) {
  r->cigar.n = r->vlist.n = r->seq.n = 0;
  int first_v = 1;
  for (int64_t k = n0; k <= n1; k++) {                             /* v_list */
    char op = nd->op[k];
    if (op == '=') continue;
    int64_t v = op == 'X' ? 0 : (op == 'I' ? nd->oplen[k] : -nd->oplen[k]);
    if (!first_v) sb_chr(&r->vlist, ',');
    sb_int(&r->vlist, v);
    first_v = 0;
  }
  for (int64_t k = n0; k <= n1; k++) {                             /* cigar + seq */
    int64_t ps = nd->ps[k], ol = nd->oplen[k];
    if (nd->op[k] != 'D') {
      int64_t hi = p + l - ps < ol ? p + l - ps : ol;
      int64_t lo = p - ps > 0 ? p - ps : 0;
      sb_int(&r->cigar, hi - lo);
    } else {
      sb_int(&r->cigar, ol);
    }
    sb_chr(&r->cigar, nd->op[k]);
    int64_t off, n;
    int64_t a = p - ps > 0 ? p - ps : 0, b = p + l - ps < ol ? p + l - ps : ol;
    py_slice(nd->seq_len[k], a, b, &off, &n);
    const char *base = (nd->src[k] ? alt_pool : ref_seq) + nd->seq_off[k];
    sb_put(&r->seq, base + off, n);
  }
  if (nd->op[n0] == 'I') {
    if (n0 == n1) {
      r->pos = nd->pr[n0] - 1;
      r->cigar.n = 0;
      sb_chr(&r->cigar, '>');
      sb_int(&r->cigar, p - nd->ps[n0]);
      sb_chr(&r->cigar, ':');
      sb_int(&r->cigar, l);
      sb_chr(&r->cigar, 'I');
    } else {
      r->pos = nd->pr[n0];
    }
  } else {
    r->pos = p - nd->ps[n0] + nd->pr[n0];
  }
}

/* ------------------------------------------------------------------------------------------------------------
 * readgenerate.read_generating_worker loop body (readgenerate.py:184-210) + fastq_lines (:222-230)
 * ---------------------------------------------------------------------------------------------------------- */
int64_t mo_generate_unit(const char *ref_seq, int64_t ref_len, int64_t region_start0,
                         const int64_t *v_pos, const char *v_op, const int64_t *v_oplen,
                         const int64_t *v_alt_off, const int64_t *v_alt_len, const char *alt_pool, int64_t n_var,
                         double p, int64_t rlen, const double *cum_tlen, int64_t n_tlen, uint32_t rng_seed,
                         const char *serial_stub, const char *chrom, int64_t cpy,
                         char **out1, int64_t *len1, char **out2, int64_t *len2) {
  int64_t cap = 2 * n_var + 1;
  nodes_t nd;
  nd.ps = (int64_t *)malloc(sizeof(int64_t) * cap); nd.pr = (int64_t *)malloc(sizeof(int64_t) * cap);
  nd.oplen = (int64_t *)malloc(sizeof(int64_t) * cap); nd.seq_off = (int64_t *)malloc(sizeof(int64_t) * cap);
  nd.seq_len = (int64_t *)malloc(sizeof(int64_t) * cap); nd.op = (char *)malloc((size_t)cap);
  nd.src = (uint8_t *)malloc((size_t)cap);
  nd.n = mo_create_node_list(ref_seq, ref_len, region_start0 + 1, v_pos, v_op, v_oplen, v_alt_off, v_alt_len, n_var,
                             nd.ps, nd.pr, nd.op, nd.oplen, nd.src, nd.seq_off, nd.seq_len);
  int64_t p_min = nd.ps[0], p_max = nd.ps[nd.n - 1] + nd.oplen[nd.n - 1];    /* readgenerate.py:192 */

  int64_t tcap = mo_template_capacity(p_min, p_max, p);
  int8_t *fo0 = (int8_t *)malloc((size_t)(tcap + 1));
  int64_t *pos[2];
  pos[0] = (int64_t *)malloc(sizeof(int64_t) * (size_t)(tcap + 1));
  pos[1] = (int64_t *)malloc(sizeof(int64_t) * (size_t)(tcap + 1));
  int64_t m = mo_generate_templates(p, rlen, cum_tlen, n_tlen, p_min, p_max, rng_seed, fo0, pos[0], pos[1]);

  uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nd.n);
  for (int64_t k = 0; k < nd.n; k++) keys[k] = (uint64_t)(nd.op[k] != 'D' ? nd.ps[k] : nd.ps[k] + 1);

  sbuf o1 = {0}, o2 = {0};
  read_t rd[2];
  memset(rd, 0, sizeof rd);
  int64_t cnt = 0;
  for (int64_t t = 0; t < m; t++) {
    int keep = 1;
    int fo[2] = {fo0[t], 1 - fo0[t]};
    int slot_of[2];
    for (int s = 0; s < 2; s++) {
      int64_t pp = pos[s][t];
      int64_t n0 = searchsorted_right_u64(keys, nd.n, pp) - 1;
      int64_t n1 = searchsorted_right_u64(keys, nd.n, pp + rlen - 1) - 1;
      read_t *r = &rd[fo[s]];
      generate_read(&nd, ref_seq, alt_pool, pp, rlen, n0, n1, r);
      int64_t nN = 0;
      for (int64_t i = 0; i < r->seq.n; i++) nN += r->seq.p[i] == 'N';
      if (nN > 2) { keep = 0; break; }                              /* readgenerate.py:204 */
      if (s == 1) {                                                 /* revcomp, readgenerate.py:56,205-206 */
        for (int64_t i = 0, j = r->seq.n - 1; i < j; i++, j--) { char c = r->seq.p[i]; r->seq.p[i] = r->seq.p[j]; r->seq.p[j] = c; }
        for (int64_t i = 0; i < r->seq.n; i++) {
          char c = r->seq.p[i];
          r->seq.p[i] = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
        }
      }
      slot_of[fo[s]] = s;
    }
    if (!keep) continue;
    cnt++;
    sbuf q = {0};
    sb_chr(&q, '@'); sb_str(&q, serial_stub); sb_chr(&q, ':'); sb_int(&q, cnt);
    sb_chr(&q, '|'); sb_str(&q, chrom); sb_chr(&q, '|'); sb_int(&q, cpy);
    for (int f = 0; f < 2; f++) {
      read_t *r = &rd[f];
      sb_chr(&q, '|'); sb_int(&q, slot_of[f]); sb_chr(&q, '|'); sb_int(&q, r->pos); sb_chr(&q, '|'); sb_int(&q, rlen);
      sb_chr(&q, '|'); sb_put(&q, r->cigar.p ? r->cigar.p : "", r->cigar.n);
      sb_chr(&q, '|'); sb_put(&q, r->vlist.p ? r->vlist.p : "", r->vlist.n);
    }
    for (int f = 0; f < 2; f++) {
      sbuf *o = f ? &o2 : &o1;
      sb_put(o, q.p, q.n); sb_chr(o, '\n');
      sb_put(o, rd[f].seq.p ? rd[f].seq.p : "", rd[f].seq.n);
      sb_str(o, "\n+\n");
      sb_reserve(o, rlen);
      memset(o->p + o->n, '~', (size_t)rlen); o->n += rlen;
      sb_chr(o, '\n');
    }
    free(q.p);
  }
  for (int f = 0; f < 2; f++) { free(rd[f].cigar.p); free(rd[f].vlist.p); free(rd[f].seq.p); }
  free(keys); free(fo0); free(pos[0]); free(pos[1]);
  free(nd.ps); free(nd.pr); free(nd.oplen); free(nd.seq_off); free(nd.seq_len); free(nd.op); free(nd.src);
  *out1 = o1.p; *len1 = o1.n; *out2 = o2.p; *len2 = o2.n;
  return m < 0 ? -1 : cnt;
}

/* ------------------------------------------------------------------------------------------------------------
 * illumina.corrupt_single_read (illumina.py:140-162) and readcorrupt.multi_process(processes=1)
 * ---------------------------------------------------------------------------------------------------------- */
void mo_corrupt_read(mo_mt *s, const char *seq, int64_t n, const double *cum_bq, int64_t n_bq,
                     const double *phred_p, char *out_seq, char *out_qual) {
  double *bq_rnd = (double *)malloc(sizeof(double) * (size_t)(n + 1));
  double *call_rnd = (double *)malloc(sizeof(double) * (size_t)(n + 1));
  int64_t *base_rnd = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
  for (int64_t i = 0; i < n; i++) bq_rnd[i] = mo_mt_double(s);
  for (int64_t i = 0; i < n; i++) call_rnd[i] = mo_mt_double(s);
  for (int64_t i = 0; i < n; i++) base_rnd[i] = (int64_t)mo_mt_interval(s, 2);
  for (int64_t i = 0; i < n; i++) {
    int64_t bq = searchsorted_left_f64(cum_bq + i * n_bq, n_bq, bq_rnd[i]);
    if (bq > 93) bq = 93;
    char b = seq[i];
    out_seq[i] = b;
    if (call_rnd[i] < phred_p[bq]) {
      const char *rot = b == 'A' ? "CTG" : b == 'C' ? "ATG" : b == 'T' ? "ACG" : b == 'G' ? "ACT" : "NNN";
      out_seq[i] = rot[base_rnd[i]];
    }
    out_qual[i] = (char)(bq + 33);
  }
  free(bq_rnd); free(call_rnd); free(base_rnd);
}

int64_t mo_corrupt_fastq(uint32_t seed, int64_t n_tpl, const char *const *names, const char *const *seq1,
                         const char *const *seq2, const int64_t *len1, const int64_t *len2,
                         const double *cum_bq, int64_t max_bp, int64_t n_bq, const double *phred_p,
                         char **out1, int64_t *olen1, char **out2, int64_t *olen2) {
  mo_mt sr, s;
  mo_mt_seed(&sr, seed);
  mo_mt_seed(&s, (uint32_t)mo_mt_interval(&sr, 0xfffffffeull));     /* worker 0's seed, readcorrupt.py:31-37 */
  sbuf o[2] = {{0}, {0}};
  char *cs = NULL, *cq = NULL;
  int64_t ccap = 0;
  for (int64_t t = 0; t < n_tpl; t++) {
    for (int mate = 0; mate < 2; mate++) {
      const char *sq = mate ? (seq2 ? seq2[t] : NULL) : seq1[t];
      if (!sq) continue;
      int64_t n = mate ? len2[t] : len1[t];
      if (n > max_bp) return -1;
      if (n + 1 > ccap) { ccap = n + 1; cs = (char *)realloc(cs, (size_t)ccap); cq = (char *)realloc(cq, (size_t)ccap); }
      mo_corrupt_read(&s, sq, n, cum_bq + (int64_t)mate * max_bp * n_bq, n_bq, phred_p, cs, cq);
      sbuf *b = &o[mate];
      sb_chr(b, '@'); sb_str(b, names[t]); sb_chr(b, '\n');
      sb_put(b, cs, n); sb_str(b, "\n+\n"); sb_put(b, cq, n); sb_chr(b, '\n');
    }
  }
  free(cs); free(cq);
  *out1 = o[0].p; *olen1 = o[0].n; *out2 = o[1].p; *olen2 = o[1].n;
  return n_tpl;
}

void mo_free(void *p) { free(p); }
