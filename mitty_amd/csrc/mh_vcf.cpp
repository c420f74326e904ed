// mh_vcf.cpp — host VCF ingest for read generation (reference mitty/lib/vcfio.py:19-126 via pysam / htslib;
// SURVEY.md §8(f) rank 3).  Plain C++ + zlib (reads plain and bgzip/gzip VCF alike); no device involved.
//
// Semantics (the same as mitty_amd/lib/vcfio.py's restatement):
//  * the sample's column from #CHROM; GT from the FORMAT key 'GT' ('.' when absent);
//  * a BED region (chrom, start0, end) fetches the records of that contig with pos0 < end and pos0 + rlen > start0,
//    in file order, rlen = len(REF) unless INFO carries END= (htslib: rlen = END - POS + 1);
//  * ploidy = number of GT entries of the region's first record, 2 for an empty region (vcfio.py:74-79);
//  * per copy c: records with GT[c] != 0; alt = (REF, ALT...)[GT[c]]; X (ref 1, alt 1), I (ref 1, alt > 1,
//    oplen = len(alt) - 1), D (ref > 1, alt 1, oplen = len(ref) - 1), anything else is a complex variant
//    (vcfio.py:116-124).
//
// filter-variants (vcfio.prepare_variant_file, vcfio.py:129-168; cli.py:20-35): mh_vcf_filter writes, per BED region
// in BED order, the region's records (the same overlap query; a record in two regions is written twice, as the
// reference's loop writes it twice) except complex ones, keeping the first 9 columns and the sample's column.
// Complex (vcfio.py:139-146): rlen > 1 and one of the sample's genotype alleles is longer than 1 and differs from
// REF.  Header: the input's meta lines, the #CHROM line cut to the sample (htslib's header re-serialisation is not
// reproduced: no htslib here).
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mitty_hip.h"

struct mh_vcf {
  std::string err;
  // per contig, records in file order
  struct Rec {
    int64_t pos1, rlen;
    uint64_t ref_off, alt_off, gt_off;   // into `text`
    uint32_t ref_len, alt_len, gt_len;
    uint64_t head_off = 0, smp_off = 0;  // filter-variants: the record's first 9 columns and the sample's column
    uint32_t head_len = 0, smp_len = 0;
  };
  bool keep_lines = false;
  std::string meta;        // '##' lines (keep_lines)
  std::string chrom_head;  // the #CHROM line's first 9 columns (keep_lines)
  std::string sample;
  std::vector<std::string> order;   // contigs in file order
  std::unordered_set<std::string> header_contigs;   // ##contig=<ID=...> names
  std::unordered_map<std::string, std::vector<Rec>> by_chrom;
  std::string text;   // REF / ALT / GT fields of every record
  // last region query
  int32_t ploidy = 0;
  struct Copy {
    std::vector<int64_t> pos, oplen, alt_off, alt_len;
    std::vector<uint8_t> op;
    std::string pool;
  };
  std::vector<Copy> copies;
};

namespace {

int32_t fail(mh_vcf *v, int32_t code, const std::string &m) {
  v->err = m;
  return code;
}

// split on '\t' without copying: [begin, end) of each field
void tabs(const char *s, size_t n, std::vector<std::pair<size_t, size_t>> &f, size_t max_fields) {
  f.clear();
  size_t a = 0;
  for (size_t i = 0; i <= n && f.size() < max_fields; i++) {
    if (i == n || s[i] == '\t') {
      f.emplace_back(a, i);
      a = i + 1;
    }
  }
  if (f.size() == max_fields && f.back().second < n) f.back().second = n;   // last field keeps the rest
}

bool parse_i64(const char *s, size_t n, int64_t &v) {
  if (!n) return false;
  int64_t x = 0;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-') { neg = true; i = 1; }
  if (i == n) return false;
  for (; i < n; i++) {
    unsigned d = (unsigned)(s[i] - '0');
    if (d > 9 || x > (INT64_MAX - 9) / 10) return false;   // not a number, or beyond int64 (htslib rejects it too)
    x = x * 10 + d;
  }
  v = neg ? -x : x;
  return true;
}

// GT "a|b" / "a/b" / "." -> allele indices (-1 = missing)
void gt_alleles(const char *s, size_t n, std::vector<int> &g) {
  g.clear();
  size_t a = 0;
  for (size_t i = 0; i <= n; i++) {
    if (i == n || s[i] == '|' || s[i] == '/') {
      int64_t x;
      g.push_back(parse_i64(s + a, i - a, x) ? (int)x : -1);
      a = i + 1;
    }
  }
}

}  // namespace

static int32_t vcf_load(const char *path, const char *sample, mh_vcf *v) {
  gzFile fp = gzopen(path, "rb");
  if (!fp) return fail(v, MH_E_ARG, std::string("cannot open ") + path);
  gzbuffer(fp, 1 << 20);
  std::vector<char> buf(1 << 22);
  std::string carry;
  long col = -1;
  std::vector<std::pair<size_t, size_t>> f;
  const std::string smp(sample);
  int32_t rc = MH_OK;
  auto line_fn = [&](const char *s, size_t n) -> int32_t {
    if (n && s[n - 1] == '\r') n--;
    if (n >= 2 && s[0] == '#' && s[1] == '#') {
      if (v->keep_lines) v->meta.append(s, n).push_back('\n');
      static const char kc[] = "##contig=<ID=";
      if (n > sizeof(kc) - 1 && memcmp(s, kc, sizeof(kc) - 1) == 0) {
        size_t e = sizeof(kc) - 1;
        while (e < n && s[e] != ',' && s[e] != '>') e++;
        v->header_contigs.emplace(s + sizeof(kc) - 1, e - (sizeof(kc) - 1));
      }
      return MH_OK;
    }
    if (n >= 6 && memcmp(s, "#CHROM", 6) == 0) {
      tabs(s, n, f, SIZE_MAX);
      if (v->keep_lines && f.size() >= 9) v->chrom_head.assign(s, f[8].second);
      for (size_t i = 0; i < f.size(); i++)
        if (std::string(s + f[i].first, f[i].second - f[i].first) == smp) col = (long)i;
      if (col < 9) return fail(v, MH_E_ARG, "invalid sample name: " + smp);
      return MH_OK;
    }
    if (n == 0) return MH_OK;
    if (col < 0) return fail(v, MH_E_ARG, "VCF has no #CHROM header line");
    tabs(s, n, f, (size_t)col + 2);
    if ((long)f.size() <= col) return fail(v, MH_E_ARG, "VCF record with too few columns");
    mh_vcf::Rec r;
    if (!parse_i64(s + f[1].first, f[1].second - f[1].first, r.pos1)) return fail(v, MH_E_ARG, "bad POS");
    r.ref_len = (uint32_t)(f[3].second - f[3].first);
    r.alt_len = (uint32_t)(f[4].second - f[4].first);
    r.rlen = r.ref_len;
    // INFO END= (htslib sets rlen from it)
    {
      const char *info = s + f[7].first;
      const size_t il = f[7].second - f[7].first;
      size_t a = 0;
      for (size_t i = 0; i <= il; i++) {
        if (i == il || info[i] == ';') {
          if (i - a > 4 && memcmp(info + a, "END=", 4) == 0) {
            int64_t e;
            if (parse_i64(info + a + 4, i - a - 4, e) && e > r.pos1 - 1) r.rlen = e - (r.pos1 - 1);
          }
          a = i + 1;
        }
      }
    }
    // GT: index of 'GT' in FORMAT, that subfield of the sample column
    const char *fmt = s + f[8].first;
    const size_t fl = f[8].second - f[8].first;
    int gi = -1, k = 0;
    size_t a = 0;
    for (size_t i = 0; i <= fl; i++) {
      if (i == fl || fmt[i] == ':') {
        if (i - a == 2 && fmt[a] == 'G' && fmt[a + 1] == 'T') gi = k;
        k++;
        a = i + 1;
      }
    }
    const char *sc = s + f[col].first;
    const size_t sl = f[col].second - f[col].first;
    std::string gt = ".";
    if (gi >= 0) {
      int kk = 0;
      size_t b = 0;
      for (size_t i = 0; i <= sl; i++) {
        if (i == sl || sc[i] == ':') {
          if (kk == gi) {
            gt.assign(sc + b, i - b);
            break;
          }
          kk++;
          b = i + 1;
        }
      }
    }
    r.ref_off = v->text.size();
    v->text.append(s + f[3].first, r.ref_len);
    r.alt_off = v->text.size();
    v->text.append(s + f[4].first, r.alt_len);
    r.gt_off = v->text.size();
    r.gt_len = (uint32_t)gt.size();
    v->text += gt;
    if (v->keep_lines) {
      r.head_off = v->text.size();
      r.head_len = (uint32_t)f[8].second;
      v->text.append(s, f[8].second);
      r.smp_off = v->text.size();
      r.smp_len = (uint32_t)(f[col].second - f[col].first);
      v->text.append(s + f[col].first, r.smp_len);
    }
    std::string chrom(s + f[0].first, f[0].second - f[0].first);
    auto &lst = v->by_chrom[chrom];
    if (lst.empty()) v->order.push_back(chrom);
    lst.push_back(r);
    return MH_OK;
  };
  for (;;) {
    int got = gzread(fp, buf.data(), (unsigned)buf.size());
    if (got < 0) {
      rc = fail(v, MH_E_ARG, std::string("read error in ") + path);
      break;
    }
    if (got == 0) break;
    size_t a = 0;
    for (size_t i = 0; i < (size_t)got; i++) {
      if (buf[i] != '\n') continue;
      if (!carry.empty()) {
        carry.append(buf.data() + a, i - a);
        rc = line_fn(carry.data(), carry.size());
        carry.clear();
      } else {
        rc = line_fn(buf.data() + a, i - a);
      }
      a = i + 1;
      if (rc != MH_OK) break;
    }
    if (rc != MH_OK) break;
    carry.append(buf.data() + a, (size_t)got - a);
  }
  if (rc == MH_OK && !carry.empty()) rc = line_fn(carry.data(), carry.size());
  if (rc == MH_OK && col < 0) rc = fail(v, MH_E_ARG, "VCF has no #CHROM header line");
  gzclose(fp);
  return rc;
}

// the records of `chrom` overlapping [start0, end) (htslib: pos0 < end and pos0 + rlen > start0), in file order
static void region_records(const mh_vcf *v, const char *chrom, int64_t start0, int64_t end,
                           std::vector<const mh_vcf::Rec *> &recs) {
  recs.clear();
  auto it = v->by_chrom.find(chrom);
  if (it == v->by_chrom.end()) return;
  for (const auto &r : it->second)
    if (r.pos1 - 1 < end && r.pos1 - 1 + r.rlen > start0) recs.push_back(&r);
}

// ALT alleles of a record as [begin, end) offsets into its ALT field ('.' = none)
static void alt_spans(const char *alt, uint32_t n, std::vector<std::pair<size_t, size_t>> &alts) {
  alts.clear();
  if (n == 1 && alt[0] == '.') return;
  size_t a = 0;
  for (size_t i = 0; i <= n; i++)
    if (i == n || alt[i] == ',') {
      alts.emplace_back(a, i);
      a = i + 1;
    }
}

extern "C" {

int32_t mh_vcf_open(const char *path, const char *sample, mh_vcf **out) {
  if (!path || !sample || !out) return MH_E_ARG;
  *out = nullptr;
  mh_vcf *v = new mh_vcf();
  *out = v;
  return vcf_load(path, sample, v);
}

int32_t mh_vcf_filter(const char *in_path, const char *sample, int32_t n_regions, const char *chroms,
                      const int64_t *start0, const int64_t *end, const char *out_path, int32_t bgzf, int32_t threads,
                      int64_t *n_written, int64_t *n_filtered, char *err, int32_t err_cap) {
  auto set_err = [&](const std::string &m) {
    if (err && err_cap > 0) {
      const size_t k = std::min<size_t>(m.size(), (size_t)err_cap - 1);
      memcpy(err, m.data(), k);
      err[k] = 0;
    }
  };
  if (!in_path || !sample || !out_path || n_regions < 0 || (n_regions > 0 && (!chroms || !start0 || !end))) {
    set_err("bad arguments");
    return MH_E_ARG;
  }
  mh_vcf v;
  v.keep_lines = true;
  int32_t rc = vcf_load(in_path, sample, &v);
  if (rc != MH_OK) {
    set_err(v.err);
    return rc;
  }
  std::string out = v.meta + v.chrom_head + "\t" + sample + "\n";
  int64_t written = 0, filtered = 0;
  std::vector<const mh_vcf::Rec *> recs;
  std::vector<std::pair<size_t, size_t>> alts;
  std::vector<int> g;
  const char *cp = chroms;
  for (int32_t k = 0; k < n_regions; k++) {
    if (!v.by_chrom.count(cp) && !v.header_contigs.count(cp)) {   // pysam's fetch: ValueError('invalid contig')
      set_err("invalid contig `" + std::string(cp) + "`");
      return MH_E_ARG;
    }
    region_records(&v, cp, start0[k], end[k], recs);
    for (const mh_vcf::Rec *r : recs) {
      const char *ref = v.text.data() + r->ref_off;
      const char *alt = v.text.data() + r->alt_off;
      alt_spans(alt, r->alt_len, alts);
      gt_alleles(v.text.data() + r->gt_off, r->gt_len, g);
      bool complex = false;
      if (r->rlen > 1) {
        for (int a : g) {
          if (a < 0) {   // the reference takes len(None) here (TypeError)
            set_err("missing genotype allele on a multi-base record at " + std::string(cp) + ":" +
                    std::to_string(r->pos1));
            return MH_E_ARG;
          }
          if ((size_t)a > alts.size()) {
            set_err("GT allele index out of range at " + std::string(cp) + ":" + std::to_string(r->pos1));
            return MH_E_ARG;
          }
          const char *as = a == 0 ? ref : alt + alts[a - 1].first;
          const size_t al = a == 0 ? r->ref_len : alts[a - 1].second - alts[a - 1].first;
          if (al > 1 && !(al == r->ref_len && memcmp(as, ref, al) == 0)) complex = true;
        }
      }
      if (complex) {
        filtered++;
        continue;
      }
      out.append(v.text.data() + r->head_off, r->head_len).push_back('\t');
      out.append(v.text.data() + r->smp_off, r->smp_len).push_back('\n');
      written++;
    }
    cp += strlen(cp) + 1;
  }
  std::string data;
  if (bgzf) {
    int64_t need = 0;
    mh_bgzf_compress(out.data(), (int64_t)out.size(), 6, threads, nullptr, 0, &need);
    data.resize((size_t)need + 28);
    int64_t used = 0;
    rc = mh_bgzf_compress(out.data(), (int64_t)out.size(), 6, threads, &data[0], need, &used);
    if (rc != MH_OK) {
      set_err("BGZF compression failed");
      return rc;
    }
    mh_bgzf_eof(&data[(size_t)used]);
    data.resize((size_t)used + 28);
  }
  const std::string &bytes = bgzf ? data : out;
  FILE *fp = fopen(out_path, "wb");
  if (!fp) {
    set_err(std::string("cannot open ") + out_path);
    return MH_E_ARG;
  }
  const bool ok = fwrite(bytes.data(), 1, bytes.size(), fp) == bytes.size();
  if (fclose(fp) != 0 || !ok) {
    set_err(std::string("write failed: ") + out_path);
    return MH_E_ARG;
  }
  if (n_written) *n_written = written;
  if (n_filtered) *n_filtered = filtered;
  return MH_OK;
}

const char *mh_vcf_error(const mh_vcf *v) { return v ? v->err.c_str() : "null handle"; }

int32_t mh_vcf_close(mh_vcf *v) {
  delete v;
  return MH_OK;
}

int32_t mh_vcf_region(mh_vcf *v, const char *chrom, int64_t start0, int64_t end, int32_t *ploidy, int64_t *n_var,
                      int64_t *alt_bytes, int32_t cap) {
  if (!v || !chrom || !ploidy) return MH_E_ARG;
  v->copies.clear();
  v->ploidy = 0;
  // pysam's fetch (vcfio.py:62): a contig neither in the header nor among the records is ValueError('invalid contig')
  if (!v->by_chrom.count(chrom) && !v->header_contigs.count(chrom))
    return fail(v, MH_E_ARG, "invalid contig `" + std::string(chrom) + "`");
  std::vector<const mh_vcf::Rec *> recs;
  region_records(v, chrom, start0, end, recs);
  std::vector<int> g;
  int32_t pl = 2;
  if (!recs.empty()) {
    gt_alleles(v->text.data() + recs[0]->gt_off, recs[0]->gt_len, g);
    pl = (int32_t)g.size();
  }
  v->ploidy = pl;
  v->copies.resize(pl);
  std::vector<std::pair<size_t, size_t>> alts;
  for (const mh_vcf::Rec *r : recs) {
    gt_alleles(v->text.data() + r->gt_off, r->gt_len, g);
    if ((int32_t)g.size() < pl)
      return fail(v, MH_E_ARG, "record at " + std::string(chrom) + ":" + std::to_string(r->pos1) +
                                   " has fewer GT entries than the region ploidy");
    const char *ref = v->text.data() + r->ref_off;
    const char *alt = v->text.data() + r->alt_off;
    alt_spans(alt, r->alt_len, alts);
    for (int32_t c = 0; c < pl; c++) {
      if (g[c] == 0) continue;
      if (g[c] < 0)
        return fail(v, MH_E_ARG, "missing genotype at " + std::string(chrom) + ":" + std::to_string(r->pos1));
      if ((size_t)g[c] > alts.size())
        return fail(v, MH_E_ARG, "GT allele index out of range at " + std::string(chrom) + ":" +
                                     std::to_string(r->pos1));
      const char *as = alt + alts[g[c] - 1].first;
      const size_t al = alts[g[c] - 1].second - alts[g[c] - 1].first;
      uint8_t o;
      int64_t ol;
      if (r->ref_len == 1) {
        o = al == 1 ? 'X' : 'I';
        ol = al == 1 ? 0 : (int64_t)al - 1;
      } else if (al == 1) {
        o = 'D';
        ol = (int64_t)r->ref_len - 1;
      } else {
        return fail(v, MH_E_COMPLEX_VARIANT, "Complex variants present in VCF. Please filter or refactor these.");
      }
      mh_vcf::Copy &cp = v->copies[c];
      cp.pos.push_back(r->pos1);
      cp.op.push_back(o);
      cp.oplen.push_back(ol);
      cp.alt_off.push_back((int64_t)cp.pool.size());
      cp.alt_len.push_back((int64_t)al);
      cp.pool.append(as, al);
    }
    (void)ref;
  }
  *ploidy = pl;
  for (int32_t c = 0; c < pl && c < cap; c++) {
    if (n_var) n_var[c] = (int64_t)v->copies[c].pos.size();
    if (alt_bytes) alt_bytes[c] = (int64_t)v->copies[c].pool.size();
  }
  return MH_OK;
}

int32_t mh_vcf_copy(mh_vcf *v, int32_t cpy, int64_t *pos, uint8_t *op, int64_t *oplen, int64_t *alt_off,
                    int64_t *alt_len, char *alt_pool) {
  if (!v || cpy < 0 || cpy >= (int32_t)v->copies.size()) return MH_E_ARG;
  const mh_vcf::Copy &c = v->copies[cpy];
  const size_t n = c.pos.size();
  if (n) {
    if (!pos || !op || !oplen || !alt_off || !alt_len) return MH_E_ARG;
    memcpy(pos, c.pos.data(), 8 * n);
    memcpy(op, c.op.data(), n);
    memcpy(oplen, c.oplen.data(), 8 * n);
    memcpy(alt_off, c.alt_off.data(), 8 * n);
    memcpy(alt_len, c.alt_len.data(), 8 * n);
  }
  if (!c.pool.empty()) {
    if (!alt_pool) return MH_E_ARG;
    memcpy(alt_pool, c.pool.data(), c.pool.size());
  }
  return MH_OK;
}

}  // extern "C"
