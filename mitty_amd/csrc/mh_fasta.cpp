// mh_fasta.cpp — host FASTA reader for the generate-reads front end (replaces pysam.FastaFile, reference
// readgenerate.py:181,186).  Plain C++ + zlib: plain or gzip/bgzip input, contig name = the header's first word,
// sequence bytes kept as stored (case and IUPAC codes pass through, as pysam's fetch returns them).
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/mitty_hip.h"

struct mh_fasta {
  std::string err;
  std::vector<std::string> names, seqs;
};

extern "C" {

int32_t mh_fasta_open(const char *path, const char *names, mh_fasta **out) {
  if (!path || !out) return MH_E_ARG;
  mh_fasta *f = new mh_fasta();
  *out = f;
  std::unordered_set<std::string> want;
  for (const char *p = names; p && *p; p += strlen(p) + 1) want.insert(p);
  gzFile fp = gzopen(path, "rb");
  if (!fp) {
    f->err = std::string("cannot open ") + path;
    return MH_E_ARG;
  }
  gzbuffer(fp, 1 << 20);
  std::vector<char> buf(1 << 22);
  std::string *cur = nullptr;   // the contig being read (nullptr: skipped or none yet)
  bool in_header = false, at_line_start = true;
  std::string header;
  for (;;) {
    const int got = gzread(fp, buf.data(), (unsigned)buf.size());
    if (got < 0) {
      f->err = std::string("read error in ") + path;
      gzclose(fp);
      return MH_E_ARG;
    }
    if (got == 0) break;
    const char *b = buf.data();
    int64_t i = 0;
    while (i < got) {
      if (at_line_start && b[i] == '>') {
        in_header = true;
        header.clear();
        i++;
        at_line_start = false;
        continue;
      }
      const char *nl = (const char *)memchr(b + i, '\n', (size_t)(got - i));
      const int64_t e = nl ? nl - b : got;
      if (in_header) {
        header.append(b + i, (size_t)(e - i));
        if (nl) {
          size_t a = 0;
          while (a < header.size() && (header[a] == ' ' || header[a] == '\t')) a++;
          size_t z = a;
          while (z < header.size() && header[z] != ' ' && header[z] != '\t' && header[z] != '\r') z++;
          const std::string name = header.substr(a, z - a);
          cur = nullptr;
          if (want.empty() || want.count(name)) {
            f->names.push_back(name);
            f->seqs.emplace_back();
            cur = &f->seqs.back();
          }
          in_header = false;
        }
      } else if (cur) {
        int64_t z = e;
        if (nl && z > i && b[z - 1] == '\r') z--;
        cur->append(b + i, (size_t)(z - i));
      }
      at_line_start = nl != nullptr;
      i = nl ? e + 1 : e;
    }
  }
  gzclose(fp);
  return MH_OK;
}

const char *mh_fasta_error(const mh_fasta *f) { return f ? f->err.c_str() : "null handle"; }

int32_t mh_fasta_count(const mh_fasta *f, int32_t *n) {
  if (!f || !n) return MH_E_ARG;
  *n = (int32_t)f->names.size();
  return MH_OK;
}

int32_t mh_fasta_contig(const mh_fasta *f, int32_t i, const char **name, const char **seq, int64_t *len) {
  if (!f || i < 0 || i >= (int32_t)f->names.size()) return MH_E_ARG;
  if (name) *name = f->names[i].c_str();
  if (seq) *seq = f->seqs[i].data();
  if (len) *len = (int64_t)f->seqs[i].size();
  return MH_OK;
}

int32_t mh_fasta_close(mh_fasta *f) {
  delete f;
  return MH_OK;
}

}  // extern "C"
