// mh_fasta.cpp — host FASTA reader for the generate-reads front end (replaces pysam.FastaFile, reference
// readgenerate.py:181,186).  Plain C++ + zlib: plain or gzip/bgzip input, contig name = the header's first word,
// sequence bytes kept as stored (case and IUPAC codes pass through, as pysam's fetch returns them).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/mitty_hip.h"

struct mh_fasta {
  std::string err;
  std::vector<std::string> names, seqs;
  // the mapped-file path: the file stays mapped; per contig its pieces (cut at line ends) and each piece's first
  // output byte; the bytes are joined on request (mh_fasta_copy, or mh_fasta_contig into `bufs`)
  const char *map = nullptr;
  size_t map_len = 0;
  std::vector<std::vector<size_t>> cuts;
  std::vector<std::vector<int64_t>> outs;   // [pieces + 1]: the last = the contig's length
  std::vector<std::unique_ptr<char[]>> bufs;
};

namespace {

unsigned fasta_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// each line of [x, y): its bytes up to the line end, less a trailing run of '\r' (the Python parse's
// rstrip(b'\r\n')); into out when given; returns the bytes kept
int64_t fasta_lines(const char *b, size_t x, size_t y, char *out) {
  int64_t k = 0;
  while (x < y) {
    const char *nl = (const char *)memchr(b + x, '\n', y - x);
    size_t e = nl ? (size_t)(nl - b) : y;
    const size_t next = nl ? e + 1 : y;
    while (e > x && b[e - 1] == '\r') e--;
    if (out) memcpy(out + k, b + x, e - x);
    k += (int64_t)(e - x);
    x = next;
  }
  return k;
}

template <typename Fn>
void fasta_run(int T, Fn fn) {
  if (T == 1) {
    fn(0);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < T; t++) pool.emplace_back(fn, t);
  for (auto &th : pool) th.join();
}

// A regular, uncompressed file: mapped, headers found by memchr for '>' (FASTA sequence lines never hold one), each
// wanted contig cut into pieces at line ends and their kept bytes counted by threads (the copy comes later, by
// threads again, straight into the caller's buffer).  Returns false (nothing read) when the file is not such a
// file; the caller then streams it.
bool fasta_mapped(const char *path, const std::unordered_set<std::string> &want, mh_fasta *f) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 2) {
    close(fd);
    return false;
  }
  const size_t n = (size_t)st.st_size;
  void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return false;
  const char *b = (const char *)m;
  if ((uint8_t)b[0] == 0x1f && (uint8_t)b[1] == 0x8b) {   // gzip / BGZF: streamed through zlib
    munmap(m, n);
    return false;
  }
  f->map = b;
  f->map_len = n;
  struct Hdr {
    size_t a, e;   // the header line [a, e)
  };
  std::vector<Hdr> hs;
  for (const char *p = b; (p = (const char *)memchr(p, '>', n - (size_t)(p - b))) != nullptr; p++) {
    if (p != b && p[-1] != '\n') continue;
    const char *nl = (const char *)memchr(p, '\n', n - (size_t)(p - b));
    const size_t e = nl ? (size_t)(nl - b) : n;
    hs.push_back(Hdr{(size_t)(p - b), e});
    if (!nl) break;
    p = nl;   // (the loop's p++ moves past the line end)
  }
  const unsigned hw = fasta_threads();
  for (size_t h = 0; h < hs.size(); h++) {
    const std::string header(b + hs[h].a + 1, hs[h].e - hs[h].a - 1);
    size_t a = 0;
    while (a < header.size() && (header[a] == ' ' || header[a] == '\t')) a++;
    size_t z = a;
    while (z < header.size() && header[z] != ' ' && header[z] != '\t' && header[z] != '\r') z++;
    const std::string name = header.substr(a, z - a);
    if (!want.empty() && !want.count(name)) continue;
    const size_t s0 = std::min(n, hs[h].e + 1), s1 = std::max(s0, h + 1 < hs.size() ? hs[h + 1].a : n);
    const size_t len = s1 - s0;
    const int T = (int)std::min<size_t>(hw, std::max<size_t>(1, len >> 22));
    std::vector<size_t> cut(T + 1, s0);
    cut[T] = s1;
    for (int t = 1; t < T; t++) {   // just after a line end
      const size_t c = std::max(s0 + len * t / T, cut[t - 1]);
      const char *nl = c < s1 ? (const char *)memchr(b + c, '\n', s1 - c) : nullptr;
      cut[t] = nl ? (size_t)(nl - b) + 1 : s1;
    }
    std::vector<int64_t> cnt(T + 1, 0);
    fasta_run(T, [&](int t) { cnt[t + 1] = fasta_lines(b, cut[t], cut[t + 1], nullptr); });
    for (int t = 0; t < T; t++) cnt[t + 1] += cnt[t];
    f->names.push_back(name);
    f->cuts.push_back(std::move(cut));
    f->outs.push_back(std::move(cnt));
  }
  f->bufs.resize(f->names.size());
  return true;
}

void fasta_copy(const mh_fasta *f, int32_t i, char *dst) {
  const std::vector<size_t> &cut = f->cuts[i];
  const std::vector<int64_t> &o = f->outs[i];
  fasta_run((int)cut.size() - 1, [&](int t) { fasta_lines(f->map, cut[t], cut[t + 1], dst + o[t]); });
}

}  // namespace

extern "C" {

int32_t mh_fasta_open(const char *path, const char *names, mh_fasta **out) {
  if (!path || !out) return MH_E_ARG;
  mh_fasta *f = new mh_fasta();
  *out = f;
  std::unordered_set<std::string> want;
  for (const char *p = names; p && *p; p += strlen(p) + 1) want.insert(p);
  if (fasta_mapped(path, want, f)) return MH_OK;
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
  if (f->map) {
    const int64_t n = f->outs[i].back();
    if (seq) {   // joined on first request, kept until close
      auto &buf = const_cast<mh_fasta *>(f)->bufs[i];
      if (!buf) {
        buf.reset(new char[(size_t)n + 1]);
        fasta_copy(f, i, buf.get());
      }
      *seq = buf.get();
    }
    if (len) *len = n;
    return MH_OK;
  }
  if (seq) *seq = f->seqs[i].data();
  if (len) *len = (int64_t)f->seqs[i].size();
  return MH_OK;
}

int32_t mh_fasta_copy(const mh_fasta *f, int32_t i, char *dst) {
  if (!f || i < 0 || i >= (int32_t)f->names.size() || !dst) return MH_E_ARG;
  if (f->map) {
    fasta_copy(f, i, dst);
  } else if (!f->seqs[i].empty()) {
    memcpy(dst, f->seqs[i].data(), f->seqs[i].size());
  }
  return MH_OK;
}

int32_t mh_fasta_close(mh_fasta *f) {
  if (f && f->map) munmap((void *)f->map, f->map_len);
  delete f;
  return MH_OK;
}

}  // extern "C"
