// mh_bgzf.cpp — BGZF framing + BAI (see mh_bgzf.h).
#include "mh_bgzf.h"

#include "../../include/mitty_hip.h"

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <thread>

namespace mh {

namespace {

void put32(std::string &s, uint32_t v) {
  char b[4] = {(char)v, (char)(v >> 8), (char)(v >> 16), (char)(v >> 24)};
  s.append(b, 4);
}
void put64(std::string &s, uint64_t v) {
  put32(s, (uint32_t)v);
  put32(s, (uint32_t)(v >> 32));
}

// One BGZF block (RFC 1952 member with the 'BC' extra field) for n <= BGZF_BLOCK input bytes.
bool bgzf_block(const uint8_t *in, int64_t n, int level, std::string &out) {
  const size_t cap = compressBound((uLong)n) + 64;
  std::string buf(18 + cap + 8, '\0');
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  zs.next_in = (Bytef *)in;
  zs.avail_in = (uInt)n;
  zs.next_out = (Bytef *)&buf[18];
  zs.avail_out = (uInt)cap;
  int rc = deflate(&zs, Z_FINISH);
  const size_t clen = zs.total_out;
  deflateEnd(&zs);
  if (rc != Z_STREAM_END) return false;
  const size_t bsize = 18 + clen + 8;
  if (bsize > 65536) return false;
  static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
  memcpy(&buf[0], hdr, 16);
  buf[16] = (char)((bsize - 1) & 0xff);
  buf[17] = (char)((bsize - 1) >> 8);
  const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), in, (uInt)n);
  std::string tail;
  put32(tail, crc);
  put32(tail, (uint32_t)n);
  memcpy(&buf[18 + clen], tail.data(), 8);
  buf.resize(bsize);
  out.swap(buf);
  return true;
}

}  // namespace

const uint8_t BGZF_EOF[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43, 2, 0,
                              0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

std::string bam_header_bytes(const std::string &text, const std::vector<std::string> &names,
                             const std::vector<int64_t> &lens) {
  std::string s("BAM\1", 4);
  put32(s, (uint32_t)text.size());
  s += text;
  put32(s, (uint32_t)names.size());
  for (size_t i = 0; i < names.size(); i++) {
    put32(s, (uint32_t)(names[i].size() + 1));
    s += names[i];
    s.push_back('\0');
    put32(s, (uint32_t)lens[i]);
  }
  return s;
}

// Deflate data in BGZF_BLOCK pieces on `threads` host threads, handing the blocks to `sink` in order.
template <typename Sink>
static bool compress_blocks(const uint8_t *data, int64_t n, int level, int threads, Sink sink) {
  const int64_t nblk = (n + BGZF_BLOCK - 1) / BGZF_BLOCK;
  if (threads < 1) threads = 1;
  const int64_t round = (int64_t)threads * 64;
  std::vector<std::string> out(std::min<int64_t>(round, std::max<int64_t>(nblk, 1)));
  for (int64_t b0 = 0; b0 < nblk; b0 += round) {
    const int64_t b1 = std::min(nblk, b0 + round);
    std::vector<std::thread> pool;
    std::vector<char> good(threads, 1);
    for (int w = 0; w < threads; w++) {
      pool.emplace_back([&, w]() {
        for (int64_t b = b0 + w; b < b1; b += threads) {
          const int64_t m = std::min<int64_t>(BGZF_BLOCK, n - b * BGZF_BLOCK);
          if (!bgzf_block(data + b * BGZF_BLOCK, m, level, out[b - b0])) good[w] = 0;
        }
      });
    }
    for (auto &t : pool) t.join();
    for (int w = 0; w < threads; w++)
      if (!good[w]) return false;
    for (int64_t b = b0; b < b1; b++)
      if (!sink(b, out[b - b0])) return false;
  }
  return true;
}

bool bgzf_write(const char *path, const std::string &header, const uint8_t *data, int64_t n, int level, int threads,
                std::vector<int64_t> &coff, std::string &err) {
  FILE *fp = fopen(path, "wb");
  if (!fp) {
    err = std::string("cannot open ") + path;
    return false;
  }
  int64_t pos = 0;
  bool ok = true;
  std::string blk;
  for (size_t h = 0; h < header.size() && ok; h += BGZF_BLOCK) {
    const int64_t m = std::min<int64_t>(BGZF_BLOCK, (int64_t)(header.size() - h));
    ok = bgzf_block((const uint8_t *)header.data() + h, m, level, blk) && fwrite(blk.data(), 1, blk.size(), fp) ==
         blk.size();
    pos += (int64_t)blk.size();
  }
  const int64_t nblk = (n + BGZF_BLOCK - 1) / BGZF_BLOCK;
  coff.assign(nblk + 1, 0);
  ok = ok && compress_blocks(data, n, level, threads, [&](int64_t b, const std::string &z) {
    coff[b] = pos;
    pos += (int64_t)z.size();
    return fwrite(z.data(), 1, z.size(), fp) == z.size();
  });
  coff[nblk] = pos;
  ok = ok && fwrite(BGZF_EOF, 1, 28, fp) == 28;
  ok = (fclose(fp) == 0) && ok;
  if (!ok) err = std::string("BGZF write failed: ") + path;
  return ok;
}

bool bgzf_write_blocks(const char *path, const std::string &header, int level, int64_t n_z,
                       const std::vector<int64_t> &boff,
                       const std::function<const uint8_t *(int64_t, int64_t)> &fetch, std::vector<int64_t> &coff,
                       std::string &err) {
  FILE *fp = fopen(path, "wb");
  if (!fp) {
    err = std::string("cannot open ") + path;
    return false;
  }
  int64_t pos = 0;
  bool ok = true;
  std::string blk;
  for (size_t h = 0; h < header.size() && ok; h += BGZF_BLOCK) {
    const int64_t m = std::min<int64_t>(BGZF_BLOCK, (int64_t)(header.size() - h));
    ok = bgzf_block((const uint8_t *)header.data() + h, m, level, blk) && fwrite(blk.data(), 1, blk.size(), fp) ==
         blk.size();
    pos += (int64_t)blk.size();
  }
  coff.resize(boff.size());
  for (size_t b = 0; b < boff.size(); b++) coff[b] = pos + boff[b];
  const int64_t piece = (int64_t)1 << 26;
  for (int64_t o = 0; o < n_z && ok; o += piece) {
    const int64_t m = std::min(piece, n_z - o);
    const uint8_t *buf = fetch(o, m);
    ok = buf && fwrite(buf, 1, (size_t)m, fp) == (size_t)m;
  }
  ok = ok && fwrite(BGZF_EOF, 1, 28, fp) == 28;
  ok = (fclose(fp) == 0) && ok;
  if (!ok && err.empty()) err = std::string("BGZF write failed: ") + path;
  return ok;
}

bool bgzf_write_stream(const char *path, const std::string &header, int level,
                       const std::function<bool(const uint8_t **, int64_t *)> &next, int64_t *data_pos,
                       int64_t *end_pos, std::string &err, bool eof) {
  FILE *fp = fopen(path, "wb");
  if (!fp) {
    err = std::string("cannot open ") + path;
    return false;
  }
  int64_t pos = 0;
  bool ok = true;
  std::string blk;
  for (size_t h = 0; h < header.size() && ok; h += BGZF_BLOCK) {
    const int64_t m = std::min<int64_t>(BGZF_BLOCK, (int64_t)(header.size() - h));
    ok = bgzf_block((const uint8_t *)header.data() + h, m, level, blk) && fwrite(blk.data(), 1, blk.size(), fp) ==
         blk.size();
    pos += (int64_t)blk.size();
  }
  *data_pos = pos;
  const uint8_t *buf = nullptr;
  int64_t len = 0;
  while (ok && next(&buf, &len)) {
    ok = fwrite(buf, 1, (size_t)len, fp) == (size_t)len;
    pos += len;
  }
  *end_pos = pos;
  ok = ok && (!eof || fwrite(BGZF_EOF, 1, 28, fp) == 28);
  ok = (fclose(fp) == 0) && ok;
  if (!ok && err.empty()) err = std::string("BGZF write failed: ") + path;
  return ok;
}

bool bai_plan(int32_t n_refs, int64_t n, const BaiRec *recs, int threads, BaiPlan &plan, std::string &err) {
  plan.refs.assign((size_t)std::max(n_refs, 0), BaiRef{});
  if (threads < 1) threads = 1;
  int64_t i = 0;
  for (int32_t tid = 0; tid < n_refs; tid++) {
    if (i < n && recs[i].tid < tid) {
      err = "BAI: records not coordinate-sorted";
      return false;
    }
    int64_t j = i;
    {   // the reference's records: a binary search (records are sorted by tid)
      int64_t lo = i, hi = n;
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (recs[mid].tid <= tid) lo = mid + 1; else hi = mid;
      }
      j = lo;
    }
    BaiRef &R = plan.refs[tid];
    R.n = j - i;
    R.vi = i;
    R.vj = j;
    if (j == i) continue;
    // pieces of the record range on threads: each its runs (record order) and its linear index (first record per
    // window); the pieces are then joined in order
    const int64_t nr = j - i;
    const int T = (int)std::min<int64_t>(threads, std::max<int64_t>(1, nr / 65536));
    std::vector<std::vector<BaiRun>> runs(T);
    std::vector<std::vector<int64_t>> lins(T);
    std::vector<char> bad(T, 0);
    auto work = [&](int t) {
      const int64_t a = i + nr * t / T, b = i + nr * (t + 1) / T;
      auto &rr = runs[t];
      auto &lin = lins[t];
      for (int64_t k = a; k < b; k++) {
        const BaiRec &r = recs[k];
        if (r.tid != tid || r.beg < 0) {   // (the binary search above assumed sorted records)
          bad[t] = 2;
          return;
        }
        if (r.bin >= 37450u) {
          bad[t] = 1;
          return;
        }
        if (!rr.empty() && rr.back().bin == r.bin && rr.back().ke == k)
          rr.back().ke = k + 1;
        else
          rr.push_back(BaiRun{r.bin, k, k + 1});
        const int64_t w0 = r.beg >> 14, w1 = (int64_t)(r.end - 1) >> 14;
        if ((int64_t)lin.size() <= w1) lin.resize(w1 + 1, -1);
        for (int64_t w = w0; w <= w1; w++)
          if (lin[w] < 0) lin[w] = k;
      }
    };
    if (T == 1) {
      work(0);
    } else {
      std::vector<std::thread> pool;
      for (int t = 0; t < T; t++) pool.emplace_back(work, t);
      for (auto &th : pool) th.join();
    }
    for (int t = 0; t < T; t++)
      if (bad[t]) {
        err = bad[t] == 1 ? "BAI: bin number out of range" : "BAI: records not coordinate-sorted";
        return false;
      }
    std::vector<BaiRun> all;
    for (int t = 0; t < T; t++)
      for (const BaiRun &r : runs[t]) {
        if (!all.empty() && all.back().bin == r.bin && all.back().ke == r.kb)
          all.back().ke = r.ke;   // a run cut by the pieces
        else
          all.push_back(r);
      }
    std::stable_sort(all.begin(), all.end(), [](const BaiRun &x, const BaiRun &y) { return x.bin < y.bin; });
    R.runs = std::move(all);
    size_t nw = 0;
    for (int t = 0; t < T; t++) nw = std::max(nw, lins[t].size());
    R.lin.assign(nw, -1);
    for (int t = 0; t < T; t++)   // the earliest piece that set a window holds its first record
      for (size_t w = 0; w < lins[t].size(); w++)
        if (R.lin[w] < 0 && lins[t][w] >= 0) R.lin[w] = lins[t][w];
    i = j;
  }
  if (i != n) {
    err = "BAI: record tid outside the header's references";
    return false;
  }
  return true;
}

bool bai_emit(const char *path, const BaiPlan &plan, const int64_t *soff, const std::vector<int64_t> &coff,
              std::string &err) {   // (soff: the offsets array the plan's positions index)
  std::string s("BAI\1", 4);
  put32(s, (uint32_t)plan.refs.size());
  for (const BaiRef &R : plan.refs) {
    if (R.n == 0) {   // no records on this reference
      put32(s, 0);
      put32(s, 0);
      continue;
    }
    uint32_t n_bins = 0;
    for (size_t r = 0; r < R.runs.size(); r++) n_bins += (r == 0 || R.runs[r].bin != R.runs[r - 1].bin) ? 1u : 0u;
    put32(s, n_bins + 1);
    for (size_t r = 0; r < R.runs.size();) {
      size_t e = r;
      while (e < R.runs.size() && R.runs[e].bin == R.runs[r].bin) e++;
      put32(s, R.runs[r].bin);
      put32(s, (uint32_t)(e - r));
      for (; r < e; r++) {
        put64(s, voffset(coff, soff[R.runs[r].kb]));
        put64(s, voffset(coff, soff[R.runs[r].ke]));
      }
    }
    // pseudo-bin 37450: (first record, end of last record), (mapped, unmapped)
    put32(s, 37450);
    put32(s, 2);
    put64(s, voffset(coff, soff[R.vi]));
    put64(s, voffset(coff, soff[R.vj]));
    put64(s, (uint64_t)R.n);
    put64(s, 0);
    // linear index: windows with no overlapping record take the next window's offset (the last one set so far
    // going backwards), i.e. the first record that can overlap anything at or after them
    std::vector<uint64_t> lin(R.lin.size());
    uint64_t next = voffset(coff, soff[R.vj]);
    for (int64_t w = (int64_t)lin.size() - 1; w >= 0; w--) {
      if (R.lin[w] >= 0) next = voffset(coff, soff[R.lin[w]]);
      lin[w] = next;
    }
    put32(s, (uint32_t)lin.size());
    for (uint64_t v : lin) put64(s, v);
  }
  put64(s, 0);   // n_no_coor
  FILE *fp = fopen(path, "wb");
  if (!fp) {
    err = std::string("cannot open ") + path;
    return false;
  }
  bool ok = fwrite(s.data(), 1, s.size(), fp) == s.size();
  ok = (fclose(fp) == 0) && ok;
  if (!ok) err = std::string("BAI write failed: ") + path;
  return ok;
}

bool bai_write(const char *path, int32_t n_refs, int64_t n, const BaiRec *recs, const int64_t *soff,
               const std::vector<int64_t> &coff, std::string &err) {
  BaiPlan plan;
  const int threads = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  return bai_plan(n_refs, n, recs, threads, plan, err) && bai_emit(path, plan, soff, coff, err);
}

}  // namespace mh

// ---- C ABI: BGZF for the compressed FASTQ sink ------------------------------------------
extern "C" int32_t mh_bgzf_compress(const char *in, int64_t len, int32_t level, int32_t threads, char *out,
                                    int64_t cap, int64_t *used) {
  if ((!in && len > 0) || len < 0 || !used || level < 0 || level > 9) return MH_E_ARG;
  int64_t w = 0;
  bool fits = true;
  bool ok = mh::compress_blocks((const uint8_t *)in, len, level, threads, [&](int64_t, const std::string &z) {
    if (fits && out && w + (int64_t)z.size() <= cap)
      memcpy(out + w, z.data(), z.size());
    else
      fits = false;
    w += (int64_t)z.size();
    return true;
  });
  *used = w;
  if (!ok) return MH_E_ARG;
  return fits ? MH_OK : MH_E_CAPACITY;
}

extern "C" int32_t mh_bgzf_eof(char *out28) {
  if (!out28) return MH_E_ARG;
  memcpy(out28, mh::BGZF_EOF, 28);
  return MH_OK;
}
