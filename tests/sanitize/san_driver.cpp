// Host-side sanitizer driver (TEST INFRASTRUCTURE): the host C++ that parses untrusted input (mh_vcf.cpp) and writes
// into caller buffers / files (mh_bgzf.cpp), built with -fsanitize=address,undefined by tests/test_host_cpu.py.
// Commands on stdin, one per line:
//   vcf <path> <sample> <chrom> <start0> <end>   open, query one region, copy every copy out; then filter-variants
//                                                 of that region into <path>.filt.vcf(.gz)
//   bgzf <nbytes> <level> <threads> <seed>       compress pseudo-random bytes (short and exact-capacity buffers too)
//   bam <path> <n_records> <seed>                BGZF BAM + BAI of synthetic sorted records
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/mitty_hip.h"
#include "../../mitty_amd/csrc/mh_bgzf.h"

static uint64_t rnd(uint64_t &s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return s >> 33;
}

static int run_vcf(const std::string &path, const std::string &sample, const std::string &chrom, int64_t s0,
                   int64_t e) {
  char err[256];
  int64_t w = 0, fl = 0;
  const std::string reg = chrom + std::string(1, '\0');
  for (int z = 0; z < 2; z++) {
    const int32_t frc = mh_vcf_filter(path.c_str(), sample.c_str(), 1, reg.c_str(), &s0, &e,
                       (path + (z ? ".filt.vcf.gz" : ".filt.vcf")).c_str(), z, 2, &w, &fl, err, (int32_t)sizeof err);
    std::printf("filter rc=%d written=%lld filtered=%lld\n", frc, (long long)w, (long long)fl);
  }
  mh_vcf *v = nullptr;
  int32_t rc = mh_vcf_open(path.c_str(), sample.c_str(), &v);
  if (rc != MH_OK) {
    std::printf("vcf open rc=%d %s\n", rc, mh_vcf_error(v));
    mh_vcf_close(v);
    return 0;
  }
  int32_t ploidy = 0;
  int64_t n_var[8] = {0}, alt_bytes[8] = {0};
  rc = mh_vcf_region(v, chrom.c_str(), s0, e, &ploidy, n_var, alt_bytes, 8);
  std::printf("vcf region rc=%d ploidy=%d\n", rc, ploidy);
  if (rc == MH_OK) {
    for (int c = 0; c < ploidy && c < 8; c++) {
      std::vector<int64_t> pos(n_var[c] + 1), oplen(n_var[c] + 1), aoff(n_var[c] + 1), alen(n_var[c] + 1);
      std::vector<uint8_t> op(n_var[c] + 1);
      std::vector<char> pool(alt_bytes[c] + 1);
      rc = mh_vcf_copy(v, c, pos.data(), op.data(), oplen.data(), aoff.data(), alen.data(), pool.data());
      std::printf("  copy %d: %lld variants rc=%d\n", c, (long long)n_var[c], rc);
    }
  }
  mh_vcf_close(v);
  return 0;
}

static int run_bgzf(int64_t n, int level, int threads, uint64_t seed) {
  std::vector<char> in(n + 1);
  for (int64_t i = 0; i < n; i++) in[i] = "ACGTN\n@+~"[rnd(seed) % 9];
  int64_t used = 0;
  int32_t rc = mh_bgzf_compress(in.data(), n, level, threads, nullptr, 0, &used);   // size query
  std::vector<char> out(used);
  int64_t used2 = 0;
  rc = mh_bgzf_compress(in.data(), n, level, threads, out.data(), (int64_t)out.size(), &used2);
  int64_t used3 = 0;
  std::vector<char> small(used > 1 ? used - 1 : 1);
  int32_t rc3 = mh_bgzf_compress(in.data(), n, level, threads, small.data(), (int64_t)small.size(), &used3);
  char eof[28];
  mh_bgzf_eof(eof);
  std::printf("bgzf n=%lld rc=%d used=%lld/%lld short rc=%d\n", (long long)n, rc, (long long)used2, (long long)used,
              rc3);
  return 0;
}

static int run_bam(const std::string &path, int64_t n, uint64_t seed) {
  std::vector<uint8_t> data;
  std::vector<int64_t> soff;
  std::vector<mh::BaiRec> recs;
  int32_t pos = 0;
  for (int64_t i = 0; i < n; i++) {
    soff.push_back((int64_t)data.size());
    const int len = 40 + (int)(rnd(seed) % 200);
    for (int k = 0; k < len; k++) data.push_back((uint8_t)rnd(seed));
    pos += (int32_t)(rnd(seed) % 500);
    recs.push_back(mh::BaiRec{(int32_t)(i * 3 / std::max<int64_t>(n, 1)), pos, pos + 150, (uint32_t)(4681 + (pos >> 14))});
  }
  soff.push_back((int64_t)data.size());
  std::vector<int64_t> coff;
  std::string err;
  const std::string hdr = mh::bam_header_bytes("@HD\tVN:1.0\n", {"1", "2", "3"}, {50000000, 20000, 8000});
  bool ok = mh::bgzf_write(path.c_str(), hdr, data.data(), (int64_t)data.size(), 6, 3, coff, err);
  ok = ok && mh::bai_write((path + ".bai").c_str(), 3, n, recs.data(), soff.data(), coff, err);
  std::printf("bam n=%lld ok=%d %s\n", (long long)n, ok ? 1 : 0, err.c_str());
  return 0;
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream is(line);
    std::string cmd;
    is >> cmd;
    if (cmd == "vcf") {
      std::string path, sample, chrom;
      int64_t s0 = 0, e = 0;
      is >> path >> sample >> chrom >> s0 >> e;
      run_vcf(path, sample, chrom, s0, e);
    } else if (cmd == "bgzf") {
      int64_t n = 0;
      int level = 6, threads = 1;
      uint64_t seed = 1;
      is >> n >> level >> threads >> seed;
      run_bgzf(n, level, threads, seed);
    } else if (cmd == "bam") {
      std::string path;
      int64_t n = 0;
      uint64_t seed = 1;
      is >> path >> n >> seed;
      run_bam(path, n, seed);
    }
  }
  return 0;
}
