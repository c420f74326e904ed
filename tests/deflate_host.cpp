// Host check of the single-thread parts of the device BGZF compressor (mitty_amd/csrc/mh_deflate.h: Huffman code
// lengths, canonical codes, the dynamic block header, CRC-32 combination).  Test infrastructure: compresses a file
// into BGZF with a sequential restatement of mh_deflate.hip's parse (64-position steps, hash of earlier steps, run
// candidate, MIN_MATCH-byte matches, every match a step's positions start, eight slices per block with sync flushes) and the shared header code; tests/test_deflate_cpu.py then
// inflates the output with Python's zlib.  usage: deflate_host IN OUT
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../mitty_amd/csrc/mh_deflate.h"

using namespace mh::df;

namespace {

constexpr int WAVES = 8, SLICE = (BLOCK + WAVES - 1) / WAVES, HB = 11;

uint32_t load4(const uint8_t *b, int x) { return b[x] | b[x + 1] << 8 | b[x + 2] << 16 | (uint32_t)b[x + 3] << 24; }
uint32_t hash4(uint32_t w) { return (w * 2654435761u) >> (32 - HB); }

struct Tok {
  int lit;          // >= 0: a literal byte
  int len, dist;    // else a match
};

int g_steps = 0;   // parse steps (the device's cost unit), reported on stderr

// mh_deflate.hip's parse: one step covers SW = DF_NP x 64 positions; every position's candidate from the table as it
// was at the step's start (or the run at distance 1); a greedy walk takes the step's matches in order (literals
// between), each extended to its end
std::vector<Tok> parse(const uint8_t *s, int S) {
  const int SW = getenv("DF_SW") ? atoi(getenv("DF_SW")) : 256;   // positions per step (mh_deflate.hip DF_NP x 64)
  std::vector<uint32_t> ht(1 << HB, 0);
  std::vector<Tok> out;
  std::vector<int> cand(SW);
  for (int cur = 0; cur < S;) {
    g_steps++;
    const int W = S - cur < SW ? S - cur : SW;
    for (int l = 0; l < SW; l++) {
      const int p = cur + l;
      cand[l] = -1;
      if (l >= W || p + MIN_MATCH > S) continue;
      const uint32_t w = load4(s, p);
      auto match = [&](int c) { return std::memcmp(s + p, s + c, MIN_MATCH) == 0; };
      if (p >= 1 && match(p - 1)) {
        cand[l] = p - 1;
      } else {
        const int c = (int)ht[hash4(w)] - 1;
        if (c >= 0 && match(c)) cand[l] = c;
      }
    }
    int x = 0, next = cur + W;
    while (x < W) {
      int m = x;
      while (m < W && cand[m] < 0) m++;
      for (int l = x; l < m; l++) out.push_back({s[cur + l], 0, 0});
      if (m >= W) {
        next = cur + W;
        break;
      }
      const int q = cur + m, j = cand[m], cap = S - q < MAX_MATCH ? S - q : MAX_MATCH;
      int L = MIN_MATCH;
      while (L < cap && s[q + L] == s[j + L]) L++;
      out.push_back({-1, L, q - j});
      x = m + L;
      next = cur + x;
    }
    for (int k = cur; k < next; k++)
      if (k + HASH_BYTES <= S) {
        uint32_t &e = ht[hash4(load4(s, k))];
        if ((uint32_t)(k + 1) > e) e = (uint32_t)(k + 1);
      }
    cur = next;
  }
  return out;
}

void codes(const uint32_t *f, int n, int limit, uint8_t *len, uint16_t *code) {
  std::vector<uint32_t> keys, A(NLIT);
  for (int s = 0; s < n; s++) {
    len[s] = 0;
    if (f[s]) keys.push_back((f[s] << 9) | (uint32_t)s);
  }
  std::sort(keys.begin(), keys.end());
  int32_t count[32], next[16];
  huffman_from_sorted(keys.data(), (int)keys.size(), limit, len, A.data(), count);
  canonical_codes(len, n, code, count, next);
}

// one slice as a deflate block (final or followed by a sync flush); returns its bytes
std::string slice_bits(const uint8_t *s, int S, bool last) {
  const std::vector<Tok> t = parse(s, S);
  uint32_t lf[NLIT] = {0}, dfq[NDIST] = {0};
  for (const Tok &k : t) {
    if (k.lit >= 0) lf[k.lit]++;
    else {
      lf[257 + len_code(k.len)]++;
      dfq[dist_code(k.dist)]++;
    }
  }
  lf[256] = 1;
  uint8_t llen[NLIT], dlen[NDIST];
  uint16_t lcode[NLIT], dcode[NDIST];
  codes(lf, NLIT, 15, llen, lcode);
  codes(dfq, NDIST, 15, dlen, dcode);
  std::vector<uint8_t> buf(4 * S + 4096, 0);
  BitSink bs{buf.data(), 0, 0, 0};
  bs.put(last ? 1u : 0u, 1);
  bs.put(2u, 2);
  HeaderScratch H;
  write_dynamic_header(bs, llen, dlen, H);
  for (const Tok &k : t) {
    if (k.lit >= 0) {
      bs.put(lcode[k.lit], llen[k.lit]);
    } else {
      const int lc = len_code(k.len), dc = dist_code(k.dist);
      bs.put(lcode[257 + lc], llen[257 + lc]);
      bs.put((uint32_t)(k.len - len_base(lc)), len_extra(lc));
      bs.put(dcode[dc], dlen[dc]);
      bs.put((uint32_t)(k.dist - dist_base(dc)), dist_extra(dc));
    }
  }
  bs.put(lcode[256], llen[256]);
  if (!last) {
    bs.put(0, 3);
    if (bs.nacc) bs.put(0, 8 - bs.nacc);
    bs.put(0xffff0000u, 32);
  }
  if (bs.nacc) bs.put(0, 8 - bs.nacc);
  return std::string((const char *)buf.data(), (size_t)bs.pos);
}

uint32_t crc_bytes(const uint8_t *p, int64_t n) {
  uint32_t c = 0xffffffffu;
  for (int64_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ CRC_POLY : c >> 1;
  }
  return ~c;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 3) return 2;
  FILE *fi = fopen(argv[1], "rb");
  if (!fi) return 2;
  std::vector<uint8_t> in;
  uint8_t tmp[1 << 16];
  size_t r;
  while ((r = fread(tmp, 1, sizeof(tmp), fi)) > 0) in.insert(in.end(), tmp, tmp + r);
  fclose(fi);
  in.resize(in.size() + 8, 0);   // (load4 reads past the end)
  const int64_t n = (int64_t)in.size() - 8;
  std::string out;
  for (int64_t b = 0; b * BLOCK < n; b++) {
    const uint8_t *blk = in.data() + b * BLOCK;
    const int bn = (int)(n - b * BLOCK < BLOCK ? n - b * BLOCK : BLOCK);
    std::string z;
    for (int w = 0; w < WAVES; w++) {
      const int s0 = w * SLICE;
      if (s0 >= bn) break;
      const int S = bn - s0 < SLICE ? bn - s0 : SLICE;
      z += slice_bits(blk + s0, S, s0 + SLICE >= bn);
    }
    // CRC by segments (the device's method) must equal the direct CRC; so must the combination of two halves
    static const CrcPowers P = make_crc_powers();
    static uint32_t tab[256];
    if (!tab[1])
      for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ CRC_POLY : c >> 1;
        tab[i] = c;
      }
    const uint32_t c = crc32_segments(blk, bn, P, tab);
    const int half = bn / 2;
    if (c != crc_bytes(blk, bn) ||
        crc_combine(crc_bytes(blk, half), crc_bytes(blk + half, bn - half), (uint64_t)(bn - half)) != c) {
      fprintf(stderr, "crc combine mismatch in block %lld\n", (long long)b);
      return 1;
    }
    const int64_t bsize = HDR + (int64_t)z.size() + TRL;
    if (bsize > MAX_BSIZE) {
      fprintf(stderr, "block %lld: %lld bytes compressed (stored on the device)\n", (long long)b, (long long)bsize);
      return 3;
    }
    const uint8_t h[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                           (uint8_t)((bsize - 1) & 0xff), (uint8_t)((bsize - 1) >> 8)};
    out.append((const char *)h, 18);
    out += z;
    const uint8_t t[8] = {(uint8_t)c, (uint8_t)(c >> 8), (uint8_t)(c >> 16), (uint8_t)(c >> 24),
                          (uint8_t)bn, (uint8_t)(bn >> 8), (uint8_t)(bn >> 16), (uint8_t)(bn >> 24)};
    out.append((const char *)t, 8);
  }
  FILE *fo = fopen(argv[2], "wb");
  if (!fo) return 2;
  fwrite(out.data(), 1, out.size(), fo);
  fclose(fo);
  fprintf(stderr, "steps %d\n", g_steps);
  return 0;
}
