// mh_jump.cpp — MT19937 jump-ahead over GF(2) (host side).
//
// numpy's RandomState is MT19937: a linear recurrence on a 19937-bit state S_t, S_{t+1} = A S_t.  With P the
// characteristic polynomial of A (degree 19937), A^J = g(A) for g = x^J mod P, so
//     S_{t+J} = sum_k g_k S_{t+k}     (Cayley-Hamilton).
// On the device the 624-word window W_t = (x_t .. x_{t+623}) of the untempered sequence stands for S_t (only the top
// bit of x_t belongs to the state; its low 31 bits never influence later words), so a segment of a stream that
// starts at output word J is seeded with  W_J = XOR_{k : g_k = 1} W_k, computed from the first ~20.6k words of the
// stream (mh_sample.hip, k_mt_segments).  This file finds P once (Berlekamp-Massey on the top-bit sequence) and
// produces g for the requested offsets (carry-less multiplication + Barrett reduction), cached per process.
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

#if defined(__x86_64__)
#include <wmmintrin.h>
#endif

namespace mh {
namespace jump {

constexpr int DEG = 19937;
constexpr int NW = (DEG + 63) / 64;   // 312 words per reduced polynomial

using Poly = std::vector<uint64_t>;

// ---- raw (untempered) MT19937 sequence --------------------------------------------------------------------------
void raw_sequence(uint32_t seed, uint32_t *x, int64_t n) {
  x[0] = seed;
  for (int i = 1; i < 624 && i < n; i++) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
  for (int64_t t = 624; t < n; t++) {
    uint32_t y = (x[t - 624] & 0x80000000u) | (x[t - 623] & 0x7fffffffu);
    x[t] = x[t - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
}

// ---- carry-less multiplication ----------------------------------------------------------------------------------
static inline void clmul64_soft(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
  lo = hi = 0;
  for (int i = 0; i < 64; i++)
    if ((b >> i) & 1) {
      lo ^= a << i;
      if (i) hi ^= a >> (64 - i);
    }
}

#if defined(__x86_64__)
__attribute__((target("pclmul,sse2"))) static void mul_pclmul(const uint64_t *a, int na, const uint64_t *b, int nb,
                                                             uint64_t *r) {
  for (int i = 0; i < na; i++) {
    if (!a[i]) continue;
    __m128i av = _mm_set_epi64x(0, (long long)a[i]);
    for (int j = 0; j < nb; j++) {
      __m128i p = _mm_clmulepi64_si128(av, _mm_set_epi64x(0, (long long)b[j]), 0x00);
      r[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p);
      r[i + j + 1] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p, p));
    }
  }
}
#endif

// r = a * b (r has na + nb words, zeroed here)
static void mul(const uint64_t *a, int na, const uint64_t *b, int nb, uint64_t *r) {
  std::memset(r, 0, sizeof(uint64_t) * (size_t)(na + nb));
#if defined(__x86_64__)
  if (__builtin_cpu_supports("pclmul")) {
    mul_pclmul(a, na, b, nb, r);
    return;
  }
#endif
  for (int i = 0; i < na; i++) {
    if (!a[i]) continue;
    for (int j = 0; j < nb; j++) {
      uint64_t lo, hi;
      clmul64_soft(a[i], b[j], lo, hi);
      r[i + j] ^= lo;
      r[i + j + 1] ^= hi;
    }
  }
}

static inline int get_bit(const uint64_t *p, int64_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1); }
static inline void flip_bit(uint64_t *p, int64_t i) { p[i >> 6] ^= (uint64_t)1 << (i & 63); }

// bits [from, from + nbits) of p as a new word array
static void extract_bits(const uint64_t *p, int64_t pw, int64_t from, int64_t nbits, uint64_t *out) {
  int64_t nw = (nbits + 63) / 64;
  for (int64_t w = 0; w < nw; w++) {
    int64_t b = from + 64 * w;
    int64_t wi = b >> 6, sh = b & 63;
    uint64_t lo = wi < pw ? p[wi] : 0, hi = wi + 1 < pw ? p[wi + 1] : 0;
    out[w] = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
  int64_t rem = nbits & 63;
  if (rem) out[nw - 1] &= ((uint64_t)1 << rem) - 1;
}

struct Field {
  Poly P;     // characteristic polynomial, DEG + 1 bits (NW + 1 words)
  Poly mu;    // floor(x^(2 DEG) / P), DEG + 1 bits
};

// Berlekamp-Massey over GF(2) on s[0..n): connection polynomial C (C_0 = 1) of length L.
static Poly berlekamp_massey(const std::vector<uint8_t> &s, int &L_out) {
  const int64_t n = (int64_t)s.size();
  const int64_t W = (n + 64) / 64 + 2;
  Poly C(W, 0), B(W, 0), T(W, 0);
  C[0] = B[0] = 1;
  int L = 0;
  int64_t m = 1;
  // reversed sequence bits so that the discrepancy is a word-wise AND with C
  const int64_t RW = (n + 63) / 64 + 2;
  Poly rev(RW, 0);
  for (int64_t i = 0; i < n; i++)
    if (s[i]) flip_bit(rev.data(), n - 1 - i);
  std::vector<uint64_t> win(W);
  for (int64_t k = 0; k < n; k++) {
    // d = sum_{i=0..L} C_i s[k - i] = sum_i C_i rev[n-1-k+i]
    const int64_t nb = L + 1;
    extract_bits(rev.data(), RW, n - 1 - k, nb, win.data());
    uint64_t acc = 0;
    for (int64_t w = 0; w < (nb + 63) / 64; w++) acc ^= C[w] & win[w];
    int d = __builtin_popcountll(acc) & 1;
    if (!d) {
      m++;
      continue;
    }
    if (2 * L <= k) T = C;
    // C ^= B << m
    const int64_t ws = m >> 6, bs = m & 63;
    for (int64_t w = W - 1; w >= ws; w--) {
      uint64_t v = B[w - ws] << bs;
      if (bs && w - ws - 1 >= 0) v |= B[w - ws - 1] >> (64 - bs);
      C[w] ^= v;
    }
    if (2 * L <= k) {
      L = (int)(k + 1 - L);
      B = T;
      m = 1;
    } else {
      m++;
    }
  }
  L_out = L;
  return C;
}

static Field build_field() {
  // top bits of x_624 .. x_{624 + 2*DEG + 64}
  const int64_t n = 2 * DEG + 64;
  std::vector<uint32_t> x(624 + n);
  raw_sequence(5489u, x.data(), 624 + n);
  std::vector<uint8_t> s(n);
  for (int64_t t = 0; t < n; t++) s[t] = (uint8_t)(x[624 + t] >> 31);
  int L = 0;
  Poly C = berlekamp_massey(s, L);
  if (L != DEG) throw std::runtime_error("MT19937 characteristic polynomial: unexpected degree");
  Field f;
  f.P.assign(NW + 1, 0);
  for (int i = 0; i <= DEG; i++)
    if (get_bit(C.data(), DEG - i)) flip_bit(f.P.data(), i);   // P = reverse(C)
  // mu = floor(x^(2 DEG) / P) by long division
  const int64_t NN = (2 * DEG + 64) / 64 + 1;
  Poly num(NN, 0), q(NW + 2, 0);
  flip_bit(num.data(), 2 * DEG);
  for (int64_t i = 2 * DEG; i >= DEG; i--) {
    if (!get_bit(num.data(), i)) continue;
    flip_bit(q.data(), i - DEG);
    const int64_t sh = i - DEG, ws = sh >> 6, bs = sh & 63;
    for (int64_t w = 0; w < NW + 1; w++) {
      uint64_t v = f.P[w];
      if (!v) continue;
      num[w + ws] ^= v << bs;
      if (bs && w + ws + 1 < NN) num[w + ws + 1] ^= v >> (64 - bs);
    }
  }
  f.mu = q;
  return f;
}

static const Field &field() {
  static Field f = build_field();
  return f;
}

// r = c mod P for c of degree < 2 DEG (c has 2*NW+2 words); Barrett: q = ((c >> DEG) * mu) >> DEG, r = c ^ q P.
static Poly reduce(const uint64_t *c, int64_t cw) {
  const Field &F = field();
  Poly hi(NW + 1, 0);
  extract_bits(c, cw, DEG, DEG + 1, hi.data());
  Poly t(2 * NW + 4, 0);
  mul(hi.data(), NW + 1, F.mu.data(), NW + 2, t.data());
  Poly q(NW + 2, 0);
  extract_bits(t.data(), 2 * NW + 3, DEG, DEG + 2, q.data());
  Poly qp(2 * NW + 4, 0);
  mul(q.data(), NW + 1, F.P.data(), NW + 1, qp.data());
  Poly full(2 * NW + 4, 0);
  for (int64_t w = 0; w < 2 * NW + 4; w++) full[w] = (w < cw ? c[w] : 0) ^ qp[w];
  // Barrett with mu = floor(x^(2 DEG) / P) is exact for deg(c) < 2 DEG: nothing may remain at or above DEG
  for (int64_t w = DEG >> 6; w < 2 * NW + 4; w++) {
    uint64_t v = full[w];
    if (w == (DEG >> 6)) v >>= (DEG & 63);
    if (v) throw std::runtime_error("MT19937 jump: Barrett reduction left high bits");
  }
  Poly r(full.begin(), full.begin() + NW);
  r[NW - 1] &= ((uint64_t)1 << (DEG & 63)) - 1;
  return r;
}

static Poly mulmod(const Poly &a, const Poly &b) {
  Poly c(2 * NW + 2, 0);
  mul(a.data(), NW, b.data(), NW, c.data());
  return reduce(c.data(), 2 * NW + 2);
}

static Poly x_pow(uint64_t J) {
  Poly r(NW, 0), base(NW, 0);
  r[0] = 1;
  base[0] = 2;   // x
  while (J) {
    if (J & 1) r = mulmod(r, base);
    J >>= 1;
    if (J) base = mulmod(base, base);
  }
  return r;
}

struct Cache {
  std::mutex mu;
  std::map<uint64_t, Poly> step;                 // L -> x^L mod P
  std::map<uint64_t, std::vector<Poly>> chain;   // L -> [x^(kL) mod P for k = 0..]
};
static Cache &cache() {
  static Cache c;
  return c;
}

// x^(k*L) mod P as 624 little-endian uint32 words (19968 bits, top bits zero).
void jump_poly_words(uint64_t L, int64_t k, uint32_t *out624) {
  Cache &c = cache();
  std::lock_guard<std::mutex> g(c.mu);
  auto &ch = c.chain[L];
  if (ch.empty()) {
    Poly one(NW, 0);
    one[0] = 1;
    ch.push_back(one);
  }
  if (!c.step.count(L)) c.step[L] = x_pow(L);
  const Poly &st = c.step[L];
  while ((int64_t)ch.size() <= k) ch.push_back(mulmod(ch.back(), st));
  const Poly &p = ch[(size_t)k];
  for (int w = 0; w < NW; w++) {
    out624[2 * w] = (uint32_t)p[w];
    out624[2 * w + 1] = (uint32_t)(p[w] >> 32);
  }
}

// Host reference of the device jump: window of the stream seeded with `seed` at output offset J (J multiple of
// nothing in particular), i.e. x_J .. x_{J+623} up to the don't-care low bits of x_J.
void window_at(uint32_t seed, uint64_t J, uint32_t *out624) {
  Poly g = x_pow(J);
  std::vector<uint32_t> x(DEG + 624 + 64);
  raw_sequence(seed, x.data(), (int64_t)x.size());
  std::memset(out624, 0, 624 * sizeof(uint32_t));
  for (int64_t k = 0; k < DEG; k++)
    if (get_bit(g.data(), k))
      for (int w = 0; w < 624; w++) out624[w] ^= x[k + w];
}

}  // namespace jump
}  // namespace mh
