// mtjump.hpp -- MT19937 jump-ahead polynomials (host side).
//
// R's Mersenne-Twister word sequence obeys x_{t+624} = x_{t+397} ^ f(x_t, x_{t+1}); on the
// 19937 bits that matter its transition A has the primitive characteristic polynomial
// phi(z) (degree 19937), acting on windows w_t = (x_t..x_{t+623}) modulo the 31 unused low
// bits of x_t.  With z^J = q(z) phi(z) + p(z), every word of A^J w_t equals the same word of
// p(A) w_t except the low bits of the first word (error q_0 * garbage), hence, using the
// polynomial of J - 1 and reading one word further,
//     x_{t+J+k} = XOR_{i : p_i = 1} x_{t+i+k+1},   p = z^(J-1) mod phi,  k = 0..623,
// so a generator can start J words ahead of a known state with one GF(2) correlation of
// the next ~20.6k words (k_mt_gen_multi).  phi is recovered here with Berlekamp-Massey
// from bit 31 of x_t (bit 0 of x_0 is one of the 31 unused bits); J-step polynomials by
// square-and-multiply mod phi.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace hdpm {

constexpr int kMtDeg = 19937;
constexpr int kPolyWords = (kMtDeg + 63) / 64;   // 312 words hold degree < 19937

using Poly = std::vector<uint64_t>;                // bit i = coefficient of z^i

inline int poly_bit(const Poly& p, int64_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1u); }
inline void poly_flip(Poly& p, int64_t i) { p[i >> 6] ^= 1ull << (i & 63); }

// dst ^= src << sh (dst sized to hold the result)
inline void poly_xor_shifted(Poly& dst, const Poly& src, int64_t sh) {
  const int64_t ws = sh >> 6;
  const int bs = (int)(sh & 63);
  for (size_t q = 0; q < src.size(); ++q) {
    const uint64_t v = src[q];
    if (!v) continue;
    dst[q + ws] ^= v << bs;
    if (bs && q + ws + 1 < dst.size()) dst[q + ws + 1] ^= v >> (64 - bs);
  }
}

inline int poly_degree(const Poly& p) {
  for (int64_t q = (int64_t)p.size() - 1; q >= 0; --q)
    if (p[q]) return (int)(q * 64 + 63 - __builtin_clzll(p[q]));
  return -1;
}

// phi(z) of R's MT19937 word recurrence (monic, degree 19937), via Berlekamp-Massey on
// bit 31 of x_t.
inline Poly mt_charpoly() {
  const int n = 2 * kMtDeg + 64;
  std::vector<uint32_t> x(n + 624);
  uint32_t seed = 4357;                 // any state with a non-degenerate bit sequence
  for (int i = 0; i < 624; i++) {
    x[i] = seed & 0xffff0000u;
    seed = 69069u * seed + 1u;
    x[i] |= (seed & 0xffff0000u) >> 16;
    seed = 69069u * seed + 1u;
  }
  for (int t = 0; t + 624 < n + 624; ++t) {
    const uint32_t y = (x[t] & 0x80000000u) | (x[t + 1] & 0x7fffffffu);
    x[t + 624] = x[t + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  // s reversed into a bit array so discrepancies are word dot products
  const int nw = (n + 63) / 64 + 2;
  Poly sr(nw, 0);
  for (int t = 0; t < n; ++t)
    if (x[t] >> 31) poly_flip(sr, n - 1 - t);
  auto window = [&](int64_t off, int q) -> uint64_t {  // bits off + 64q .. +63 of sr
    const int64_t b = off + 64 * (int64_t)q, w = b >> 6;
    const int s = (int)(b & 63);
    uint64_t lo = w < nw ? sr[w] : 0, hi = w + 1 < nw ? sr[w + 1] : 0;
    return s ? (lo >> s) | (hi << (64 - s)) : lo;
  };
  const int cw = (n + 63) / 64 + 2;
  Poly C(cw, 0), B(cw, 0), T;
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  for (int N = 0; N < n; ++N) {
    // d = sum_{i=0..L} c_i s[N-i],  s[N-i] = sr[n-1-N+i]
    const int64_t off = n - 1 - N;
    uint64_t acc = 0;
    const int qmax = L / 64;
    for (int q = 0; q <= qmax; ++q) {
      uint64_t cq = C[q];
      if (q == qmax) cq &= (L % 64 == 63) ? ~0ull : ((1ull << (L % 64 + 1)) - 1);
      acc ^= cq & window(off, q);
    }
    const int d = __builtin_popcountll(acc) & 1;
    if (!d) {
      m++;
    } else if (2 * L <= N) {
      T = C;
      poly_xor_shifted(C, B, m);
      L = N + 1 - L;
      B = T;
      m = 1;
    } else {
      poly_xor_shifted(C, B, m);
      m++;
    }
  }
  // C(z) is the connection polynomial 1 + c_1 z + ... + c_L z^L; phi is its reciprocal
  Poly phi(kPolyWords + 1, 0);
  for (int i = 0; i <= L; ++i)
    if (poly_bit(C, i)) poly_flip(phi, L - i);
  if (L != kMtDeg) phi.clear();
  return phi;
}

// r (any degree < 2*19937) reduced mod phi, returned with kPolyWords words.
inline Poly poly_mod(Poly r, const Poly& phi) {
  for (int64_t i = (int64_t)r.size() * 64 - 1; i >= kMtDeg; --i)
    if (poly_bit(r, i)) poly_xor_shifted(r, phi, i - kMtDeg);
  r.resize(kPolyWords);
  return r;
}

inline Poly poly_mulmod(const Poly& a, const Poly& b, const Poly& phi) {
  Poly r(2 * kPolyWords + 2, 0);
  for (int64_t i = 0; i < (int64_t)a.size() * 64; ++i)
    if (poly_bit(a, i)) poly_xor_shifted(r, b, i);
  return poly_mod(r, phi);
}

inline Poly poly_sqrmod(const Poly& a, const Poly& phi) {
  Poly r(2 * kPolyWords + 2, 0);
  for (size_t q = 0; q < a.size(); ++q) {
    uint64_t v = a[q];
    for (int b = 0; v; ++b, v >>= 1)
      if (v & 1u) poly_flip(r, 2 * (64 * (int64_t)q + b));
  }
  return poly_mod(r, phi);
}

// z^J mod phi
inline Poly poly_xpow(uint64_t J, const Poly& phi) {
  Poly r(kPolyWords, 0);
  r[0] = 1;
  for (int b = 63; b >= 0; --b) {
    r = poly_sqrmod(r, phi);
    if ((J >> b) & 1u) {   // multiply by z
      Poly s(kPolyWords + 1, 0);
      poly_xor_shifted(s, r, 1);
      r = poly_mod(s, phi);
    }
  }
  return r;
}

// Host reference of the device jump: the window J words ahead of X (a block array),
// p = z^(J-1) mod phi.
inline void mt_jump_host(const uint32_t* X, const Poly& p, uint32_t* out) {
  std::vector<uint32_t> seq(33 * 624);
  std::memcpy(seq.data(), X, 624 * 4);
  seq[0] &= 0x80000000u;
  for (int t = 0; t + 624 < 33 * 624; ++t) {
    const uint32_t y = (seq[t] & 0x80000000u) | (seq[t + 1] & 0x7fffffffu);
    seq[t + 624] = seq[t + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  for (int k = 0; k < 624; ++k) {
    uint32_t acc = 0;
    for (int i = 0; i < kMtDeg; ++i)
      if (poly_bit(p, i)) acc ^= seq[i + k + 1];
    out[k] = acc;
  }
}

}  // namespace hdpm
