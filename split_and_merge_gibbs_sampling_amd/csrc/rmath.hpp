// rmath.hpp -- host-side R/Rcpp/GSL-compatible numerics used by the hdpm runtime.
//
// The reference sampler draws every random number from R's global Mersenne-Twister
// through Rcpp sugar and R nmath, and evaluates the HIG normaliser with GSL.  The
// runtime keeps ONE R-compatible stream on the host (the device receives contiguous
// slices of it), so these restatements must consume draws exactly as R does:
//   Rng            R src/main/RNG.c  (set.seed scrambling, MT_genrand, fixup)
//   sample_prob1   Rcpp sugar sample(x, 1, TRUE, p): FixupProb + revsort + SampleReplace
//   rbeta          R nmath rbeta.c (Cheng 1978, BB / BC)
//   qbeta01_lt     hg:359 branch test R::qbeta(0.1, a, b) < x  (as pbeta(x) > 0.1)
//   hyperg_2F1     GSL gsl_sf_hyperg_2F1_e, positive-series branch
//   rhig1 / bisec  code/hyperg.cpp:221-287, 346-378
#pragma once
#include <cfloat>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <unordered_map>
#include <vector>

#include <math.h>  // lgamma_r

namespace hdpm {

enum Status : int {
  kOk = 0,
  kValidate = 1,   // validate_state -> Rcpp::stop (cf:146-172)
  kGsl = 2,        // norm_const2 throws (hg:38-45)
  kProb = 3,       // FixupProb stop()
  kWalker = 4,     // (no longer returned: Walker alias sampling is restated)
  kArg = 5,        // bad argument / capacity
  kDevice = 6,     // HIP runtime failure
  kNoDevice = 7,   // no HIP device / extension unusable
};

// ------------------------------------------------------------------ R MT19937
// Inverse of MT19937's tempering: the mt word behind a raw output.
inline uint32_t mt_untemper(uint32_t y) {
  y ^= y >> 18;                                  // self-inverse
  y ^= (y << 15) & 0xefc60000u;                  // self-inverse (the shifted bits leave the word)
  uint32_t r = y;
  for (int i = 0; i < 5; ++i) r = y ^ ((r << 7) & 0x9d2c5680u);
  y = r;
  for (int i = 0; i < 3; ++i) r = y ^ (r >> 11);
  return r;
}

struct Rng {
  int32_t mti = 625;
  uint32_t mt[624];
  uint64_t pos = 0;     // outputs drawn since the last (re)seed
  uint64_t epoch = 0;   // bumped whenever the state is replaced from outside

  void set_seed(uint32_t seed) {  // RNG_Init(MERSENNE_TWISTER, seed) + FixupSeeds
    for (int j = 0; j < 50; j++) seed = 69069u * seed + 1u;
    seed = 69069u * seed + 1u;  // i_seed[0] (dummy[0]) is overwritten by FixupSeeds
    for (int j = 0; j < 624; j++) { seed = 69069u * seed + 1u; mt[j] = seed; }
    mti = 624;
    pos = 0;
    epoch++;
  }
  void import625(const int32_t* s) {
    mti = s[0];
    for (int i = 0; i < 624; i++) mt[i] = (uint32_t)s[i + 1];
    pos = 0;
    epoch++;
  }
  void export625(int32_t* s) const {
    s[0] = mti;
    for (int i = 0; i < 624; i++) s[i + 1] = (int32_t)mt[i];
  }
  void twist() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int kk;
    uint32_t y;
    for (kk = 0; kk < 624 - 397; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < 623; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk - 227] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
    mti = 0;
  }
  // Raw tempered 32-bit output (MT_genrand before the 2^-32 scaling).
  uint32_t raw() {
    if (mti >= 624) {
      if (mti == 625) {  // MT_sgenrand(4357): never seeded
        uint32_t seed = 4357;
        for (int i = 0; i < 624; i++) {
          mt[i] = seed & 0xffff0000u;
          seed = 69069u * seed + 1u;
          mt[i] |= (seed & 0xffff0000u) >> 16;
          seed = 69069u * seed + 1u;
        }
      }
      twist();
    }
    pos++;
    uint32_t y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // Fill n raw outputs (same stream as n calls of raw()).
  void raw_block(uint32_t* out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = raw();
  }
  double unif() { return raw_to_unif(raw()); }
  static inline double raw_to_unif(uint32_t y) {
    const double i2_32m1 = 2.328306437080797e-10;
    double x = (double)y * 2.3283064365386963e-10;
    if (x <= 0.0) return 0.5 * i2_32m1;
    if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
    return x;
  }
};

// ------------------------------------------------------------------ Rcpp sample
// R sort.c revsort: descending heapsort of a[0..n) carrying ib[].
inline void revsort(double* a0, int* ib0, int n) {
  if (n <= 1) return;
  double* a = a0 - 1;
  int* ib = ib0 - 1;
  int l = (n >> 1) + 1, ir = n, i, j, ii;
  double ra;
  for (;;) {
    if (l > 1) {
      l = l - 1;
      ra = a[l];
      ii = ib[l];
    } else {
      ra = a[ir];
      ii = ib[ir];
      a[ir] = a[1];
      ib[ir] = ib[1];
      if (--ir == 1) {
        a[1] = ra;
        ib[1] = ii;
        return;
      }
    }
    i = l;
    j = l << 1;
    while (j <= ir) {
      if (j < ir && a[j] > a[j + 1]) ++j;
      if (ra > a[j]) {
        a[i] = a[j];
        ib[i] = ib[j];
        j += (i = j);
      } else {
        j = ir + 1;
      }
    }
    a[i] = ra;
    ib[i] = ii;
  }
}

// sample(x, 1, TRUE, probs) split into its parameter-only part -- FixupProb, the Walker
// check, revsort and the cumulative sums, into p (n doubles) and perm (n ints) -- and the
// pick for the uniform rU.  prep returns 0 or a negative Status.
// Walker's alias table (Rcpp sugar WalkerSample, R random.c walker_ProbSampleReplace) over
// the FixupProb-normalised p: q[i] = p[i] n, entries with q < 1 listed from the front of HL
// and the others from the back, each small entry aliased to the current large one; then
// q[i] += i.  On return p holds q and a the aliases (entries the loop never assigns keep
// q >= 1 in exact arithmetic; R leaves their alias uninitialised, here they alias themselves).
inline void walker_table(double* p, int* a, int n) {
  std::vector<int> HL((size_t)n);
  int h = -1, l = n;
  for (int i = 0; i < n; i++) {
    p[i] = p[i] * n;
    a[i] = i;
    if (p[i] < 1.) HL[++h] = i; else HL[--l] = i;
  }
  if (h >= 0 && l < n) {
    for (int k = 0; k < n - 1; k++) {
      const int i = HL[k], j = HL[l];
      a[i] = j;
      p[j] += p[i] - 1;
      if (p[j] < 1.) l++;
      if (l >= n) break;
    }
  }
  for (int i = 0; i < n; i++) p[i] += i;
}

// FixupProb, then either the cumulative sums in revsort order (returns 0; p = cumulative
// probabilities, perm = 1-based indices) or, with more than 200 entries of n p > 0.1,
// Walker's alias table (returns 1; p = q + i, perm = aliases).  Negative: a Status.
inline int sample_prob1_prep(const double* probs, int n, double* p, int* perm) {
  double sum = 0.0;
  int npos = 0;
  for (int i = 0; i < n; i++) {
    double x = probs[i];
    if (!std::isfinite(x) || x < 0) return -kProb;
    if (x > 0) { npos++; sum += x; }
  }
  if (npos == 0) return -kProb;
  for (int i = 0; i < n; i++) p[i] = probs[i] / sum;
  int nc = 0;
  for (int i = 0; i < n; i++) nc += (n * p[i] > 0.1);
  if (nc > 200) {
    walker_table(p, perm, n);
    return 1;
  }
  for (int i = 0; i < n; i++) perm[i] = i + 1;
  revsort(p, perm, n);
  for (int i = 1; i < n; i++) p[i] += p[i - 1];
  return 0;
}

// The draw with its uniform rU; mode = sample_prob1_prep's return (0 or 1).
inline int sample_prob1_pick(const double* cum, const int* perm, int n, double rU, int mode = 0) {
  if (mode == 1) {                       // Walker: rU n, k = (int) rU n, k or its alias
    const double r = rU * n;
    const int k = (int)r;
    return r < cum[k] ? k : perm[k];
  }
  int j;
  for (j = 0; j < n - 1; j++)
    if (rU <= cum[j]) break;
  return perm[j] - 1;
}

// sample(x, 1, TRUE, probs) given the uniform rU it will consume.  Returns a 0-based
// position or a negative Status.  `p` is scratch (n doubles), `perm` scratch (n ints).
inline int sample_prob1_u(const double* probs, int n, double rU, double* p, int* perm) {
  const int st = sample_prob1_prep(probs, n, p, perm);
  if (st < 0) return st;
  return sample_prob1_pick(p, perm, n, rU, st);
}

inline int sample_prob1(Rng& rng, const double* probs, int n, std::vector<double>& p,
                        std::vector<int>& perm) {
  if ((int)p.size() < n) { p.resize(n); perm.resize(n); }
  // Validation happens before the draw in Rcpp (FixupProb precedes unif_rand()).
  double sum = 0.0;
  int npos = 0;
  for (int i = 0; i < n; i++) {
    double x = probs[i];
    if (!std::isfinite(x) || x < 0) return -kProb;
    if (x > 0) { npos++; sum += x; }
  }
  if (npos == 0) return -kProb;
  (void)sum;
  return sample_prob1_u(probs, n, rng.unif(), p.data(), perm.data());
}

// ------------------------------------------------------------------ nmath rbeta
// Split into the parameter-only setup (parallelisable) and the draw that consumes the
// stream; rbeta(rng, aa, bb) == rbeta_draw(rng, rbeta_setup(aa, bb)) operation for operation.
struct RBeta {
  enum Kind { kConst, kCoin, kBC, kBB } kind;
  double aa, a, b, alpha, beta, gamma, delta, k1, k2, cval;
};

__attribute__((always_inline)) inline RBeta rbeta_setup(double aa, double bb) {
  RBeta r{};
  r.aa = aa;
  r.kind = RBeta::kConst;
  if (std::isnan(aa) || std::isnan(bb) || aa < 0. || bb < 0.) { r.cval = NAN; return r; }
  if (!std::isfinite(aa) && !std::isfinite(bb)) { r.cval = 0.5; return r; }
  if (aa == 0. && bb == 0.) { r.kind = RBeta::kCoin; return r; }
  if (!std::isfinite(aa) || bb == 0.) { r.cval = 1.0; return r; }
  if (!std::isfinite(bb) || aa == 0.) { r.cval = 0.0; return r; }
  r.a = std::fmin(aa, bb);
  r.b = std::fmax(aa, bb);
  r.alpha = r.a + r.b;
  if (r.a <= 1.0) {  // Algorithm BC
    r.kind = RBeta::kBC;
    r.beta = 1.0 / r.a;
    r.delta = 1.0 + r.b - r.a;
    r.k1 = r.delta * (0.0138889 + 0.0416667 * r.a) / (r.b * r.beta - 0.777778);
    r.k2 = 0.25 + (0.5 + 0.25 / r.delta) * r.a;
  } else {           // Algorithm BB
    r.kind = RBeta::kBB;
    r.beta = std::sqrt((r.alpha - 2.0) / (2.0 * r.a * r.b - r.alpha));
    r.gamma = r.a + 1.0 / r.beta;
  }
  return r;
}

// A uniform source yields u and, on request, logit(u) = log(u / (1 - u)) -- the only
// transcendental of an rbeta attempt that depends on the stream alone.
struct RngSrc {
  Rng& r;
  double next(double* lg) {
    const double u = r.unif();
    if (lg) *lg = std::log(u / (1.0 - u));
    return u;
  }
  // an rbeta BB attempt's two uniforms; lz = log(u1 * u1 * u2) or NaN (not precomputed)
  void pair(double* u1, double* lg1, double* u2, double* lz) {
    *u1 = next(lg1);
    *u2 = next(nullptr);
    *lz = NAN;
  }
};

// One attempt of Cheng's algorithm BB (nmath rbeta, a > 1) for uniforms u1, u2 with
// lg1 = log(u1 / (1 - u1)): true when accepted, with w set; rbeta_bb_value(w) is the draw.
// The draw loop and the speculative batches in update_phi share these, so both round
// identically.
// lz, when not NaN, is log(u1 * u1 * u2) computed ahead (same expression as below).
__attribute__((always_inline)) inline bool rbeta_bb_attempt(const RBeta& p, double u1, double lg1, double u2,
                                                             double lz, double* w_out) {
  const double expmax = DBL_MAX_EXP * M_LN2;
  const double a = p.a, b = p.b, alpha = p.alpha;
  const double v = p.beta * lg1;
  double w;
  if (v <= expmax) {
    w = a * std::exp(v);
    if (!std::isfinite(w)) w = DBL_MAX;
  } else {
    w = DBL_MAX;
  }
  *w_out = w;
  const double z = u1 * u1 * u2;
  const double r = p.gamma * v - 1.3862944;
  const double s = a + r - w;
  if (s + 2.609438 >= 5.0 * z) return true;
  const double t = lz == lz ? lz : std::log(z);
  if (s > t) return true;
  return !(r + alpha * std::log(alpha / (b + w)) < t);
}

__attribute__((always_inline)) inline double rbeta_bb_value(const RBeta& p, double w) {
  return (p.aa != p.a) ? p.b / (p.b + w) : w / (p.b + w);
}

template <class S>
__attribute__((always_inline)) inline double rbeta_draw_s(S& src, const RBeta& p) {
  const double expmax = DBL_MAX_EXP * M_LN2;
  if (p.kind == RBeta::kConst) return p.cval;
  if (p.kind == RBeta::kCoin) return (src.next(nullptr) < 0.5) ? 0. : 1.;
  const double a = p.a, b = p.b, alpha = p.alpha, beta = p.beta;
  double r, s, t = 0, u1, u2, v = 0, w = 0, y, z, lg1;
  auto vw = [&](double AA) {
    v = beta * lg1;                       // beta * log(u1 / (1 - u1))
    if (v <= expmax) {
      w = AA * std::exp(v);
      if (!std::isfinite(w)) w = DBL_MAX;
    } else {
      w = DBL_MAX;
    }
  };
  if (p.kind == RBeta::kBC) {
    for (;;) {
      u1 = src.next(&lg1);
      u2 = src.next(nullptr);
      if (u1 < 0.5) {
        y = u1 * u2;
        z = u1 * y;
        if (0.25 * u2 + z - y >= p.k1) continue;
      } else {
        z = u1 * u1 * u2;
        if (z <= 0.25) {
          vw(b);
          break;
        }
        if (z >= p.k2) continue;
      }
      vw(b);
      if (alpha * (std::log(alpha / (a + w)) + v) - 1.3862944 >= std::log(z)) break;
    }
    return (p.aa == a) ? a / (a + w) : w / (a + w);
  }
  (void)r; (void)s; (void)t; (void)v; (void)z;
  for (;;) {
    double lz;
    src.pair(&u1, &lg1, &u2, &lz);
    if (rbeta_bb_attempt(p, u1, lg1, u2, lz, &w)) break;
  }
  return rbeta_bb_value(p, w);
}

__attribute__((always_inline)) inline double rbeta_draw(Rng& rng, const RBeta& p) {
  RngSrc src{rng};
  return rbeta_draw_s(src, p);
}

// A prefix of the stream generated ahead of its consumer: u[k] is the k-th uniform after
// the state at fill() and lg[k] its logit (filled in parallel by the caller); restore()
// leaves an Rng exactly as after c draws (same mt array and mti as drawing them one by
// one, so .Random.seed matches).  Past the prefix, next() continues on the live Rng.
struct StreamAhead {
  Rng start;
  std::vector<double> u, lg, lz;   // lz[k] = log(u[k] * u[k] * u[k + 1])
  std::vector<int64_t> vfirst;                 // first word index served by each mt array
  std::vector<std::array<uint32_t, 624>> arr;  // mt array versions (arr[0] = start.mt)
  int64_t n = 0, used = 0;
  Rng* live = nullptr;
  bool spilled = false;
  const uint32_t* raw = nullptr;   // fill_raw: tempered words; u[] is filled by logits()
  const uint32_t* rawblk = nullptr;  // fill_raw: the words from the start of the state's block
  int mti0 = 0;

  bool fill(const Rng& r, int64_t N) {
    n = 0;
    used = 0;
    spilled = false;
    raw = nullptr;
    rawblk = nullptr;
    if (r.mti > 624) return false;           // never seeded: let the live Rng handle it
    start = r;
    Rng g = r;
    u.resize(N);
    lg.resize(N);
    lz.resize(N);
    vfirst.assign(1, 0);
    arr.resize(1);
    std::memcpy(arr[0].data(), g.mt, sizeof(g.mt));
    for (int64_t k = 0; k < N; ++k) {
      const bool tw = g.mti >= 624;
      const uint32_t y = g.raw();
      if (tw) {
        vfirst.push_back(k);
        arr.emplace_back();
        std::memcpy(arr.back().data(), g.mt, sizeof(g.mt));
      }
      u[k] = Rng::raw_to_unif(y);
    }
    n = N;
    return true;
  }
  // The same prefix from words generated elsewhere (the device windows): r is the state
  // before the first word (mt array, mti); blk holds the tempered words of r's block from
  // its start, then the following blocks (at least through the block of word N - 1), so
  // word k is blk[r.mti + k] and every later state array is the untempered block.  u[] is
  // computed by logits(), the arrays by restore() when needed.
  void fill_raw(const Rng& r, const uint32_t* blk, int64_t N) {
    start = r;
    used = 0;
    spilled = false;
    rawblk = blk;
    mti0 = r.mti;
    raw = blk + r.mti;
    u.resize(N);
    lg.resize(N);
    lz.resize(N);
    vfirst.assign(1, 0);
    arr.resize(1);
    n = N;
  }
  void logits(int64_t a, int64_t b) {
    if (raw)
      for (int64_t k = a; k < b; ++k) u[k] = Rng::raw_to_unif(raw[k]);
    for (int64_t k = a; k < b; ++k) {
      lg[k] = std::log(u[k] / (1.0 - u[k]));
      const double un = k + 1 < b || !raw ? u[k + 1 < n ? k + 1 : k] : Rng::raw_to_unif(raw[k + 1 < n ? k + 1 : k]);
      lz[k] = k + 1 < n ? std::log(u[k] * u[k] * un) : NAN;
    }
  }
  void restore(Rng& r, int64_t c) const {
    const uint64_t ep = r.epoch;
    if (c == 0) {
      r = start;
    } else if (rawblk) {
      const int64_t w = c - 1;
      const int64_t v = (mti0 + w) / 624;
      for (int i = 0; i < 624; ++i) r.mt[i] = mt_untemper(rawblk[624 * v + i]);
      r.mti = (int32_t)(mti0 + w - 624 * v + 1);
      r.pos = start.pos + (uint64_t)c;
    } else {
      const int64_t w = c - 1;
      size_t v = 0;
      while (v + 1 < vfirst.size() && vfirst[v + 1] <= w) ++v;
      std::memcpy(r.mt, arr[v].data(), sizeof(r.mt));
      r.mti = v == 0 ? (int32_t)(start.mti + c) : (int32_t)(w - vfirst[v] + 1);
      r.pos = start.pos + (uint64_t)c;
    }
    r.epoch = ep;
  }
  // Entries produced by other threads in chunks: positions at or past `avail` are read only
  // after wait_avail(pos) (which returns the new limit); unset, the whole prefix is ready.
  int64_t avail = INT64_MAX;
  std::function<int64_t(int64_t)> wait_avail;
  void need(int64_t pos) {
    if (pos >= avail && pos < n) avail = wait_avail(pos);
  }

  double next(double* lgout) {
    if (used < n) {
      need(used);
      if (lgout) *lgout = lg[used];
      return u[used++];
    }
    if (!spilled && n > 0) {
      restore(*live, n);
      spilled = true;
    }
    ++used;
    const double x = live->unif();
    if (lgout) *lgout = std::log(x / (1.0 - x));
    return x;
  }
  void pair(double* u1, double* lg1, double* u2, double* lzo) {
    if (used + 1 < n) {
      need(used + 1);
      *u1 = u[used];
      *lg1 = lg[used];
      *u2 = u[used + 1];
      *lzo = lz[used];
      used += 2;
      return;
    }
    *u1 = next(lg1);
    *u2 = next(nullptr);
    *lzo = NAN;
  }
  // Leave the live Rng after everything drawn so far.
  void finish() {
    if (n > 0 && !spilled) restore(*live, used);
  }
};

inline double rbeta(Rng& rng, double aa, double bb) { return rbeta_draw(rng, rbeta_setup(aa, bb)); }

// ------------------------------------------------------------------ qbeta branch test
// lgamma without the global signgam write (the host pool evaluates these concurrently)
inline double lgam(double x) {
  int sg;
  return ::lgamma_r(x, &sg);
}

namespace detail {
inline double betacf(double a, double b, double x) {
  const double FPMIN = 1e-300, EPS = 1e-16;
  double qab = a + b, qap = a + 1.0, qam = a - 1.0, c = 1.0, d = 1.0 - qab * x / qap;
  if (std::fabs(d) < FPMIN) d = FPMIN;
  d = 1.0 / d;
  double h = d;
  for (int m = 1; m <= 200000; m++) {
    int m2 = 2 * m;
    double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
    d = 1.0 + aa * d; if (std::fabs(d) < FPMIN) d = FPMIN;
    c = 1.0 + aa / c; if (std::fabs(c) < FPMIN) c = FPMIN;
    d = 1.0 / d; h *= d * c;
    aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
    d = 1.0 + aa * d; if (std::fabs(d) < FPMIN) d = FPMIN;
    c = 1.0 + aa / c; if (std::fabs(c) < FPMIN) c = FPMIN;
    d = 1.0 / d;
    double del = d * c;
    h *= del;
    if (std::fabs(del - 1.0) < EPS) break;
  }
  return h;
}
}  // namespace detail

inline double pbeta(double x, double a, double b) {
  if (x <= 0.0) return 0.0;
  if (x >= 1.0) return 1.0;
  double lbt = lgam(a + b) - lgam(a) - lgam(b) + a * std::log(x) +
               b * std::log1p(-x);
  if (x < (a + 1.0) / (a + b + 2.0)) return std::exp(lbt) * detail::betacf(a, b, x) / a;
  return 1.0 - std::exp(lbt) * detail::betacf(b, a, 1.0 - x) / b;
}

// R::qbeta(0.1, a, b, 1, 0) < x   <=>   pbeta(x; a, b) > 0.1.
// Cantelli's inequality settles most calls without the continued fraction: with mean mu
// and variance s2 of Beta(a, b), P(X > x) <= s2 / (s2 + (x - mu)^2) for x > mu and
// P(X <= x) <= s2 / (s2 + (mu - x)^2) for x < mu.
inline bool qbeta01_lt(double a, double b, double x) {
  if (std::isnan(a) || std::isnan(b) || a < 0 || b < 0) return false;
  if (b == 0) return false;
  if (a == 0) return x > 0;
  const double mu = a / (a + b);
  const double s2 = a * b / ((a + b) * (a + b) * (a + b + 1.0));
  const double dlt = x - mu;
  const double bound = s2 / (s2 + dlt * dlt);
  if (dlt > 0 && bound < 0.85) return true;    // P(X <= x) >= 0.15 > 0.1
  if (dlt < 0 && bound < 0.05) return false;   // P(X <= x) <= 0.05 < 0.1
  return pbeta(x, a, b) > 0.1;
}

// ------------------------------------------------------------------ GSL 2F1
enum { GSL_SUCCESS = 0, GSL_EDOM = 1, GSL_EMAXITER = 11, GSL_EUNIMPL = 24 };

inline int hyperg_2F1(double a, double b, double c, double x, double* val) {
  const double eps = 2.2204460492503131e-16, loc_eps = 1000.0 * eps;
  *val = 0.0;
  if (x < -1.0 || 1.0 <= x) return GSL_EDOM;
  if (std::fabs(c - b) < loc_eps || std::fabs(c - a) < loc_eps) {
    *val = std::exp((c - a - b) * std::log(1.0 - x));
    return GSL_SUCCESS;
  }
  if (!(a >= 0.0 && b >= 0.0 && c >= 0.0 && x >= 0.0 && x < 0.995)) return GSL_EUNIMPL;
  if (std::fabs(c) < eps) return GSL_EUNIMPL;
  double sum_pos = 1.0, sum_neg = 0.0, del_pos = 1.0, del_neg = 0.0, del = 1.0, k = 0.0;
  int i = 0;
  do {
    if (++i > 30000) { *val = sum_pos - sum_neg; return GSL_EMAXITER; }
    del *= (a + k) * (b + k) * x / ((c + k) * (k + 1.0));
    if (del > 0.0) {
      del_pos = del;
      sum_pos += del;
    } else if (del == 0.0) {
      del_pos = 0.0;
      del_neg = 0.0;
      break;
    } else {
      del_neg = -del;
      sum_neg -= del;
    }
    k += 1.0;
  } while (std::fabs((del_pos + del_neg) / (sum_pos - sum_neg)) > eps);
  *val = sum_pos - sum_neg;
  return GSL_SUCCESS;
}

// Extension (HDPM_OPT_HIG_LOGSPACE; not the reference): log 2F1.  The reference's series
// runs first; when it ends finite its log is returned, so those values keep their bits.
// When it overflows (clusters of ~1.4k+ members) or runs out of its 30000
// terms, the same positive series is summed again with the partial sum rescaled by 2^-960
// whenever it passes 2^960, for up to 10^7 terms.  Statuses as hyperg_2F1.
//
// The HIG constants only take 2F1(A, 1; C; x) = (C-1) x^(1-C) (1-x)^(C-A-1) B_x(C-1, A-C+1)
// (DLMF 15.4 / 8.17), and in the upper tail of the incomplete beta its log has the closed
// form log2f1_a1_upper below (lgamma and the continued fraction of pbeta, ~1e-15 relative).
// Where that puts log 2F1 above 712 the plain series would overflow (log DBL_MAX = 709.78)
// after summing up to ~5 A terms, so the closed form is returned without it.
inline double log2f1_a1_upper(double A, double C, double x) {
  const double p = C - 1.0, q = A - C + 1.0;
  // log B_x(p, q) = lbeta(p, q) + log1p(-I_{1-x}(q, p))
  const double lbeta = lgam(p) + lgam(q) - lgam(p + q);
  const double lt = q * std::log1p(-x) + p * std::log(x) - std::log(q) + std::log(detail::betacf(q, p, 1.0 - x)) - lbeta;
  return std::log(p) - p * std::log(x) - q * std::log1p(-x) + lbeta + std::log1p(-std::exp(lt));
}

inline int log_hyperg_2F1(double a, double b, double c, double x, double* lval) {
  const double eps = 2.2204460492503131e-16, loc_eps = 1000.0 * eps;
  double L = NAN;
  if ((a == 1.0 || b == 1.0) && x > 0.0 && x < 1.0) {
    const double A = b == 1.0 ? a : b, p = c - 1.0, q = A - c + 1.0;
    if (p > 0.0 && q > 0.0 && x >= (p + 1.0) / (p + q + 2.0)) {
      L = log2f1_a1_upper(A, c, x);
      if (L > 712.0) {
        *lval = L;
        return GSL_SUCCESS;
      }
    }
  }
  double plain;
  const int st = hyperg_2F1(a, b, c, x, &plain);
  *lval = NAN;
  if (st == GSL_SUCCESS && std::isfinite(plain)) {
    *lval = std::log(plain);
    return st;
  }
  if (st != GSL_SUCCESS && st != GSL_EMAXITER) return st;
  if (std::isfinite(L)) {
    *lval = L;
    return GSL_SUCCESS;
  }
  if (std::fabs(c - b) < loc_eps || std::fabs(c - a) < loc_eps) {
    *lval = (c - a - b) * std::log(1.0 - x);       // exp() overflowed in the plain path
    return GSL_SUCCESS;
  }
  double sum = 1.0, del = 1.0, k = 0.0, scale = 0.0;
  int i = 0;
  do {
    if (++i > 10000000) { *lval = std::log(sum) + scale * M_LN2; return GSL_EMAXITER; }
    del *= (a + k) * (b + k) * x / ((c + k) * (k + 1.0));
    if (del == 0.0) break;
    sum += del;
    if (sum > 0x1p960) {
      sum *= 0x1p-960;
      del *= 0x1p-960;
      scale += 960.0;
    }
    k += 1.0;
  } while (std::fabs(del / sum) > eps);
  *lval = scale == 0.0 ? std::log(sum) : std::log(sum) + scale * M_LN2;
  return GSL_SUCCESS;
}

// hg:11-48.  Sets *err = kGsl where the reference throws.  `logspace`: the extension above
// (an overflowing series gives its finite log instead of the throw).
inline double norm_const2(double d, double c, double m, int* err, bool logspace = false) {
  if (logspace) {
    double lv;
    const int st = log_hyperg_2F1(d + c, 1, d + 2, (m - 1) / m, &lv);
    if (st != GSL_SUCCESS) {
      if (st == GSL_EMAXITER) return -INFINITY;
      *err = kGsl;
      return NAN;
    }
    if (!std::isfinite(lv)) { *err = kGsl; return NAN; }
    return std::log(d + 1) + (d + c) * std::log(m) - lv;
  }
  double val;
  int st = hyperg_2F1(d + c, 1, d + 2, (m - 1) / m, &val);
  if (st != GSL_SUCCESS) {
    if (st == GSL_EMAXITER) return -INFINITY;
    *err = kGsl;
    return NAN;
  }
  if (!std::isfinite(val) || val == 0) { *err = kGsl; return NAN; }
  return std::log(d + 1) + (d + c) * std::log(m) - std::log(val);
}

inline double lF_conK2(double u, double d, double c, double m, double lK, bool logspace = false) {  // hg:183-217
  if (u == 0) return -INFINITY;
  if (u == 1) return 0;
  double x = u * (m - 1) / (1 + u * (m - 1));
  double lapp;
  if (logspace) {
    if (log_hyperg_2F1(1, d + c, d + 2, x, &lapp) != GSL_SUCCESS) lapp = NAN;
  } else {
    double app;
    if (hyperg_2F1(1, d + c, d + 2, x, &app) != GSL_SUCCESS) app = NAN;
    lapp = std::log(app);
  }
  return lK - std::log(d + 1) + (d + 1) * std::log(u) - (d + c) * std::log(1 + u * (m - 1)) + lapp;
}

inline double bisec_hyper2(double d, double c, double m, double Omega, int* err,
                           bool logspace = false) {  // hg:221-287
  double centro = 0.5;
  double lK = norm_const2(d, c, m, err, logspace);
  if (*err) return NAN;
  double app = lF_conK2(centro, d, c, m, lK, logspace) - std::log(Omega);
  double su, giu;
  int counter = 1;
  if (app < 0) { giu = 0.5; su = 1; } else { giu = 0; su = 0.5; }
  while (((su - giu) > 0.000000001) & (counter < 150)) {
    centro = (su + giu) / 2;
    app = lF_conK2(centro, d, c, m, lK, logspace) - std::log(Omega);
    if (app < 0) giu = centro; else su = centro;
    counter = counter + 1;
  }
  return centro;
}

// rhig(1, v, w, m) (hg:346-378); `beta_path` is the cached hg:359 decision.
inline double rhig1_decided(Rng& rng, double v, double w, double m, bool beta_path, int* err,
                            bool logspace = false) {
  double out;
  if (beta_path) {
    double x = rbeta(rng, w + 1, v - 1);
    while (x > (m - 1) / m) x = rbeta(rng, w + 1, v - 1);
    out = x / ((m - 1) * (1 - x));
  } else {
    double Omega = rng.unif();
    out = bisec_hyper2(w, v, m, Omega, err, logspace);
    if (*err) return NAN;
  }
  return -1 / std::log(out);
}

inline bool rhig_beta_path(double v, double w, double m) {
  return qbeta01_lt(w + 1, v - 1, (m - 1) / m) && (m - 1) / m > 4 / 5;
}

inline double rhig1(Rng& rng, double v, double w, double m, int* err, bool logspace = false) {
  return rhig1_decided(rng, v, w, m, rhig_beta_path(v, w, m), err, logspace);
}

// dhamming (cf:355-377) split into its two attribute-level values: the device adds
// tab_match when x == c and tab_mismatch otherwise, which is bit-identical to calling
// dhamming(x, c, s, m) because numerator - denominator is evaluated the same way.
inline void dhamming_pair(double s, int attrisize, double* match, double* mismatch) {
  double exp_term = std::exp(1.0 / s);
  double attr_ratio = (attrisize - 1.0) / exp_term;
  double denominator = std::log(1.0 + attr_ratio);
  double num0 = -0 / s;          // diff = 0 -> (double)(-0) / s = +0.0
  double num1 = -1 / s;          // diff = 1 -> (double)(-1) / s
  *match = num0 - denominator;
  *mismatch = num1 - denominator;
}

}  // namespace hdpm
