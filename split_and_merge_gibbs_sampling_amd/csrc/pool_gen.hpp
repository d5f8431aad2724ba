// pool_gen.hpp -- the latent pool (code/launcher.cpp:67-77, 123-129) generated in parallel,
// stream-exactly: shared host/device arithmetic and the host-side parse.
//
// The reference draws P entries one after another from R's stream: per entry D centers
// (one uniform each, common_functions.cpp:185-202) then D sigmas (sample_sigma_1_cluster,
// cf:218-235), each sigma a rhig (hyperg.cpp:346-378) that repeats rbeta(w + 1, v - 1)
// (nmath Cheng BB / BC, two uniforms per attempt) until an attempt is accepted and
// x <= (m - 1) / m.  Only the attempt outcomes make the stream positions data-dependent,
// so the device
//   1. generates the whole slice of the stream (k_mt_gen_multi, jump-ahead),
//   2. decides every possible attempt, one per (stream position, attribute class):
//      accept(p) = rbeta attempt on (u_p, u_{p+1}) accepted and x <= (m - 1) / m,
//      packed per class and position parity (k_pool_accept),
// then the host walks the entries: D positions of centers, then for each run of
// attributes of one class the run's length-th accepted attempt at the parity of the run's
// start (popcounts over the packed words), which gives every entry's start; finally the
// device recomputes the accepted attempts of every entry and the sigma / dhamming tables /
// bound records from them (k_pool_values).  Every floating-point step is the host's own
// (glibc_math.hpp replicas of libm exp/log, IEEE add/mul/div), so the pool, and the
// stream position after it, are bit-identical to the sequential generator.
//
// Classes: attributes with equal (v_j, w_j, m_j).  Only rbeta kinds BB and BC with the
// rhig beta path qualify; anything else (the bisection path, degenerate rbeta arguments)
// uses the sequential host generator.
#pragma once
#include <cstdint>

#include "glibc_math.hpp"

namespace hdpm {

struct PoolClass {
  int kind;          // 2 = BC, 3 = BB (RBeta::Kind)
  int pad;
  double aa, a, b, alpha, beta, gamma, k1, k2;   // rbeta_setup(w + 1, v - 1)
  double thr;        // (m - 1) / m   (hyperg.cpp:360)
  double m;          // m_j as double
};

// R's unif_rand() fixup of one MT output
HDPM_HD inline double pool_unif(uint32_t y) {
  const double i2_32m1 = 2.328306437080797e-10;
  const double x = (double)y * 2.3283064365386963e-10;
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

// One rbeta attempt on (u1, u2) (rmath.hpp rbeta_bb_attempt / the BC loop body, operation
// for operation); true when accepted, with the draw in *x.
HDPM_HD inline bool pool_attempt(const PoolClass& C, double u1, double u2, const uint64_t* texp,
                                 const uint64_t* tlog, double* x) {
  const double expmax = 1024 * 0.693147180559945309417232121458;   // DBL_MAX_EXP * M_LN2
  const double lg1 = glibc::log_r(u1 / (1.0 - u1), tlog);
  const double v = C.beta * lg1;
  if (C.kind == 3) {   // BB
    const double a = C.a, b = C.b, alpha = C.alpha;
    double w;
    if (v <= expmax) {
      w = a * glibc::exp_r(v, texp);
      if (!(w <= 1.7976931348623157e308)) w = 1.7976931348623157e308;
    } else {
      w = 1.7976931348623157e308;
    }
    *x = (C.aa != C.a) ? b / (b + w) : w / (b + w);
    const double z = u1 * u1 * u2;
    const double r = C.gamma * v - 1.3862944;
    const double s = a + r - w;
    if (s + 2.609438 >= 5.0 * z) return true;
    const double t = glibc::log_r(z, tlog);
    if (s > t) return true;
    return !(r + alpha * glibc::log_r(alpha / (b + w), tlog) < t);
  }
  // BC
  const double a = C.a, b = C.b, alpha = C.alpha;
  double z;
  if (u1 < 0.5) {
    const double y = u1 * u2;
    z = u1 * y;
    if (0.25 * u2 + z - y >= C.k1) return false;
  } else {
    z = u1 * u1 * u2;
    if (z > 0.25 && z >= C.k2) return false;
  }
  double w;
  if (v <= expmax) {
    w = b * glibc::exp_r(v, texp);
    if (!(w <= 1.7976931348623157e308)) w = 1.7976931348623157e308;
  } else {
    w = 1.7976931348623157e308;
  }
  *x = (C.aa == a) ? a / (a + w) : w / (a + w);
  if (!(u1 < 0.5) && z <= 0.25) return true;
  return alpha * (glibc::log_r(alpha / (a + w), tlog) + v) - 1.3862944 >= glibc::log_r(z, tlog);
}

// accept(p) of the packed tables: attempt accepted and x <= (m - 1) / m
HDPM_HD inline bool pool_accept(const PoolClass& C, double u1, double u2, const uint64_t* texp,
                                const uint64_t* tlog) {
  double x = 0.0;
  return pool_attempt(C, u1, u2, texp, tlog, &x) && !(x > C.thr);
}

// sigma of an accepted attempt (hyperg.cpp:360-365, 377) and its dhamming pair
// (rmath.hpp dhamming_pair, common_functions.cpp:355-377)
HDPM_HD inline void pool_sigma_tables(const PoolClass& C, double x, int attrisize, const uint64_t* texp,
                                      const uint64_t* tlog, double* sigma, double* match, double* mismatch) {
  const double m = C.m;
  const double out = x / ((m - 1) * (1 - x));
  const double s = -1 / glibc::log_r(out, tlog);
  *sigma = s;
  const double exp_term = glibc::exp_r(1.0 / s, texp);
  const double attr_ratio = (attrisize - 1.0) / exp_term;
  const double denominator = glibc::log_r(1.0 + attr_ratio, tlog);
  const double num0 = 0 / s;
  const double num1 = -1 / s;
  *match = num0 - denominator;
  *mismatch = num1 - denominator;
}

// index (0-based) of the k-th set bit of v (k < popcount(v))
HDPM_HD inline int pool_select64(uint64_t v, int k) {
  int base = 0;
  for (int sh = 32; sh >= 1; sh >>= 1) {
    const uint64_t lo = v & ((sh == 64 ? ~0ull : (1ull << sh) - 1));
    const int c = __builtin_popcountll(lo);
    if (k >= c) {
      k -= c;
      v >>= sh;
      base += sh;
    } else {
      v = lo;
    }
  }
  return base;
}

// ------------------------------------------------------------------ host parse
// Packed accept tables: bm[(c * 2 + par) * nwords + w] bit i = accept of class c at
// stream position 2 (64 w + i) + par.
struct PoolRuns {
  int n = 0;
  const int* cls = nullptr;   // class of run r
  const int* len = nullptr;   // attributes in run r
};

// Position after the len-th accepted attempt at parity(pos), from pos; -1 past the tables.
HDPM_HD inline int64_t pool_select_run(const uint64_t* B, int64_t nwords, int64_t pos, int len) {
  const int par = (int)(pos & 1);
  const int64_t slot = pos >> 1;
  int64_t w = slot >> 6;
  if (w >= nwords) return -1;
  uint64_t word = B[w] & (~0ull << (slot & 63));
  int need = len;
  for (;;) {
    const int c = __builtin_popcountll(word);
    if (c >= need) return 2 * (w * 64 + pool_select64(word, need - 1)) + par + 2;
    need -= c;
    if (++w >= nwords) return -1;
    word = B[w];
  }
}

// F(pos): where the entry that starts at pos ends (the next entry's start): D center
// uniforms, then per run the len-th accepted attempt of its class; -1 past the tables.
HDPM_HD inline int64_t pool_entry_end(const uint64_t* bm, int64_t nwords, int d, const PoolRuns& R, int64_t pos) {
  pos += d;
  for (int r = 0; r < R.n; ++r) {
    pos = pool_select_run(bm + ((int64_t)R.cls[r] * 2 + (pos & 1)) * nwords, nwords, pos, R.len[r]);
    if (pos < 0) return -1;
  }
  return pos;
}

// Entry starts (relative to the slice) for entries [e0, e1) from `pos` (the start of e0);
// returns the position after entry e1 - 1, or -1 when the tables end first.
inline int64_t pool_parse(const uint64_t* bm, int64_t nwords, int d, const PoolRuns& R, int64_t pos, int64_t e0,
                          int64_t e1, int64_t* starts) {
  for (int64_t e = e0; e < e1; ++e) {
    starts[e] = pos;
    pos = pool_entry_end(bm, nwords, d, R, pos);
    if (pos < 0) return -1;
  }
  return pos;
}

// ------------------------------------------------------------------ entry starts by segments
// s_{e+1} = F(s_e), s_0 = 0: a chain through the whole slice.  The slice is cut into chunks of
// B positions.  The first start of the chain at or after chunk c's first position X_c lies in
// the window [X_c, X_c + Lw) whenever every entry is shorter than Lw, so every candidate of the
// window (every position, or every even one when D is even: all starts are then even) is
// walked to its first start >= X_{c+1}:  T_c[i] = that start's candidate index in chunk c + 1's
// window | entries walked << 16.  The chain is the path through the tables from candidate 0 of
// chunk 0: composed per group of G chunks (one thread per candidate), followed over the groups
// serially, unrolled per chunk, and each chunk then walks its entries from its true first
// start and writes them.  Exact for any slice; an entry longer than Lw on the chain (beyond
// 14 standard deviations) is reported and the host parses serially.
struct PoolSegPlan {
  int64_t B = 0;        // positions per chunk (even)
  int step = 2;         // candidate spacing: 2 when D is even, else 1
  int ncand = 0;        // candidates per window, < 0xFFFF
  int64_t nchunks = 0;  // ceil(count / B)
  int G = 64;           // chunks per group
  int64_t ngroups = 0;
};
constexpr uint32_t kSegBad = 0xFFFFu;   // low half of a table cell: the walk left the tables / window

// T_c[i] (see above)
HDPM_HD inline uint32_t pool_seg_cell(const uint64_t* bm, int64_t nwords, int d, const PoolRuns& R,
                                      const PoolSegPlan& sp, int64_t c, int i) {
  const int64_t X = c * sp.B, Xn = X + sp.B;
  int64_t p = X + (int64_t)i * sp.step;
  uint32_t n = 0;
  while (p < Xn) {
    p = pool_entry_end(bm, nwords, d, R, p);
    if (p < 0 || ++n >= 0xFFFFu) return kSegBad;
  }
  const int64_t j = (p - Xn) / sp.step;
  return j < sp.ncand ? (uint32_t)j | (n << 16) : kSegBad;
}

#ifdef __HIPCC__
// ------------------------------------------------------------------ device kernels (pool.hip)
struct PoolAcceptArgs {
  const uint32_t* raw;     // the slice of the stream (count outputs)
  int64_t count;
  int nclass;
  const PoolClass* cls;
  uint64_t* bm;            // [nclass][2][nwords]
  int64_t nwords;          // ceil(count / 128)
  const uint64_t* gtab;    // kGlibcExpTab then kGlibcLogTab (512 words)
  int par_mask;            // bit p: the parity-p tables are read (d even: entries and runs all start even)
};

// The entry starts by segments (k_pool_seg, k_pool_seg_group, k_pool_seg_top, k_pool_seg_fill,
// k_pool_seg_emit; see PoolSegPlan above).
struct PoolSegArgs {
  const uint64_t* bm;
  int64_t nwords;
  int d;
  PoolRuns R;              // device arrays
  PoolSegPlan sp;
  int64_t P;
  uint32_t* T;             // [nchunks][ncand]
  int32_t* gj;             // [ngroups][ncand] the group's composed next index (-1: a broken cell)
  int32_t* gn;             // [ngroups][ncand] entries over the group
  int32_t* cidx;           // [nchunks] the chain's first start in chunk c (candidate index; -1: not on it)
  int64_t* cE;             // [nchunks] its entry index
  int64_t* aux;            // [1] the group unrolled by k_pool_seg_top (ngroups: none)
  int64_t* starts;         // [P + 1]
  int* err;                // bit 2: the chain left a window (serial host parse); bit 3: the tables end before entry P
};

struct PoolValueArgs {
  const uint32_t* raw;
  int64_t count;
  const int64_t* starts;   // P + 1 entry starts (relative to raw)
  int64_t P;
  int d, dp, wb, Ws, bw;
  const int32_t* att;
  int nruns;
  const int* run_cls;
  const int* run_len;
  const PoolClass* cls;
  const uint64_t* bm;
  int64_t nwords;
  const uint64_t* gtab;
  uint8_t* codes;          // [P][dp]
  double* tab;             // [P][d][2]
  double* sig;             // [P][d]
  uint64_t* bnd;           // [P][bw]
  int* err;                // bit 0: walk disagrees with the host parse, bit 1: rejected attempt
};

hipError_t launch_pool_accept(const PoolAcceptArgs& a, hipStream_t s);
hipError_t launch_pool_values(const PoolValueArgs& a, hipStream_t s);
hipError_t launch_pool_seg(const PoolSegArgs& a, hipStream_t s);
#endif

}  // namespace hdpm
