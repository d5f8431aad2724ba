// pool_host.hpp -- host-side planning of the stream-exact pool generator (pool_gen.hpp):
// attribute classes and runs, slice-length estimate, untempering, and a host model of the
// whole pipeline that tests compare with the sequential generator.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "pool_gen.hpp"
#include "rmath.hpp"

namespace hdpm {

struct PoolPlan {
  bool ok = false;                 // every attribute on the rhig beta path with rbeta BB / BC
  std::vector<PoolClass> cls;
  std::vector<int> run_cls, run_len;
  std::vector<double> accept;      // per class: P(attempt accepted and x <= (m-1)/m)
  double mean_len = 0, var_len = 0;   // stream positions per entry
};

// Classes = distinct (v_j, w_j, m_j); runs = maximal stretches of one class in attribute
// order.  Acceptance rates are estimated on a private stream (not the chain's).
inline PoolPlan pool_plan(int d, const int32_t* att, const double* v, const double* w, int max_classes = 16) {
  PoolPlan pl;
  std::vector<int> cl(d);
  std::vector<double> key;   // (v, w, m) triples
  for (int j = 0; j < d; ++j) {
    const double mj = (double)att[j];
    if (!rhig_beta_path(v[j], w[j], mj)) return pl;
    const RBeta rb = rbeta_setup(w[j] + 1, v[j] - 1);
    if (rb.kind != RBeta::kBB && rb.kind != RBeta::kBC) return pl;
    int c = -1;
    for (size_t q = 0; q < pl.cls.size(); ++q)
      if (key[3 * q] == v[j] && key[3 * q + 1] == w[j] && key[3 * q + 2] == mj) c = (int)q;
    if (c < 0) {
      if ((int)pl.cls.size() >= max_classes) return pl;
      PoolClass C{};
      C.kind = rb.kind == RBeta::kBB ? 3 : 2;
      C.aa = rb.aa; C.a = rb.a; C.b = rb.b; C.alpha = rb.alpha; C.beta = rb.beta; C.gamma = rb.gamma;
      C.k1 = rb.k1; C.k2 = rb.k2;
      C.thr = (mj - 1) / mj;
      C.m = mj;
      c = (int)pl.cls.size();
      pl.cls.push_back(C);
      key.insert(key.end(), {v[j], w[j], mj});
    }
    cl[j] = c;
  }
  for (int j = 0; j < d; ++j) {
    if (j > 0 && cl[j] == cl[j - 1]) { pl.run_len.back()++; continue; }
    pl.run_cls.push_back(cl[j]);
    pl.run_len.push_back(1);
  }
  Rng r;
  r.set_seed(7331u);
  const int trials = 20000;
  for (const PoolClass& C : pl.cls) {
    int acc = 0;
    for (int t = 0; t < trials; ++t) {
      const double u1 = r.unif(), u2 = r.unif();
      acc += pool_accept(C, u1, u2, glibc::kGlibcExpTab, glibc::kGlibcLogTab);
    }
    pl.accept.push_back(std::max(acc, 1) / (double)trials);
  }
  pl.mean_len = d;
  for (int j = 0; j < d; ++j) {
    const double p = pl.accept[cl[j]];
    pl.mean_len += 2.0 / p;
    pl.var_len += 4.0 * (1.0 - p) / (p * p);
  }
  pl.ok = true;
  return pl;
}

// Slice length that holds P entries with overwhelming probability (mean + 10 sd + 0.5%),
// plus `extra` for a retry after an overrun.
inline int64_t pool_slice_len(const PoolPlan& pl, int64_t P, double extra = 1.0) {
  const double mu = pl.mean_len * (double)P, sd = std::sqrt(pl.var_len * (double)P);
  return (int64_t)((mu * 1.005 + 10.0 * sd) * extra) + 4096;
}

// (mt_untemper: rmath.hpp)

// Chunking of the segment parse (pool_gen.hpp PoolSegPlan): windows of Lw = mean + 14 sd +
// 16 positions (one entry's length, with margin), ~128 entries per chunk, 64 chunks per group.
inline PoolSegPlan pool_seg_plan(const PoolPlan& pl, int d, int64_t count) {
  PoolSegPlan sp;
  sp.step = (d % 2 == 0) ? 2 : 1;
  int64_t Lw = (int64_t)std::ceil(pl.mean_len + 14.0 * std::sqrt(pl.var_len)) + 16;
  Lw = (Lw + 1) & ~(int64_t)1;
  sp.ncand = (int)(Lw / sp.step);
  int64_t B = (int64_t)std::ceil(128.0 * pl.mean_len);
  B = std::max(B, 2 * Lw);
  sp.B = (B + 1) & ~(int64_t)1;
  sp.nchunks = (count + sp.B - 1) / sp.B;
  sp.G = 64;
  sp.ngroups = (sp.nchunks + sp.G - 1) / sp.G;
  return sp;
}

// Host model of the segment parse, step for step as the device kernels (pool.hip k_pool_seg*):
// the entry starts [0, P] into starts; returns the position after entry P - 1, -1 when the
// tables end before it, -2 when the chain leaves a window.
inline int64_t pool_parse_segments(const uint64_t* bm, int64_t nwords, int d, const PoolRuns& R, const PoolSegPlan& sp,
                                   int64_t P, int64_t* starts) {
  const int64_t nc = sp.nchunks;
  std::vector<uint32_t> T((size_t)nc * sp.ncand);
  for (int64_t c = 0; c < nc; ++c)
    for (int i = 0; i < sp.ncand; ++i) T[(size_t)c * sp.ncand + i] = pool_seg_cell(bm, nwords, d, R, sp, c, i);
  std::vector<int32_t> gj((size_t)sp.ngroups * sp.ncand), gn(gj.size());
  for (int64_t g = 0; g < sp.ngroups; ++g)          // k_pool_seg_group
    for (int i = 0; i < sp.ncand; ++i) {
      int idx = i, n = 0;
      bool bad = false;
      for (int64_t c = g * sp.G; c < std::min(nc, (g + 1) * sp.G); ++c) {
        const uint32_t t = T[(size_t)c * sp.ncand + idx];
        if ((t & 0xFFFFu) == kSegBad) { bad = true; break; }
        idx = (int)(t & 0xFFFFu);
        n += (int)(t >> 16);
      }
      gj[(size_t)g * sp.ncand + i] = bad ? -1 : idx;
      gn[(size_t)g * sp.ncand + i] = n;
    }
  std::vector<int32_t> cidx(nc, -1);
  std::vector<int64_t> cE(nc, 0);
  int64_t gfin = sp.ngroups;                          // k_pool_seg_top
  {
    int idx = 0;
    int64_t E = 0;
    for (int64_t g = 0; g < sp.ngroups; ++g) {
      const int32_t j = gj[(size_t)g * sp.ncand + idx], n = gn[(size_t)g * sp.ncand + idx];
      cidx[g * sp.G] = idx;
      cE[g * sp.G] = E;
      if (j < 0 || E + n > P) {
        gfin = g;
        for (int64_t c = g * sp.G; c < std::min(nc, (g + 1) * sp.G) && E <= P; ++c) {
          cidx[c] = idx;
          cE[c] = E;
          const uint32_t t = T[(size_t)c * sp.ncand + idx];
          if ((t & 0xFFFFu) == kSegBad) break;
          idx = (int)(t & 0xFFFFu);
          E += t >> 16;
        }
        break;
      }
      idx = j;
      E += n;
    }
    if (gfin == sp.ngroups) return -1;
  }
  for (int64_t g = 0; g < gfin; ++g) {                // k_pool_seg_fill
    int idx = cidx[g * sp.G];
    int64_t E = cE[g * sp.G];
    for (int64_t c = g * sp.G; c < std::min(nc, (g + 1) * sp.G); ++c) {
      cidx[c] = idx;
      cE[c] = E;
      const uint32_t t = T[(size_t)c * sp.ncand + idx];
      idx = (int)(t & 0xFFFFu);
      E += t >> 16;
    }
  }
  int err = 0;
  for (int64_t c = 0; c < nc; ++c) {                  // k_pool_seg_emit
    if (cidx[c] < 0) continue;
    const int64_t Xn = (c + 1) * sp.B;
    int64_t p = c * sp.B + (int64_t)cidx[c] * sp.step, e = cE[c];
    bool done = false;
    while (p < Xn) {
      starts[e] = p;
      if (e == P) { done = true; break; }
      p = pool_entry_end(bm, nwords, d, R, p);
      if (p < 0) { err |= 8; done = true; break; }
      ++e;
    }
    if (!done && !(c + 1 < nc && cidx[c + 1] == (p - Xn) / sp.step && cE[c + 1] == e)) err |= 4;
  }
  if (err & 8) return -1;
  if (err & 4) return -2;
  return starts[P];
}

// Host model of the device pipeline on `raw` (the slice): packed accept tables, parse,
// values.  Returns the position after the P-th entry, or -1 on overrun.
inline int64_t pool_model(const PoolPlan& pl, int d, const int32_t* att, const uint32_t* raw, int64_t count, int64_t P,
                          uint8_t* centers, double* sigma) {
  const int nc = (int)pl.cls.size();
  const int64_t nwords = (count + 127) / 128;
  std::vector<uint64_t> bm((size_t)nc * 2 * nwords, 0);
  for (int64_t p = 0; p + 1 < count; ++p) {
    const double u1 = pool_unif(raw[p]), u2 = pool_unif(raw[p + 1]);
    const int par = (int)(p & 1);
    const int64_t slot = p >> 1;
    for (int c = 0; c < nc; ++c)
      if (pool_accept(pl.cls[c], u1, u2, glibc::kGlibcExpTab, glibc::kGlibcLogTab))
        bm[((size_t)c * 2 + par) * nwords + (slot >> 6)] |= 1ull << (slot & 63);
  }
  std::vector<int64_t> starts(P + 1);
  PoolRuns R{(int)pl.run_cls.size(), pl.run_cls.data(), pl.run_len.data()};
  const int64_t end = pool_parse(bm.data(), nwords, d, R, 0, 0, P, starts.data());
  if (end < 0) return -1;
  starts[P] = end;
  for (int64_t e = 0; e < P; ++e) {
    const int64_t s = starts[e];
    for (int j = 0; j < d; ++j) centers[e * d + j] = (uint8_t)(int)(att[j] * pool_unif(raw[s + j]) + 1);
    int64_t pos = s + d;
    int j = 0;
    for (size_t r = 0; r < pl.run_cls.size(); ++r) {
      const PoolClass& C = pl.cls[pl.run_cls[r]];
      for (int t = 0; t < pl.run_len[r]; ++t, ++j) {
        for (;;) {   // next accepted attempt at this parity
          double x = 0.0;
          const bool acc = pool_attempt(C, pool_unif(raw[pos]), pool_unif(raw[pos + 1]), glibc::kGlibcExpTab,
                                        glibc::kGlibcLogTab, &x);
          pos += 2;
          if (acc && !(x > C.thr)) {
            double m0, m1;
            pool_sigma_tables(C, x, att[j], glibc::kGlibcExpTab, glibc::kGlibcLogTab, &sigma[e * d + j], &m0, &m1);
            break;
          }
        }
      }
    }
    if (pos != starts[e + 1]) return -1;
  }
  return end;
}

}  // namespace hdpm
