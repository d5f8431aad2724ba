// phi.hip -- update_phi (code/common_functions.cpp:511-591) on the device.
//
// For every cluster t of the update (ascending labels, cf:535) the reference draws d
// centers -- sample(1:m_j, 1, TRUE, prob) with prob from the cluster's frequency table
// (cf:461-509, 560) -- then d sigmas -- rhig(1, v', w', m_j) (cf:572-589, hyperg.cpp:346-378)
// with v' = v + matches, w' = w + mismatches of the drawn center.  A center draw takes one
// uniform; a sigma draw on rhig's beta path takes 2 uniforms per rbeta attempt, repeated
// while rejected or above (m_j - 1) / m_j.  Where each draw starts therefore depends on every
// earlier rejection -- the serial part of the update.  Here:
//
//   k_phi_prep   one thread per (cluster, attribute): the center probabilities, Rcpp
//                sample's FixupProb / revsort / cumulative sums, the levels the draw can
//                pick and, per pickable level, the sigma's rbeta setup (rhig's branch test
//                decided exactly as the host does, hg:359)
//   k_phi_logits the two stream-only logarithms of an rbeta attempt at every position
//   k_phi_masks  every candidate's acceptance at every drift of a window around the expected
//                drift, as bit masks (one wave = 64 drifts; all items at once)
//   k_phi_cwalk  every cluster walked from every start drift of its window at once (one wave
//                each): the center picks, then the sigma draws 64 at a time by a fixed-point
//                iteration over the masks (each round fixes every lane up to the next
//                rejection) -> the cluster's end drift as a function of its start drift
//   k_phi_chain  the clusters' actual start drifts: T lookups in those functions
//   k_phi_values one wave per cluster: its walk from its actual drift, the accepted attempts'
//                draws, sigma = -1/log(out), the dhamming tables, the bound record
//                (UploadLayout staging for k_scatter_clusters) and the regrouped
//                log-likelihood of the cluster (cf:379-401 as sum_j matches * tab0 +
//                mismatches * tab1)
//
// Every value that decides a draw is the host's bit for bit: IEEE adds, multiplies and
// divides (-ffp-contract=off), glibc's exp / log replicas (glibc_math.hpp), and the branch
// test's Cantelli bounds; its continued-fraction pbeta runs in device libm and an outcome
// within 1e-7 of the threshold is left to the host (kPhiAmbig), as are Walker tables
// (> 200 levels), the bisection path (rare: a center most members do not share) and a drift
// outside the masks' window.  On any status nothing is committed and the host's update
// runs instead, from the same stream position.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"
#include "pool_gen.hpp"

namespace hdpm {

namespace {

__device__ __forceinline__ PoolClass as_pool(const PhiCand& c) {
  PoolClass p;
  p.kind = c.kind;
  p.pad = 0;
  p.aa = c.aa; p.a = c.a; p.b = c.b; p.alpha = c.alpha; p.beta = c.beta; p.gamma = c.gamma;
  p.k1 = c.k1; p.k2 = c.k2; p.thr = c.thr; p.m = c.m;
  return p;
}

__device__ __forceinline__ void set_status(int* st, int code) { atomicMax(st, code); }

// The update's status: plain codes (launch_phi: the status words are zeroed before the call),
// or tagged with the call's generation (launch_phi2: gen << 4 | code, no zeroing; a word of an
// earlier call reads as 0 -- generations only grow, so atomicMax keeps the current call's).
__device__ __forceinline__ void phi_set_status(const PhiArgs& a, int code) {
  atomicMax(a.status, a.gen > 0 ? (a.gen << 4) | code : code);
}
__device__ __forceinline__ int phi_get_status(const PhiArgs& a) {
  const int v = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.gen <= 0) return v;
  return (v >> 4) == a.gen ? (v & 15) : 0;
}


// Serial revsort (R sort.c) on one thread: a[0..n) descending with 1-based levels in ib.
template <class PR, class PM>
__device__ __forceinline__ void phi_revsort_t(PR a0, PM ib0, int n) {
  if (n <= 1) return;
  PR a = a0 - 1;
  PM ib = ib0 - 1;
  int l = (n >> 1) + 1, ir = n, i, j;
  uint8_t ii;
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

// The continued fraction of the incomplete beta (rmath.hpp detail::betacf) and pbeta, in
// device libm: used only for the branch test, with a margin (phi_beta_path).
__device__ __noinline__ double phi_betacf(double a, double b, double x) {
  const double FPMIN = 1e-300, EPS = 1e-16;
  double qab = a + b, qap = a + 1.0, qam = a - 1.0, c = 1.0, d = 1.0 - qab * x / qap;
  if (fabs(d) < FPMIN) d = FPMIN;
  d = 1.0 / d;
  double h = d;
  for (int m = 1; m <= 200000; m++) {
    const int m2 = 2 * m;
    double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
    d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
    c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
    d = 1.0 / d; h *= d * c;
    aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
    d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
    c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
    d = 1.0 / d;
    const double del = d * c;
    h *= del;
    if (fabs(del - 1.0) < EPS) break;
  }
  return h;
}

__device__ __noinline__ double phi_pbeta(double x, double a, double b) {
  if (x <= 0.0) return 0.0;
  if (x >= 1.0) return 1.0;
  const double lbt = lgamma(a + b) - lgamma(a) - lgamma(b) + a * log(x) + b * log1p(-x);
  if (x < (a + 1.0) / (a + b + 2.0)) return exp(lbt) * phi_betacf(a, b, x) / a;
  return 1.0 - exp(lbt) * phi_betacf(b, a, 1.0 - x) / b;
}

// rhig_beta_path (rmath.hpp: qbeta01_lt(w + 1, v - 1, (m - 1) / m) && (m - 1) / m > 4 / 5):
// 1 beta path, 0 bisection, -1 undecided here (pbeta within 1e-7 of 0.1).
__device__ int phi_beta_path(double v, double w, double m) {
  const double x = (m - 1) / m;
  if (!(x > 0)) return 0;                    // (m - 1) / m > 4 / 5 with 4 / 5 == 0 (hg:359)
  const double a = w + 1, b = v - 1;
  if (isnan(a) || isnan(b) || a < 0 || b < 0) return 0;
  if (b == 0) return 0;
  if (a == 0) return x > 0 ? 1 : 0;
  const double mu = a / (a + b);
  const double s2 = a * b / ((a + b) * (a + b) * (a + b + 1.0));
  const double dlt = x - mu;
  const double bound = s2 / (s2 + dlt * dlt);
  if (dlt > 0 && bound < 0.85) return 1;
  if (dlt < 0 && bound < 0.05) return 0;
  const double p = phi_pbeta(x, a, b);
  if (fabs(p - 0.1) < 1e-7) return -1;
  return p > 0.1 ? 1 : 0;
}

// rbeta_setup (rmath.hpp; nmath rbeta's constants) for kinds BB and BC; false otherwise.
__device__ bool phi_rbeta_setup(double aa, double bb, PhiCand* c) {
  if (isnan(aa) || isnan(bb) || aa < 0. || bb < 0.) return false;
  if (isinf(aa) || isinf(bb) || aa == 0. || bb == 0.) return false;
  c->aa = aa;
  c->a = fmin(aa, bb);
  c->b = fmax(aa, bb);
  c->alpha = c->a + c->b;
  c->beta = 0; c->gamma = 0; c->k1 = 0; c->k2 = 0;
  if (c->a <= 1.0) {
    c->kind = 2;
    c->beta = 1.0 / c->a;
    const double delta = 1.0 + c->b - c->a;
    c->k1 = delta * (0.0138889 + 0.0416667 * c->a) / (c->b * c->beta - 0.777778);
    c->k2 = 0.25 + (0.5 + 0.25 / delta) * c->a;
  } else {
    c->kind = 3;
    c->beta = sqrt((c->alpha - 2.0) / (2.0 * c->a * c->b - c->alpha));
    c->gamma = c->a + 1.0 / c->beta;
  }
  return true;
}

// phase marks (HDPM_PHI_TIMING): thread 0 of workgroup `blk` stamps slot q
__device__ __forceinline__ void phi2_mark(const PhiArgs& a, int blk, int q) {
  if (a.tdbg && (int)blockIdx.x == blk && threadIdx.x == 0) a.tdbg[q] = wall_clock64();
}
// (the latest workgroup to reach the mark)
__device__ __forceinline__ void phi2_mark_last(const PhiArgs& a, int q) {
  if (a.tdbg && threadIdx.x == 0) atomicMax(&a.tdbg[q], (unsigned long long)wall_clock64());
}

__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
  const int lane = threadIdx.x & 63;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(x, o);
    if (lane >= o) x += t;
  }
  *total = __shfl(x, 63);
  return x - v;
}

}  // namespace

// One rbeta attempt as pool_attempt (pool_gen.hpp), operation for operation, with the two
// stream-only logarithms read from the per-position tables: lg1 = log(u1 / (1 - u1)) and
// lzz = log(u1 * u1 * u2) (BB; BC's u1 >= 0.5 branch).  BC's other branch forms
// z = u1 * (u1 * u2), which rounds differently, and takes its log here.
__device__ __forceinline__ bool phi_attempt(const PoolClass& C, double u1, double u2, double lg1, double lzz,
                                            const uint64_t* texp, const uint64_t* tlog, double* x) {
  const double expmax = 1024 * 0.693147180559945309417232121458;   // DBL_MAX_EXP * M_LN2
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
    const double t = lzz;
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
  const double lz = u1 < 0.5 ? glibc::log_r(z, tlog) : lzz;
  return alpha * (glibc::log_r(alpha / (a + w), tlog) + v) - 1.3862944 >= lz;
}

// ------------------------------------------------------------------ prep
// Per-thread scratch for the levels of one attribute: LDS when m_j <= kPhiLdsLevels, else
// the global cum / perm rows themselves.
constexpr int kPhiLdsLevels = 16;

// One (cluster, attribute): the center probabilities (as the host's pj_phaseA, cf:496-503),
// sample_prob1_prep (FixupProb, Walker check, revsort, cumulative sums) in pr / pm, the
// candidates per pickable level.  Returns a PhiStatus; *det_out, *nact_out.  Called with LDS
// or global scratch (two copies, so the compiler keeps each address space).
// (nn, lab, sg: the cluster's size and label and the item's current sigma, loaded by the caller)
template <class PR, class PM>
__device__ __forceinline__ int phi_prep_item_in(const PhiArgs& a, int t, int j, int64_t idx, int nn, int lab, double sg,
                                                PR pr, PM pm, const uint64_t* tabs, bool* det_out, int* nact_out,
                                                PhiCand* cpick = nullptr, double ucen = -1.0) {
  const int mj = a.att[j], off = a.aoff[j];
  const unsigned* f = a.freq + ((int64_t)lab * a.d + j) * a.mmax;
  for (int l = 0; l < mj; ++l) pr[l] = (-((double)nn - (double)f[l])) / sg;
  double mx = pr[0];
  for (int l = 1; l < mj; ++l) if (pr[l] > mx) mx = pr[l];
  for (int l = 0; l < mj; ++l) pr[l] = glibc::exp_r(pr[l] - mx, tabs);
  double sum = 0.0;
  for (int l = 0; l < mj; ++l) sum += pr[l];
  for (int l = 0; l < mj; ++l) pr[l] = pr[l] / sum;
  double s2 = 0.0;
  int npos = 0;
  for (int l = 0; l < mj; ++l) {
    const double x = pr[l];
    if (!isfinite(x) || x < 0) return kPhiProb;
    if (x > 0) { npos++; s2 += x; }
  }
  if (npos == 0) return kPhiProb;
  for (int l = 0; l < mj; ++l) pr[l] = pr[l] / s2;
  int nc = 0;
  for (int l = 0; l < mj; ++l) nc += (mj * pr[l] > 0.1);
  if (nc > 200) return kPhiWalker;
  for (int l = 0; l < mj; ++l) pm[l] = (uint8_t)(l + 1);
  phi_revsort_t(pr, pm, mj);
  for (int l = 1; l < mj; ++l) pr[l] += pr[l - 1];
  // the pick is perm[0] whatever the uniform when cum[0] >= 1 (a uniform is < 1); when the
  // center's uniform is known (ucen >= 0: the update's first cluster, whose draws start at
  // drift 0) it is the level that uniform takes (sample_prob1_pick: the first sorted position
  // with u <= cum, the last one otherwise)
  bool det = mj == 1 || pr[0] >= 1.0;
  int sp = 0;
  if (!det && ucen >= 0.0) {
    while (sp < mj - 1 && !(ucen <= pr[sp])) ++sp;
    det = true;
  }
  *det_out = det;
  a.det[idx] = det ? pm[sp] : 0;
  a.ikind[idx] = 0;
  // candidates: the levels the draw can pick (sorted position s: the last, or cum rising)
  PhiCand* cb = a.cand + (int64_t)t * a.sumatt + off;
  int nact = 0;
  for (int s = 0; s < mj; ++s) {
    const int l = pm[s] - 1;
    PhiCand c{};
    c.kind = 0;
    const bool pickable = det ? s == sp : (s == mj - 1 || pr[s] > (s > 0 ? pr[s - 1] : 0.0));
    if (pickable) {
      const double sumdelta = (double)f[l];
      const double nw_ = a.w[j] + nn - sumdelta, nv_ = a.v[j] + sumdelta;
      const double m = (double)mj;
      const int bp = phi_beta_path(nv_, nw_, m);
      if (bp < 0) return kPhiAmbig;
      c.kind = 1;                                   // bisection path (or a degenerate rbeta)
      if (bp == 1 && phi_rbeta_setup(nw_ + 1, nv_ - 1, &c)) {
        c.thr = (m - 1) / m;
        c.m = m;
        nact++;
      }
      if (det) a.ikind[idx] = (uint8_t)c.kind;
    }
    if (cpick && det && s == sp) *cpick = c;        // (the fixed pick's candidate, for the caller)
    cb[l] = c;
  }
  *nact_out = nact;
  return 0;
}
template <class PR, class PM>
__device__ __forceinline__ int phi_prep_item(const PhiArgs& a, int t, int j, int64_t idx, PR pr, PM pm,
                                             const uint64_t* tabs, bool* det_out, int* nact_out) {
  return phi_prep_item_in(a, t, j, idx, a.cnt[t], a.lab[t], a.sig_in[(int64_t)t * a.d + j], pr, pm, tabs, det_out,
                          nact_out);
}

// Prep of the items of workgroup `blk` (tabs: the glibc exp table in LDS).
__device__ __forceinline__ void phi_prep_block(const PhiArgs& a, int blk, const uint64_t* tabs, double* spr,
                                               uint8_t* spm) {
  const int lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blk * blockDim.x + threadIdx.x;
  const bool ok = idx < (int64_t)a.T * a.d;
  const int t = ok ? (int)(idx / a.d) : 0, j = ok ? (int)(idx - (int64_t)t * a.d) : 0;
  int status = 0, nact = 0;
  bool det = false;
  if (ok) {
    const int mj = a.att[j], off = a.aoff[j];
    if (mj <= kPhiLdsLevels) {
      double* pr = spr + threadIdx.x * kPhiLdsLevels;
      uint8_t* pm = spm + threadIdx.x * kPhiLdsLevels;
      status = phi_prep_item(a, t, j, idx, pr, pm, tabs, &det, &nact);
      if (!status) {
        double* gpr = a.cum + (int64_t)t * a.sumatt + off;
        uint8_t* gpm = a.perm + (int64_t)t * a.sumatt + off;
        for (int l = 0; l < mj; ++l) { gpr[l] = pr[l]; gpm[l] = pm[l]; }
      }
    } else {
      status = phi_prep_item(a, t, j, idx, a.cum + (int64_t)t * a.sumatt + off, a.perm + (int64_t)t * a.sumatt + off,
                             tabs, &det, &nact);
    }
  }
  // the composition trees need every pick fixed and on rhig's beta path
  // (a cluster with a pick that depends on the uniform is walked per start drift, k_phi_cwalk,
  // when it fits one walk segment; otherwise the update is re-run by the walks, kPhiNonDet)
  if (ok && !status && a.tree) {
    const int kd = a.ikind[idx];
    if (!det) {
      if (a.S > 1) status = kPhiNonDet;
      else atomicOr(&a.tnd[t], 1);
    } else {
      status = kd == 1 ? kPhiBisect : (kd != 2 && kd != 3) ? kPhiInactive : 0;
    }
  }
  if (status) set_status(a.status, status);
  // the wave's candidates to evaluate, appended with one atomic per wave
  int tot = 0;
  const int before = wave_excl_scan(ok && !status ? nact : 0, &tot);
  int base = 0;
  if (lane == 0 && tot) base = atomicAdd(a.act, tot);
  base = __shfl(base, 0);
  if (ok && !status && nact) {
    const int mj = a.att[j], off = a.aoff[j];
    const PhiCand* cb = a.cand + (int64_t)t * a.sumatt + off;
    int e = base + before;
    for (int l = 0; l < mj; ++l) {
      const int kd = cb[l].kind;
      if (kd != 2 && kd != 3) continue;
      if (e < a.nact_cap) {
        a.act[1 + 2 * e] = (int)((int64_t)t * a.sumatt + off + l);
        a.act[2 + 2 * e] = det ? -1 - (int)idx : (int)idx;     // negative: item-indexed mask row
      } else {
        set_status(a.status, kPhiCap);
      }
      ++e;
    }
  }
}

// ------------------------------------------------------------------ stream logits
// lg[p] = log(u_p / (1 - u_p)) and lzz[p] = log(u_p * u_p * u_(p+1)) over the positions any
// draw of the update can take (the same expressions as rbeta's, rmath.hpp RngSrc / BB).
__device__ __forceinline__ void phi_logits_block(const PhiArgs& a, int blk, int nblk, const uint64_t* tlog) {
  for (int64_t p = (int64_t)blk * blockDim.x + threadIdx.x; p < a.span; p += (int64_t)nblk * blockDim.x) {
    const double u1 = pool_unif(a.raw[p]), u2 = pool_unif(a.raw[p + 1]);
    a.lg[p] = glibc::log_r(u1 / (1.0 - u1), tlog);
    a.lzz[p] = glibc::log_r(u1 * u1 * u2, tlog);
  }
}

// Both in one launch: workgroups [0, nprep) prepare the items, the others compute the logits
// (independent work; one dispatch less on the update's dependency chain).
__global__ __launch_bounds__(256) void k_phi_prep(PhiArgs a, int nprep) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  __shared__ uint64_t tabs[512];
  __shared__ double spr[256 * kPhiLdsLevels];
  __shared__ uint8_t spm[256 * kPhiLdsLevels];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  __syncthreads();
  if ((int)blockIdx.x < nprep) phi_prep_block(a, blockIdx.x, tabs, spr, spm);
  else phi_logits_block(a, blockIdx.x - nprep, gridDim.x - nprep, tabs + 256);
}

// ------------------------------------------------------------------ masks
// mask[cand][q] bit i: the rbeta attempt at drift lo + 64 q + i of the candidate's item is
// accepted with x <= (m - 1) / m (rhig's loop ends there).
__global__ __launch_bounds__(256) void k_phi_masks(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  __shared__ uint64_t tabs[512];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int nact = min(*a.act, (int)a.nact_cap);
  const int64_t total = (int64_t)nact * a.nw;
  const int64_t nwv = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); wv < total; wv += nwv) {
    const int e = (int)(wv / a.nw), q = (int)(wv - (int64_t)e * a.nw);
    const int ci = a.act[1 + 2 * e];
    const int kr = a.act[2 + 2 * e];
    const bool det = kr < 0;
    const int64_t k = det ? -1 - (int64_t)kr : kr;
    const int t = (int)(k / a.d), j = (int)(k - (int64_t)t * a.d);
    const PoolClass C = as_pool(a.cand[ci]);
    const int64_t nominal = (int64_t)t * 3 * a.d + a.d + 2 * (int64_t)j;
    const int64_t pos = nominal + phi_lo(k, a.rate, a.sdev) + 64 * (int64_t)q + lane;
    bool acc = false;
    if (pos < a.span) {
      double x = 0.0;
      acc = phi_attempt(C, pool_unif(a.raw[pos]), pool_unif(a.raw[pos + 1]), a.lg[pos], a.lzz[pos], tabs, tabs + 256,
                        &x) &&
            !(x > C.thr);
    }
    const uint64_t b = __ballot(acc);
    if (lane == 0) (det ? a.maskd + k * a.nw : a.mask + (int64_t)ci * a.nw)[q] = b;
  }
}

// ------------------------------------------------------------------ walks
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Start-drift window of cluster t for the speculative walks.
__device__ __forceinline__ int64_t phi_clo(int t, const PhiArgs& a) { return phi_lo((int64_t)t * a.d, a.rate, a.sdev); }

// LDS image of cluster t for its walks: the mask rows of the items whose pick does not
// depend on the uniform ([d][nw] words), their picks + 1 (det) and kinds.
struct PhiClusterLds {
  const uint64_t* maskd;
  const uint8_t* det;
  const uint8_t* ikind;
};

__device__ __forceinline__ void phi_stage_cluster(const PhiArgs& a, int t, uint64_t* m, uint8_t* det, uint8_t* ik) {
  const int64_t nwd = (int64_t)a.d * a.nw;
  const uint64_t* src = a.maskd + (int64_t)t * nwd;
  for (int64_t q = threadIdx.x; q < nwd; q += blockDim.x) m[q] = src[q];
  for (int j = threadIdx.x; j < a.d; j += blockDim.x) {
    det[j] = a.det[(int64_t)t * a.d + j];
    ik[j] = a.ikind[(int64_t)t * a.d + j];
  }
}

// Cluster t of the update from start drift `delta` (one wave): the d center picks, then
// the d sigma draws 64 at a time.  Lane j's drift is the batch's drift plus the extra
// uniforms of the lanes before it; each round recomputes every lane's extra from its mask
// words at its current drift, and stops when no drift changes (each round fixes every lane
// up to the next rejection).  Returns the end drift, or -1 (a pick outside the candidates
// or a drift outside the masks' windows).  spick: LDS (d bytes); sapos: per attribute the
// accepted attempt's position, or nullptr.
__device__ __forceinline__ int64_t phi_walk_cluster(const PhiArgs& a, const PhiClusterLds& C, int t, int64_t delta,
                                                    uint8_t* spick,
                                    int64_t* sapos, int* why) {
  const int lane = threadIdx.x & 63;
  const int d = a.d;
  const int64_t base = (int64_t)t * 3 * d;
  bool bad = false;
  for (int j = lane; j < d; j += 64) {
    const int dt = C.det[j];
    int pk = 0;
    if (dt) {
      pk = dt - 1;
      const int kd = C.ikind[j];
      if (kd != 2 && kd != 3) { bad = true; *why = kd == 1 ? kPhiBisect : kPhiInactive; }
    } else {
      const int64_t pos = base + delta + j;
      if (pos >= a.span) bad = true;
      else {
        const double rU = pool_unif(a.raw[pos]);
        const int mj = a.att[j];
        const double* cum = a.cum + (int64_t)t * a.sumatt + a.aoff[j];
        int s;
        for (s = 0; s < mj - 1; ++s)
          if (rU <= cum[s]) break;
        pk = a.perm[(int64_t)t * a.sumatt + a.aoff[j] + s] - 1;
        const int kd = a.cand[(int64_t)t * a.sumatt + a.aoff[j] + pk].kind;
        if (kd != 2 && kd != 3) { bad = true; *why = kd == 1 ? kPhiBisect : kPhiInactive; }
      }
    }
    spick[j] = (uint8_t)pk;
  }
  wave_lds_sync();
  if (__ballot(bad)) {
    if (*why == 0) *why = kPhiShort;
    return -1;
  }
  for (int j0 = 0; j0 < d; j0 += 64) {
    const int j = j0 + lane;
    const bool act = j < d;
    const int64_t k = (int64_t)t * d + j;
    // the lane's three mask words from the batch's start drift (a batch drifts < 128)
    uint64_t w0 = 0, w1 = 0, w2 = 0;
    int64_t wlo = 0;
    if (act) {
      const int64_t lo = phi_lo(k, a.rate, a.sdev);
      const int64_t q = delta >= lo ? (delta - lo) >> 6 : -1;
      if (q < 0 || q >= a.nw) bad = true;
      else {
        if (C.det[j]) {                        // LDS image
          const uint64_t* m = C.maskd + (int64_t)j * a.nw;
          w0 = m[q];
          w1 = q + 1 < a.nw ? m[q + 1] : 0ull;
          w2 = q + 2 < a.nw ? m[q + 2] : 0ull;
        } else {                               // global candidate rows
          const uint64_t* m = a.mask + ((int64_t)t * a.sumatt + a.aoff[j] + spick[j]) * a.nw;
          w0 = m[q];
          w1 = q + 1 < a.nw ? m[q + 1] : 0ull;
          w2 = q + 2 < a.nw ? m[q + 2] : 0ull;
        }
        wlo = lo + 64 * q;
      }
    }
    if (__ballot(bad)) { *why = kPhiWindow; return -1; }
    int64_t dl = delta;
    int ex = 0, tot = 0;
    for (;;) {
      ex = 0;
      if (act) {
        int o = (int)(dl - wlo);
        ex = -1;
        for (int r = 0; o < 192; ++r, o += 2) {
          const uint64_t wd = o < 64 ? w0 : o < 128 ? w1 : w2;
          if ((wd >> (o & 63)) & 1ull) { ex = 2 * r; break; }
        }
        if (ex < 0) { bad = true; ex = 0; }
      }
      if (__ballot(bad)) { *why = kPhiWindow; return -1; }
      const int before = wave_excl_scan(ex, &tot);
      const int64_t nd = delta + before;
      const bool changed = act && nd != dl;
      dl = nd;
      if (!__ballot(changed)) break;
    }
    if (act && sapos) sapos[j] = base + d + 2 * (int64_t)j + dl + ex;   // the accepted attempt
    delta += tot;
  }
  return delta;
}

// LDS of the cluster image: d nw mask words, d det bytes, d kind bytes (16-B aligned)
__host__ __device__ inline size_t phi_cluster_lds(int d, int nw) {
  return ((size_t)d * nw * 8 + 2 * (size_t)d + 15) & ~(size_t)15;
}

// Every walk segment from every start drift of its window: F[t S + s][c] = the drift after
// items [s L, (s + 1) L) of cluster t from phi_lo(t d + s L) + c.  The walks are independent:
// a thread carries kPhiIlp start drifts through the segment's sigma draws at once (each draw
// a lookup in the item's mask row; independent chains hide the LDS latency).  A workgroup
// stages its cluster's image in LDS: the mask rows of the items whose pick does not depend on
// the uniform, and each item's window start.  The others' picks depend on the cluster's
// start drift: drawn per thread from the stream (segment 0 only -- a later segment's start
// drift is not the cluster's; such a cluster sets kPhiWindow and the host updates).
constexpr int kPhiIlp = 4;

__host__ __device__ inline size_t phi_cwalk_image(int d, int nw) {
  return phi_cluster_lds(d, nw) + (((size_t)d * 4 + 4 + 15) & ~(size_t)15);
}

__global__ __launch_bounds__(1024) void k_phi_cwalk(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  extern __shared__ __attribute__((aligned(16))) uint8_t wl[];
  if (*a.status != 0) return;
  const int d = a.d, nw = a.nw;
  const int ts = blockIdx.x / a.groups, g = blockIdx.x - ts * a.groups;
  const int t = ts / a.S, sg = ts - t * a.S;
  // tree mode: only the clusters with a pick that depends on the uniform (one segment)
  if (a.tree && !a.tnd[t]) return;
  const int j0 = sg * a.L, j1 = min(d, j0 + a.L);
  uint64_t* m = reinterpret_cast<uint64_t*>(wl);
  uint8_t* det = wl + (size_t)d * nw * 8;
  uint8_t* ik = det + d;
  int* slo = reinterpret_cast<int*>(wl + phi_cluster_lds(d, nw));
  int* nd = slo + d;                       // [0]: uniform-dependent picks in the segment, -1: none possible
  phi_stage_cluster(a, t, m, det, ik);
  for (int j = threadIdx.x; j < d; j += blockDim.x) slo[j] = (int)phi_lo((int64_t)t * d + j, a.rate, a.sdev);
  __syncthreads();
  if (threadIdx.x == 0) {
    int cnt = 0;                           // -1: a fixed pick whose sigma the device does not draw
    for (int j = j0; j < j1 && cnt >= 0; ++j)
      if (det[j] && ik[j] != 2 && ik[j] != 3) cnt = -1;
      else if (!det[j]) cnt = sg == 0 ? cnt + 1 : -1;
    nd[0] = cnt;
  }
  __syncthreads();
  const int cstep = a.groups * blockDim.x;
  const int c0 = g * blockDim.x + threadIdx.x;
  uint16_t* root = a.tree ? a.tree + ((int64_t)t * a.tpc + phi_loff(a.tnb, phi_ltop(a.tnb))) * a.tW : nullptr;
  if (root && g == 0)                      // start drifts past the walks' window
    for (int c = a.Wc + threadIdx.x; c < a.tW; c += blockDim.x) root[c] = kPhiBad;
  if (c0 >= a.Wc) return;
  const int64_t clo = phi_lo((int64_t)t * d + j0, a.rate, a.sdev);
  int64_t dt0[kPhiIlp], delta[kPhiIlp];
  int code[kPhiIlp];
  const bool img = nd[0] >= 0;
#pragma unroll
  for (int u = 0; u < kPhiIlp; ++u) {
    const int c = c0 + u * cstep;
    dt0[u] = clo + c;
    delta[u] = dt0[u];
    code[u] = c < a.Wc ? (img ? 0 : -2) : -6;     // -2 image, -3 pick, -4 window, -5 rejections, -6 unused
  }
  const int64_t base = (int64_t)t * 3 * d;
  if (img && nd[0] == 0) {
    // every pick of the segment is fixed: a branch-free walk, the chains' LDS reads in flight
    // together (a chain that leaves its window or runs out of attempts keeps walking a clamped
    // row and is marked)
    const unsigned lim = 64u * (unsigned)(nw - 1);
    int dl[kPhiIlp];
#pragma unroll
    for (int u = 0; u < kPhiIlp; ++u) dl[u] = (int)delta[u];
    for (int j = j0; j < j1; ++j) {
      const int sl = slo[j];
      const uint64_t* row = m + (size_t)j * nw;
      uint64_t lo[kPhiIlp], hi[kPhiIlp];
      int sh[kPhiIlp];
      bool bad[kPhiIlp];
#pragma unroll
      for (int u = 0; u < kPhiIlp; ++u) {
        const int off = dl[u] - sl;
        bad[u] = (unsigned)off >= lim;
        const int q = bad[u] ? 0 : off >> 6;
        sh[u] = off & 63;
        lo[u] = row[q];
        hi[u] = row[q + 1];
      }
#pragma unroll
      for (int u = 0; u < kPhiIlp; ++u) {
        const uint64_t win = sh[u] ? (lo[u] >> sh[u]) | (hi[u] << (64 - sh[u])) : lo[u];
        const uint64_t acc = win & 0x5555555555555555ull;
        const int ncode = bad[u] ? -4 : (acc ? 0 : -5);
        code[u] = code[u] ? code[u] : ncode;
        dl[u] += acc ? __builtin_ctzll(acc) : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < kPhiIlp; ++u) delta[u] = dl[u];
  } else {
  for (int j = j0; j < j1; ++j) {
    const int sl = slo[j];
    const bool dj = det[j] != 0;
    uint64_t lo[kPhiIlp], hi[kPhiIlp];
    int sh[kPhiIlp];
    bool live = false;
#pragma unroll
    for (int u = 0; u < kPhiIlp; ++u) {
      lo[u] = 0; hi[u] = 0; sh[u] = 0;
      if (code[u] != 0) continue;
      const int64_t off = delta[u] - sl;
      if (off < 0 || off >= 64 * (nw - 1)) { code[u] = -4; continue; }
      const int q = (int)(off >> 6);
      sh[u] = (int)(off & 63);
      if (dj) {
        lo[u] = m[(int64_t)j * nw + q];        // LDS
        hi[u] = m[(int64_t)j * nw + q + 1];
      } else {
        // a pick that depends on the uniform (cf:560 at this start drift): drawn here
        const int64_t pos = base + dt0[u] + j;
        if (pos >= a.span) { code[u] = -3; continue; }
        const double rU = pool_unif(a.raw[pos]);
        const int mj = a.att[j];
        const double* cum = a.cum + (int64_t)t * a.sumatt + a.aoff[j];
        int s;
        for (s = 0; s < mj - 1; ++s)
          if (rU <= cum[s]) break;
        const int64_t ci = (int64_t)t * a.sumatt + a.aoff[j] + a.perm[(int64_t)t * a.sumatt + a.aoff[j] + s] - 1;
        const int kd = a.cand[ci].kind;
        if (kd != 2 && kd != 3) { code[u] = -3; continue; }
        lo[u] = a.mask[ci * nw + q];
        hi[u] = a.mask[ci * nw + q + 1];
      }
      live = true;
    }
    if (!live) break;
#pragma unroll
    for (int u = 0; u < kPhiIlp; ++u) {
      if (code[u] != 0) continue;
      const uint64_t win = sh[u] ? (lo[u] >> sh[u]) | (hi[u] << (64 - sh[u])) : lo[u];
      const uint64_t acc = win & 0x5555555555555555ull;
      if (!acc) { code[u] = -5; continue; }
      delta[u] += __builtin_ctzll(acc);
    }
  }
  }
#pragma unroll
  for (int u = 0; u < kPhiIlp; ++u) {
    const int c = c0 + u * cstep;
    if (c >= a.Wc) continue;
    if (root)                              // tree mode: the cluster's root table (extra uniforms)
      root[c] = code[u] == 0 && delta[u] - dt0[u] < (int64_t)kPhiBad ? (uint16_t)(delta[u] - dt0[u]) : kPhiBad;
    else
      a.F[(int64_t)ts * a.Wc + c] = code[u] == 0 && delta[u] <= 0x7fffffff ? (int)delta[u] : (code[u] ? code[u] : -1);
  }
}

// One walk segment of cluster t from drift `delta` by one thread, from global memory (a
// segment after the first whose picks depend on the uniform, i.e. on the cluster's start
// drift dt, which its table cannot index): the end drift, or < 0.
__device__ int64_t phi_walk_serial(const PhiArgs& a, int t, int j0, int j1, int64_t dt, int64_t delta) {
  const int d = a.d, nw = a.nw;
  const int64_t base = (int64_t)t * 3 * d;
  for (int j = j0; j < j1; ++j) {
    const int64_t off = delta - phi_lo((int64_t)t * d + j, a.rate, a.sdev);
    if (off < 0 || off >= 64 * (int64_t)(nw - 1)) return -4;
    const int q = (int)(off >> 6), sh = (int)(off & 63);
    const uint64_t* row;
    if (a.det[(int64_t)t * d + j]) {
      const int kd = a.ikind[(int64_t)t * d + j];
      if (kd != 2 && kd != 3) return -3;
      row = a.maskd + ((int64_t)t * d + j) * nw;
    } else {
      const int64_t pos = base + dt + j;
      if (pos >= a.span) return -3;
      const double rU = pool_unif(a.raw[pos]);
      const int64_t cb = (int64_t)t * a.sumatt + a.aoff[j];
      int s;
      for (s = 0; s < a.att[j] - 1; ++s)
        if (rU <= a.cum[cb + s]) break;
      const int64_t ci = cb + a.perm[cb + s] - 1;
      const int kd = a.cand[ci].kind;
      if (kd != 2 && kd != 3) return -3;
      row = a.mask + ci * nw;
    }
    const uint64_t lo = row[q], hi = row[q + 1];
    const uint64_t win = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    const uint64_t acc = win & 0x5555555555555555ull;
    if (!acc) return -5;
    delta += __builtin_ctzll(acc);
  }
  return delta;
}

// The segments' actual start drifts: delta_0 = 0, delta after segment (t, s) =
// F[t S + s][delta - phi_lo(t d + s L)] (the table staged in LDS when it fits, many loads in
// flight per thread); dts[t] = cluster t's start drift.
__global__ __launch_bounds__(1024) void k_phi_chain(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  extern __shared__ int sF[];
  if (*a.status != 0) return;
  const int64_t nF = (int64_t)a.T * a.S * a.Wc;
  const bool lds = nF <= 16384;
  if (lds) {
    constexpr int U = 16;
    for (int64_t q0 = (int64_t)threadIdx.x; q0 < nF; q0 += (int64_t)U * blockDim.x) {
      int v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + (int64_t)u * blockDim.x;
        v[u] = q < nF ? a.F[q] : 0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + (int64_t)u * blockDim.x;
        if (q < nF) sF[q] = v[u];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const int* F = lds ? sF : a.F;
  int64_t delta = 0;
  for (int t = 0; t < a.T; ++t) {
    a.dts[t] = delta;
    for (int sg = 0; sg < a.S; ++sg) {
      const int64_t c = delta - phi_lo((int64_t)t * a.d + (int64_t)sg * a.L, a.rate, a.sdev);
      if (c < 0 || c >= a.Wc) { set_status(a.status, kPhiWindow); return; }
      int64_t e = F[((int64_t)t * a.S + sg) * a.Wc + c];
      if (e == -2 && sg > 0) e = phi_walk_serial(a, t, sg * a.L, min(a.d, (sg + 1) * a.L), a.dts[t], delta);
      if (e < 0) { set_status(a.status, kPhiWindow); return; }
      delta = e;
    }
  }
  const int64_t cons = (int64_t)a.T * 3 * a.d + delta;
  if (cons + 1 > a.span) set_status(a.status, kPhiShort);
  *(int64_t*)(a.status + 2) = cons;
  if (a.pos_out) *a.pos_out = *a.pos_in + a.sweep_len + cons;
}

// ------------------------------------------------------------------ values
// One workgroup per cluster: wave 0 walks it again from its actual drift (picks and accepted
// positions into LDS); then every wave takes attributes: the accepted attempts' draws,
// sigma = -1/log(out), the dhamming tables; then the bound record (wave w: plane word w) and
// the regrouped log-likelihood terms.  LDS: the cluster image, picks, positions, per
// attribute (sigma, match, mismatch), per thread the partial sums.
// The values of cluster t once its picks (spick) and accepted attempts' positions (sapos)
// are known: every wave takes attributes -- the accepted attempts' draws, sigma = -1/log(out),
// the dhamming tables -- then the bound record (wave w: plane word w) and the regrouped
// log-likelihood terms.  wtab: LDS [d][2]; red: LDS [64]; wmx, wmn: LDS [16]; sbad: LDS flag
// (0 on entry).  Called by every thread of the workgroup.
__device__ __forceinline__ void phi_values_body(const PhiArgs& a, int t, const uint8_t* spick, const int64_t* sapos, double* wtab,
                                const uint64_t* texp, const uint64_t* tlog, double* red, double* wmx, double* wmn,
                                int* sbad, const int* lab_cnt = nullptr) {
  // (lab_cnt: a device copy of the labels then the counts, else a.lab / a.cnt)
  const int* labs = lab_cnt ? lab_cnt : a.lab;
  const int* cnts = lab_cnt ? lab_cnt + a.T : a.cnt;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nth = blockDim.x;
  const int d = a.d;
  const UploadLayout L = upload_layout(a.T, a.dp, d, a.bw);
  uint8_t* codes = a.stage + L.off_codes + (size_t)t * a.dp;
  double* tab = reinterpret_cast<double*>(a.stage + L.off_tab) + (size_t)t * 2 * d;
  uint64_t* rec = reinterpret_cast<uint64_t*>(a.stage + L.off_bnd) + (size_t)t * a.bw;
  const int nn = cnts[t];
  const unsigned* fb = a.freq + (int64_t)labs[t] * d * a.mmax;
  double hi = 0.0, lo = 0.0;                     // regrouped log-likelihood terms (Neumaier)
  auto add = [&](double x) {
    const double s = hi + x;
    lo += fabs(hi) >= fabs(x) ? (hi - s) + x : (x - s) + hi;
    hi = s;
  };
  double A = 0.0, sc = 0.0, dmx = 0.0, dmn = __builtin_inf();
  bool bad = false;
  for (int j = threadIdx.x; j < a.dp; j += nth) {
    if (j >= d) { codes[j] = 0; continue; }
    const int64_t k = (int64_t)t * d + j;
    const int pk = spick[j];
    const PoolClass C = as_pool(a.cand[(int64_t)t * a.sumatt + a.aoff[j] + pk]);
    const int64_t p = sapos[j];
    double x = 0.0;
    if (!(p + 1 < a.span)) {
      bad = true;
    } else {
      const double u1 = pool_unif(a.raw[p]), u2 = pool_unif(a.raw[p + 1]);
      // the stream logits from the tables, or (launch_phi2: no tables) the same expressions here
      const double lg1 = a.lg ? a.lg[p] : glibc::log_r(u1 / (1.0 - u1), tlog);
      const double lzz = a.lzz ? a.lzz[p] : glibc::log_r(u1 * u1 * u2, tlog);
      if (!phi_attempt(C, u1, u2, lg1, lzz, texp, tlog, &x) || x > C.thr) bad = true;
    }
    double sg, m0, m1;
    pool_sigma_tables(C, x, a.att[j], texp, tlog, &sg, &m0, &m1);
    codes[j] = (uint8_t)(pk + 1);
    a.pick[k] = (uint8_t)pk;
    wtab[2 * j] = m0;
    wtab[2 * j + 1] = m1;
    tab[2 * j] = m0;
    tab[2 * j + 1] = m1;
    a.sig_out[k] = sg;
    if (a.sig_dev) a.sig_dev[k] = sg;
    A += m0;
    sc += fmax(fabs(m0), fabs(m1));
    const double dj = m0 - m1;
    dmx = fmax(dmx, dj);
    dmn = fmin(dmn, dj);
    const double fm = (double)fb[(int64_t)j * a.mmax + pk];
    add(fm * m0);
    add(((double)nn - fm) * m1);
  }
  if (bad) atomicOr(sbad, 1);
  phi2_mark(a, 0, 16);
  // per wave: A and scale summed (any order: only the bound's slack sees their rounding),
  // the log-likelihood pairs in lane order
  {
    // the lanes' (hi, lo) pairs by a butterfly of error-free sums (TwoSum: the exact rounding
    // error whatever the order, so every lane ends with the same pair)
    double H = hi, Lo = lo;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double x = __shfl_xor(H, o), y = __shfl_xor(Lo, o);
      const double s = H + x, bb = s - H;
      const double err = (H - (s - bb)) + (x - bb);
      H = s;
      Lo = (Lo + y) + err;
      A += __shfl_xor(A, o);
      sc += __shfl_xor(sc, o);
    }
    if (lane == 0) {
      red[wid] = A;
      red[16 + wid] = sc;
      red[32 + wid] = H;
      red[48 + wid] = Lo;
    }
  }
  __syncthreads();
  if (*sbad) {
    if (threadIdx.x == 0) phi_set_status(a, kPhiWindow);
    return;
  }
  // the block's sums: A, scale (any order: only the bound's slack sees their rounding),
  // dmax, dmin; the log-likelihood pairs in thread order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dmx = fmax(dmx, __shfl_xor(dmx, o));
    dmn = fmin(dmn, __shfl_xor(dmn, o));
  }
  if (lane == 0) { wmx[wid] = dmx; wmn[wid] = dmn; }
  __syncthreads();
  dmx = 0.0;
  dmn = __builtin_inf();
  for (int q = 0; q < nth / 64; ++q) { dmx = fmax(dmx, wmx[q]); dmn = fmin(dmn, wmn[q]); }
  const double delta = dmx > 0 ? dmx / ((1 << kQ) - 1) : 0.0;
  phi2_mark(a, 0, 17);
  // bound record (Ctx::bounds_for, kernels.hpp "Bound data per parameter entry"): wave w
  // builds plane word w
  for (int k = wid; k < a.Ws; k += nth / 64) {
    const int j = 64 * k + lane;
    const bool valid = j < d;
    const unsigned code = valid ? spick[j] : 0u;
    int q = 0;
    if (valid) {
      const double dj = wtab[2 * j] - wtab[2 * j + 1];
      q = delta > 0 ? (int)floor(dj / delta) : 0;
      q = min(max(q, 0), (1 << kQ) - 1);
      while (q > 0 && delta * q > dj) --q;
      while (q < (1 << kQ) - 1 && delta * (q + 1) <= dj) ++q;
    }
    for (int b = 0; b < a.wb; ++b) {
      const uint64_t bits = __ballot(valid && ((code >> b) & 1u));
      if (lane == 0) rec[b * a.Ws + k] = bits;
    }
    for (int b = 0; b < kQ; ++b) {
      const uint64_t bits = __ballot(valid && ((q >> b) & 1));
      if (lane == 0) rec[(a.wb + b) * a.Ws + k] = bits;
    }
  }
  phi2_mark(a, 0, 18);
  if (threadIdx.x == 0) {
    double As = 0.0, scs = 0.0, H = 0.0, Lo = 0.0;
    for (int q = 0; q < nth / 64; ++q) {
      As += red[q];
      scs += red[16 + q];
      const double x = red[32 + q];
      const double s = H + x;
      Lo += fabs(H) >= fabs(x) ? (H - s) + x : (x - s) + H;
      H = s;
      Lo += red[48 + q];
    }
    double* sv = reinterpret_cast<double*>(rec + (a.wb + kQ) * a.Ws);
    sv[0] = As;
    sv[1] = delta;
    sv[2] = dmn > 0 ? dmn : 0.0;
    sv[3] = scs;
    reinterpret_cast<int*>(a.stage + L.off_counts)[t] = nn;
    reinterpret_cast<int*>(a.stage + L.off_slot)[t] = a.slot_of ? a.slot_of[t] : labs[t];
    a.ll[2 * t] = H;
    a.ll[2 * t + 1] = Lo;
  }
}

// One workgroup per cluster: wave 0 walks it again from its actual drift (picks and accepted
// positions into LDS), then phi_values_body.  LDS: the cluster image, picks, positions, per
// attribute (sigma, match, mismatch), per thread the partial sums.
__global__ __launch_bounds__(1024) void k_phi_values(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  extern __shared__ __attribute__((aligned(16))) uint8_t wl[];
  __shared__ uint64_t tabs[512];
  __shared__ double red[4 * 16];
  __shared__ double wmx[16], wmn[16];
  __shared__ int sbad;
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  if (threadIdx.x == 0) sbad = 0;
  if (*a.status != 0) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int t = blockIdx.x;
  const int d = a.d;
  uint64_t* m = reinterpret_cast<uint64_t*>(wl);
  uint8_t* det = wl + (size_t)d * a.nw * 8;
  uint8_t* ik = det + d;
  phi_stage_cluster(a, t, m, det, ik);
  double* wtab = reinterpret_cast<double*>(wl + phi_cluster_lds(d, a.nw));   // [d][2]
  int64_t* sapos = reinterpret_cast<int64_t*>(wtab + 2 * d);
  uint8_t* spick = reinterpret_cast<uint8_t*>(sapos + d);
  __syncthreads();
  if (wid == 0) {
    int why = 0;
    const PhiClusterLds C{m, det, ik};
    if (phi_walk_cluster(a, C, t, a.dts[t], spick, sapos, &why) < 0 && lane == 0) {
      set_status(a.status, why ? why : kPhiWindow);
      sbad = 1;
    }
  }
  __syncthreads();
  if (sbad) return;
  phi_values_body(a, t, spick, sapos, wtab, tabs, tabs + 256, red, wmx, wmn, &sbad);
}

// ------------------------------------------------------------------ composition trees
// When every pick of the update is fixed (k_phi_prep, tree mode), item k's sigma draw is a
// function of the drift alone: f_k(delta) = delta + 2 r with r the attempts its mask rejects
// from delta on.  The update's drift is f_{T d - 1} o ... o f_0 (0), T d dependent steps; a
// tree of compositions has log2(d) levels of independent table lookups instead.  A table holds
// the extra uniforms its node consumes from each of tW start drifts phi_lo(first item) + c.

// One item's step from drift e (mask row in `row`, window start `lo`): false outside the
// windows or with no acceptance in the 32 attempts the two mask words hold.
__device__ __forceinline__ bool phi_tree_step(const uint64_t* row, int lo, int W, int* e) {
  const int off = *e - lo;
  if ((unsigned)off >= (unsigned)W) return false;
  const int q = off >> 6, sh = off & 63;
  const uint64_t w0 = row[q], w1 = row[q + 1];
  const uint64_t win = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  const uint64_t acc = win & 0x5555555555555555ull;
  if (!acc) return false;
  *e += __builtin_ctzll(acc);
  return true;
}

// (left then right) at start offset c of the left table: the composed extra, or kPhiBad
__device__ __forceinline__ uint16_t phi_tree_compose(const uint16_t* L, const uint16_t* R, int lo_l, int lo_r, int W,
                                                     int c) {
  const uint16_t v = L[c];
  if (v == kPhiBad) return kPhiBad;
  const int cr = lo_l + c + v - lo_r;
  if ((unsigned)cr >= (unsigned)W) return kPhiBad;
  const uint16_t r = R[cr];
  if (r == kPhiBad || (int)v + (int)r >= (int)kPhiBad) return kPhiBad;
  return (uint16_t)(v + r);
}

__host__ __device__ inline size_t phi_tree_lds(int SB, int nw, int W) {
  return align16((size_t)4 * SB * nw * 8) + align16((size_t)4 * SB * 4) + align16((size_t)2 * SB * W * 2);
}

// Workgroup (t, s): level-0 tables of blocks [s SB, s SB + SB) of cluster t (each from the
// item masks staged in LDS: a 4-item walk per start drift), then levels 1 .. log2(SB) of that
// segment (compositions in LDS); every table also goes to a.tree.
__global__ __launch_bounds__(1024) void k_phi_tree(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  if (*a.status != 0) return;
  const int S = a.tS, SB = a.tSB, nb = a.tnb, W = a.tW, nw = a.nw, d = a.d;
  const int t = blockIdx.x / S, s = blockIdx.x - t * S;
  if (a.tnd[t]) return;                              // walked per start drift (k_phi_cwalk)
  const int b0 = s * SB, nblk = min(nb - b0, SB);
  const int j0 = 4 * b0, nit = min(d, 4 * (b0 + nblk)) - j0;
  uint64_t* M = reinterpret_cast<uint64_t*>(sm);
  int* slo = reinterpret_cast<int*>(sm + align16((size_t)4 * SB * nw * 8));
  uint16_t* A = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(slo) + align16((size_t)4 * SB * 4));
  {
    const uint64_t* src = a.maskd + ((int64_t)t * d + j0) * nw;
    for (int q = threadIdx.x; q < nit * nw; q += blockDim.x) M[q] = src[q];
    for (int j = threadIdx.x; j < nit; j += blockDim.x) slo[j] = (int)phi_lo((int64_t)t * d + j0 + j, a.rate, a.sdev);
  }
  __syncthreads();
  uint16_t* G = a.tree + (int64_t)t * a.tpc * W;
  for (int idx = threadIdx.x; idx < nblk * W; idx += blockDim.x) {
    const int b = idx / W, c = idx - b * W;
    const int jb = 4 * b, je = min(nit, jb + 4);
    const int start = slo[jb] + c;
    int e = start;
    bool ok = true;
    for (int j = jb; j < je && ok; ++j) ok = phi_tree_step(M + (size_t)j * nw, slo[j], W, &e);
    const uint16_t v = ok && e - start < (int)kPhiBad ? (uint16_t)(e - start) : kPhiBad;
    A[idx] = v;
    G[(int64_t)(b0 + b) * W + c] = v;
  }
  const int ltop = phi_ltop(nb);
  int np = nblk;                                     // nodes of the segment at the level below
  // level l's tables at A + (l & 1) SB W (offsets from one LDS base: no pointer swaps)
  for (int l = 1; l <= ltop && (1 << l) <= SB; ++l) {
    __syncthreads();
    const uint16_t* cur = A + (size_t)((l - 1) & 1) * SB * W;
    uint16_t* nxt = A + (size_t)(l & 1) * SB * W;
    const int nl = (np + 1) / 2;
    const int off = phi_loff(nb, l) + (b0 >> l);
    for (int idx = threadIdx.x; idx < nl * W; idx += blockDim.x) {
      const int li = idx / W, c = idx - li * W;
      const uint16_t* Lt = cur + (size_t)(2 * li) * W;
      uint16_t v;
      if (2 * li + 1 < np) {
        const int jl = 4 * ((2 * li) << (l - 1)), jr = 4 * ((2 * li + 1) << (l - 1));
        v = phi_tree_compose(Lt, cur + (size_t)(2 * li + 1) * W, slo[jl], slo[jr], W, c);
      } else {
        v = Lt[c];
      }
      nxt[(size_t)li * W + c] = v;
      G[(int64_t)(off + li) * W + c] = v;
    }
    np = nl;
  }
}

// Levels above the segments (tS > 1): one workgroup per cluster composes them in a.tree.
__global__ __launch_bounds__(1024) void k_phi_tree_top(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (*a.status != 0) return;
  const int nb = a.tnb, W = a.tW, d = a.d, t = blockIdx.x;
  if (a.tnd[t]) return;
  int lseg = 0;
  while ((1 << lseg) < a.tSB) ++lseg;
  const int ltop = phi_ltop(nb);
  uint16_t* G = a.tree + (int64_t)t * a.tpc * W;
  for (int l = lseg + 1; l <= ltop; ++l) {
    const int np = phi_lcount(nb, l - 1), nl = phi_lcount(nb, l);
    const uint16_t* P = G + (int64_t)phi_loff(nb, l - 1) * W;
    uint16_t* Q = G + (int64_t)phi_loff(nb, l) * W;
    for (int idx = threadIdx.x; idx < nl * W; idx += blockDim.x) {
      const int i = idx / W, c = idx - i * W;
      const uint16_t* Lt = P + (size_t)(2 * i) * W;
      uint16_t v;
      if (2 * i + 1 < np) {
        const int jl = 4 * ((2 * i) << (l - 1)), jr = 4 * ((2 * i + 1) << (l - 1));
        v = phi_tree_compose(Lt, P + (size_t)(2 * i + 1) * W, (int)phi_lo((int64_t)t * d + jl, a.rate, a.sdev),
                             (int)phi_lo((int64_t)t * d + jr, a.rate, a.sdev), W, c);
      } else {
        v = Lt[c];
      }
      Q[(size_t)i * W + c] = v;
    }
    __syncthreads();
  }
}

__host__ __device__ inline size_t phi_values2_lds(int d, int nb, int T, int W, int nw) {
  // (the roots of the clusters before each are always staged in LDS; then the cluster image
  // of a cluster walked per start drift)
  return align16((size_t)2 * d * 8) + align16((size_t)d * 8) + align16((size_t)d) + align16((size_t)2 * nb * 4 + 8) +
         align16((size_t)T * W * 2) + phi_cluster_lds(d, nw);
}

// One workgroup per cluster t of a tree-mode update: its start drift (the root tables of the
// clusters before it, composed from drift 0), the start drift of every tree node down to the
// level-0 blocks (one lookup per node and level), each block's 4 items walked from its start
// (picks fixed: det), then phi_values_body.  The last cluster also writes the consumption.
__global__ __launch_bounds__(1024) void k_phi_values2(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  extern __shared__ __attribute__((aligned(16))) uint8_t wl[];
  __shared__ uint64_t tabs[512];
  __shared__ double red[4 * 16];
  __shared__ double wmx[16], wmn[16];
  __shared__ int sbad;
  __shared__ int sdt;
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  if (threadIdx.x == 0) sbad = 0;
  if (*a.status != 0) return;
  const int t = blockIdx.x, d = a.d, W = a.tW, nb = a.tnb, nw = a.nw;
  double* wtab = reinterpret_cast<double*>(wl);
  int64_t* sapos = reinterpret_cast<int64_t*>(wl + align16((size_t)2 * d * 8));
  uint8_t* spick = reinterpret_cast<uint8_t*>(sapos) + align16((size_t)d * 8);
  int* st = reinterpret_cast<int*>(spick + align16((size_t)d));     // node starts: two levels
  uint16_t* R = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(st) + align16((size_t)2 * nb * 4 + 8));
  uint8_t* img = reinterpret_cast<uint8_t*>(R) + align16((size_t)a.T * W * 2);   // cluster image (non-det)
  const int ltop = phi_ltop(nb);
  const int64_t rootoff = (int64_t)phi_loff(nb, ltop) * W;
  // the start drift of cluster t: the clusters before it from drift 0 (their roots in LDS)
  for (int q = threadIdx.x; q < t * W; q += blockDim.x) {
    const int u = q / W, c = q - u * W;
    R[q] = a.tree[(int64_t)u * a.tpc * W + rootoff + c];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int e = 0;
    bool ok = true;
    for (int u = 0; u < t && ok; ++u) {
      const int c = e - (int)phi_lo((int64_t)u * d, a.rate, a.sdev);
      if ((unsigned)c >= (unsigned)W) { ok = false; break; }
      const uint16_t v = R[(size_t)u * W + c];
      if (v == kPhiBad) ok = false;
      else e += v;
    }
    sdt = ok ? e : -1;
    if (!ok) sbad = 1;
    else a.dts[t] = e;
  }
  __syncthreads();
  if (sbad) {
    if (threadIdx.x == 0) set_status(a.status, kPhiWindow);
    return;
  }
  const uint16_t* G = a.tree + (int64_t)a.tpc * W * t;
  if (a.tnd[t]) {
    // a pick depends on the uniform: one wave walks the cluster from its start drift
    uint64_t* m = reinterpret_cast<uint64_t*>(img);
    uint8_t* det = img + (size_t)d * nw * 8;
    uint8_t* ik = det + d;
    phi_stage_cluster(a, t, m, det, ik);
    __syncthreads();
    if ((threadIdx.x >> 6) == 0) {
      int why = 0;
      const PhiClusterLds C{m, det, ik};
      if (phi_walk_cluster(a, C, t, sdt, spick, sapos, &why) < 0 && (threadIdx.x & 63) == 0) {
        set_status(a.status, why ? why : kPhiWindow);
        sbad = 1;
      }
    }
    __syncthreads();
    if (sbad) return;
  } else {
  // node starts, from the root down (ping-pong between the two halves of st)
  // level l's node starts at st + ((ltop - l) & 1) nb (offsets from one LDS base)
  if (threadIdx.x == 0) st[0] = sdt;
  __syncthreads();
  for (int l = ltop; l >= 1; --l) {
    const int* cur = st + ((ltop - l) & 1) * nb;
    int* nxt = st + ((ltop - l + 1) & 1) * nb;
    const int nc = phi_lcount(nb, l - 1);
    const uint16_t* Lv = G + (int64_t)phi_loff(nb, l - 1) * W;
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
      int sv = cur[i >> 1];
      if ((i & 1) && sv >= 0) {
        // right child: after its left sibling's items
        const int jl = 4 * ((i - 1) << (l - 1));
        const int c = sv - (int)phi_lo((int64_t)t * d + jl, a.rate, a.sdev);
        const uint16_t v = (unsigned)c < (unsigned)W ? Lv[(size_t)(i - 1) * W + c] : kPhiBad;
        sv = v == kPhiBad ? -1 : sv + v;
      }
      nxt[i] = sv;
    }
    __syncthreads();
  }
  const int* cur = st + (ltop & 1) * nb;              // level 0
  // each block's items from its start: the accepted attempt's position and the fixed pick
  const int64_t base = (int64_t)t * 3 * d;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    int e = cur[b];
    bool ok = e >= 0;
    for (int j = 4 * b; j < min(d, 4 * b + 4); ++j) {
      const int64_t k = (int64_t)t * d + j;
      spick[j] = (uint8_t)(a.det[k] - 1);
      if (!ok) continue;
      ok = phi_tree_step(a.maskd + k * nw, (int)phi_lo(k, a.rate, a.sdev), W, &e);
      // the accepted attempt: nominal position + drift before the item + the rejected attempts
      sapos[j] = base + d + 2 * (int64_t)j + e;
    }
    if (!ok) atomicOr(&sbad, 1);
  }
  __syncthreads();
  if (sbad) {
    if (threadIdx.x == 0) set_status(a.status, kPhiWindow);
    return;
  }
  }
  if (t == a.T - 1 && threadIdx.x == 0) {
    const uint16_t v = (unsigned)(sdt - (int)phi_lo((int64_t)t * d, a.rate, a.sdev)) < (unsigned)W
                           ? G[rootoff + sdt - (int)phi_lo((int64_t)t * d, a.rate, a.sdev)]
                           : kPhiBad;
    if (v == kPhiBad) {
      set_status(a.status, kPhiWindow);
    } else {
      const int64_t cons = (int64_t)a.T * 3 * d + sdt + v;
      if (cons + 1 > a.span) set_status(a.status, kPhiShort);
      *(int64_t*)(a.status + 2) = cons;
      if (a.pos_out) *a.pos_out = *a.pos_in + a.sweep_len + cons;
    }
  }
  phi_values_body(a, t, spick, sapos, wtab, tabs, tabs + 256, red, wmx, wmn, &sbad);
}

// ------------------------------------------------------------------ fast path (launch_phi2)
// The common case of a converged chain: every center pick of the update is fixed (its
// cumulative probability reaches 1 at the first sorted level) and on rhig's beta path, so
// item k's sigma draw is a function of the drift alone, f_k(delta) = delta + 2 (attempts its
// mask rejects from delta on) -- the composition trees of k_phi_tree, laid out for latency:
//
//   k_phi2_group   one workgroup per group of gs consecutive items of a cluster: the items'
//                  preparation (phi_prep_item), the stream logits of the positions the group
//                  can read (in LDS), the items' masks over the window (LDS and maskd), and the
//                  group's table: the extra uniforms of its gs items from each of tW start drifts
//   k_phi2_tree    one workgroup per cluster: its group tables composed in LDS into the
//                  cluster's table (phi2_tree_body).  (Run by the last group workgroup of each
//                  cluster instead, behind a per-cluster arrival counter, it cost ~80 us at C4:
//                  every workgroup's agent-scope release writes back its XCD's L2.)
//   k_phi2_values  one workgroup per cluster: its groups' start drifts (the group tables from
//                  the cluster's start), each group walked by one wave (a lane per item,
//                  fixed-point rounds over the prefetched mask words), then phi_values_body; the
//                  last workgroup writes the status and the consumption for the host
//
// No copies: the labels, counts and sigmas can be read from (coherent) host memory and the
// picks, sigmas and log-likelihood pairs written there; the status words carry the call's
// generation instead of being zeroed.  Any case the fast path does not take (a pick that
// depends on the uniform, the bisection path, an ambiguous branch test, a drift outside the
// windows) is a status, and the caller runs launch_phi or the host job from the same stream
// position; nothing else is committed.

// n uint16 words (a multiple of 8, 16-B aligned at both ends) from global memory into LDS,
// 16 B per load and 4 loads in flight per thread
__device__ __forceinline__ void phi2_stage_u16(uint16_t* dst, const uint16_t* src, int n) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const int n4 = n >> 3, step = blockDim.x;
  for (int q0 = threadIdx.x; q0 < n4; q0 += 4 * step) {
    const int q1 = min(q0 + step, n4 - 1), q2 = min(q0 + 2 * step, n4 - 1), q3 = min(q0 + 3 * step, n4 - 1);
    // (clamped indices: a lane past the end reloads and rewrites the last vector, same value)
    const uint4 v0 = s4[q0], v1 = s4[q1], v2 = s4[q2], v3 = s4[q3];
    d4[q0] = v0;
    d4[q1] = v1;
    d4[q2] = v2;
    d4[q3] = v3;
  }
}


// A chained update's stream slice from its predecessor's end (PhiArgs::chain_in); false: the
// predecessor did not complete or the slice is not inside the window (the update is off).
// Wave-uniform (readfirstlane): the branches on it are scalar.
__device__ __forceinline__ bool phi2_chain(PhiArgs& a) {
  if (!a.chain_in) return true;
  const int ok = __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(&a.chain_in->ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (!ok) return false;
  const uint64_t e = __hip_atomic_load((const uint64_t*)&a.chain_in->end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t elo = __builtin_amdgcn_readfirstlane((uint32_t)e), ehi = __builtin_amdgcn_readfirstlane((uint32_t)(e >> 32));
  const int64_t p = (int64_t)(((uint64_t)ehi << 32) | elo) + a.sweep_len;
  const int64_t r = p - a.win_start;
  if (r < 0 || r + a.span + 1 > a.win_count) return false;
  a.pos0 = p;
  a.raw = a.win_raw + r;
  a.nraw = a.win_count - r;
  a.raw_back = r;
  // the index of p in its block (engine.cpp mti_at)
  const int64_t head = a.win_mti0 >= 624 ? 0 : 624 - a.win_mti0;
  if (r < head) {
    a.mti_pos = a.win_mti0 + (int)r;
  } else {
    const int k = (int)((r - head) % 624);
    a.mti_pos = k == 0 ? 624 : k;
  }
  return true;
}

constexpr int kPhi2MaxG = 512;        // groups per cluster (d <= 4096 at gs = 8)
constexpr int kPhi2MaxT = 1024;       // clusters of one fast-path update

__host__ __device__ inline int phi2_npos(int gs, int nw, double rate) {
  // positions a group can read: 2 (gs - 1) nominal steps, the growth of the window start over
  // the group (<= rate (gs - 1) + 1), 64 nw drifts, the attempt's second uniform
  return 2 * (gs - 1) + (int)(rate * (gs - 1)) + 2 + 64 * nw + 2;
}
__host__ __device__ inline size_t phi2_group_lds(int gs, int nw, double rate) {
  return align16((size_t)gs * sizeof(PoolClass)) + align16((size_t)gs * 4) + align16((size_t)gs * nw * 8) +
         align16((size_t)gs * kPhiLdsLevels * 8) + align16((size_t)gs * kPhiLdsLevels) +
         3 * align16((size_t)phi2_npos(gs, nw, rate) * 8);
}
__host__ __device__ inline size_t phi2_tree_lds(int T, int G, int tW) {
  (void)T;
  return align16((size_t)(G + (G + 1) / 2) * tW * 2);
}
__host__ __device__ inline size_t phi2_values_lds(int d, int G, int tW, int T) {
  return align16((size_t)G * tW * 2) + align16((size_t)(G + 1) * 8) + align16((size_t)2 * d * 8) + align16((size_t)d * 8) +
         align16((size_t)d) + align16((size_t)T * tW * 2);
}

__global__ __launch_bounds__(512) void k_phi2_group(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  if (!phi2_chain(a)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  __shared__ uint64_t tabs[512];
  __shared__ int sbad;
  const int gs = a.gs, G = a.G, d = a.d, nw = a.nw, tW = a.tW;
  const int t = blockIdx.x / G, g = blockIdx.x - t * G;
  const int j0 = g * gs, ni = min(gs, d - j0);
  const int64_t k0 = (int64_t)t * d + j0;
  phi2_mark_last(a, 19);
  PoolClass* sp = reinterpret_cast<PoolClass*>(sm);
  int* slo = reinterpret_cast<int*>(sm + align16((size_t)gs * sizeof(PoolClass)));
  __shared__ int snw[64];
  uint64_t* smk = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(slo) + align16((size_t)gs * 4));
  double* spr = reinterpret_cast<double*>(reinterpret_cast<uint8_t*>(smk) + align16((size_t)gs * nw * 8));
  uint8_t* spm = reinterpret_cast<uint8_t*>(spr) + align16((size_t)gs * kPhiLdsLevels * 8);
  const int npos = phi2_npos(gs, nw, a.rate);
  double* su = reinterpret_cast<double*>(spm + align16((size_t)gs * kPhiLdsLevels));
  double* slg = su + (align16((size_t)npos * 8) >> 3);
  double* slz = slg + (align16((size_t)npos * 8) >> 3);
  phi2_mark(a, 0, 0);
  // the inputs first (possibly in host memory: one round trip, all loads in flight together,
  // beside the glibc tables'); the label and count copied to the device for k_phi2_values
  int in_lab = 0, in_cnt = 0;
  double in_sig = 0.0;
  if ((int)threadIdx.x < ni) {
    in_lab = a.lab[t];
    in_cnt = a.cnt[t];
    in_sig = a.sig_in[k0 + threadIdx.x];
  }
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  if (threadIdx.x == 0) sbad = 0;
  __syncthreads();
  // 1. the items' windows: start lo and the mask words worth evaluating, [lo, hi) (later words
  // stay 0: a drift past phi_hi fails the walk, as it would the window model)
  if ((int)threadIdx.x < ni) {
    const int64_t k = k0 + threadIdx.x;
    slo[threadIdx.x] = (int)phi_lo(k, a.rate, a.sdev);
    snw[threadIdx.x] = (int)min((int64_t)nw, ((phi_hi(k, a.rate, a.sdev) - slo[threadIdx.x]) >> 6) + 2);
  }
  __syncthreads();
  // 2. the stream logits (while the inputs, possibly in host memory, are on their way) of every position the group's masks read
  const int64_t nom0 = (int64_t)t * 3 * d + d + 2 * (int64_t)j0;
  const int64_t p0 = nom0 + slo[0];
  const int64_t plast = nom0 + 2 * (int64_t)(ni - 1) + slo[ni - 1] + 64 * (int64_t)nw;   // last attempt's first uniform
  if (plast - p0 + 2 > npos) {                                // (window model: never)
    if (threadIdx.x == 0) phi_set_status(a, kPhiWindow);
    return;
  }
  const int np = (int)(plast - p0 + 2);
  const uint64_t* tlog = tabs + 256;
  // (waves 1.. compute the logits while wave 0's lanes prepare the items: the preparation is a
  // long dependent chain per item, the logits are independent work)
  for (int q = (int)threadIdx.x - 64; q < np; q += (int)blockDim.x - 64) {
    if (q < 0) break;
    const int64_t p = p0 + q;
    double u = 0.5, lg = 0.0, lz = 0.0;
    if (p < a.span + 1) u = pool_unif(a.raw[p]);
    if (p < a.span) {
      const double u2 = pool_unif(a.raw[p + 1]);
      lg = glibc::log_r(u / (1.0 - u), tlog);
      lz = glibc::log_r(u * u * u2, tlog);
    }
    su[q] = u;
    slg[q] = lg;
    slz[q] = lz;
  }
  phi2_mark(a, 0, 1);
  // 3. the items: center probabilities, fixed pick, rbeta setup (as k_phi_prep)
  if (threadIdx.x == 0 && g == 0) {
    a.lab_dev[t] = in_lab;
    a.lab_dev[a.T + t] = in_cnt;
  }
  if ((int)threadIdx.x < ni) {
    const int i = threadIdx.x, j = j0 + i;
    const int64_t k = k0 + i;
    const int mj = a.att[j], off = a.aoff[j];
    bool det = false;
    int nact = 0, status;
    PhiCand cp{};
    // the first cluster's center draws take the slice's first d uniforms whatever the drifts:
    // its picks are fixed by them (later clusters start after the drifts before them)
    const double ucen = t == 0 ? pool_unif(a.raw[j]) : -1.0;
    if (mj <= kPhiLdsLevels) {
      status = phi_prep_item_in(a, t, j, k, in_cnt, in_lab, in_sig, spr + i * kPhiLdsLevels, spm + i * kPhiLdsLevels,
                                tabs, &det, &nact, &cp, ucen);
    } else {
      status = phi_prep_item_in(a, t, j, k, in_cnt, in_lab, in_sig, a.cum + (int64_t)t * a.sumatt + off,
                                a.perm + (int64_t)t * a.sumatt + off, tabs, &det, &nact, &cp, ucen);
    }
    if (!status && !det) status = kPhiNonDet;
    if (!status) {
      if (cp.kind == 1) status = kPhiBisect;
      else if (cp.kind != 2 && cp.kind != 3) status = kPhiInactive;
    }
    if (status) {
      phi_set_status(a, status);
      sbad = 1;
    } else {
      sp[i] = as_pool(cp);
    }
  }
  __syncthreads();
  phi2_mark(a, 0, 2);
  phi2_mark_last(a, 20);
  if (sbad) return;
  // 4. masks: bit i of word q of item j is the attempt at drift lo_j + 64 q + i (as k_phi_masks)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  // a wave per item (its rbeta setup in registers), two attempts per lane in flight
  for (int i = wid; i < ni; i += nwv) {
    const PoolClass C = sp[i];
    const int cnw = snw[i];
    const int64_t cpos = nom0 + 2 * (int64_t)i + slo[i];
    for (int q = 0; q < nw; q += 2) {
      const int64_t pa = cpos + 64 * (int64_t)q + lane, pb = pa + 64;
      const int la = (int)(pa - p0), lb = la + 64;
      bool acc0 = false, acc1 = false;
      double x0 = 0.0, x1 = 0.0;
      if (q < cnw && pa < a.span)
        acc0 = phi_attempt(C, su[la], su[la + 1], slg[la], slz[la], tabs, tlog, &x0) && !(x0 > C.thr);
      if (q + 1 < cnw && pb < a.span)
        acc1 = phi_attempt(C, su[lb], su[lb + 1], slg[lb], slz[lb], tabs, tlog, &x1) && !(x1 > C.thr);
      const uint64_t b0 = __ballot(acc0), b1 = __ballot(acc1);
      if (lane == 0) {
        smk[i * nw + q] = b0;
        a.maskd[(k0 + i) * nw + q] = b0;
        if (q + 1 < nw) {
          smk[i * nw + q + 1] = b1;
          a.maskd[(k0 + i) * nw + q + 1] = b1;
        }
      }
    }
  }
  __syncthreads();
  phi2_mark(a, 0, 3);
  phi2_mark_last(a, 21);
  // 4. the group's table: the extra uniforms of its items from start drift lo_0 + c
  uint16_t* out = a.gtab2 + ((int64_t)t * G + g) * tW;
  for (int c = threadIdx.x; c < tW; c += blockDim.x) {
    const int start = slo[0] + c;
    int e = start;
    bool ok = true;
    for (int i = 0; i < ni && ok; ++i) ok = phi_tree_step(smk + i * nw, slo[i], tW, &e);
    out[c] = ok && e - start < (int)kPhiBad ? (uint16_t)(e - start) : kPhiBad;
  }
  __syncthreads();
  phi2_mark(a, 0, 4);
  phi2_mark_last(a, 22);
}

// Cluster t's group tables composed into its table (a.roots) in LDS `st` (phi2_tree_lds);
// sglo: [G] LDS scratch.
__device__ __forceinline__ void phi2_tree_body(const PhiArgs& a, int t, uint16_t* st, int* sglo) {
  const int G = a.G, tW = a.tW, d = a.d, gs = a.gs;
  phi2_mark(a, 0, 5);
  __shared__ int sok;
  if (threadIdx.x == 0) sok = phi_get_status(a) == 0;   // (one atomic load per workgroup, not per thread)
  __syncthreads();
  if (!sok) return;
  uint16_t* A = st;                                     // G tables, then the levels above in B
  uint16_t* B = st + (size_t)G * tW;
  for (int g = threadIdx.x; g < G; g += blockDim.x) sglo[g] = (int)phi_lo((int64_t)t * d + (int64_t)g * gs, a.rate, a.sdev);
  phi2_stage_u16(A, a.gtab2 + (int64_t)t * G * tW, G * tW);
  __syncthreads();
  phi2_mark(a, 0, 6);
  uint16_t* cur = A;
  uint16_t* nxt = B;
  int np = G, span = 1;                                 // nodes, groups per node
  while (np > 1) {
    const int nl = (np + 1) / 2;
    // every node of the level at once (the lookups of different nodes are independent)
    for (int c = threadIdx.x; c < tW; c += blockDim.x) {
      for (int li = 0; li < nl; ++li) {
        const uint16_t* L = cur + (size_t)(2 * li) * tW;
        uint16_t v;
        if (2 * li + 1 < np)
          v = phi_tree_compose(L, cur + (size_t)(2 * li + 1) * tW, sglo[2 * li * span], sglo[(2 * li + 1) * span], tW, c);
        else
          v = L[c];
        nxt[(size_t)li * tW + c] = v;
      }
    }
    __syncthreads();
    // ping-pong: the level just written becomes the source; the next goes where the old source was
    cur = nxt;
    nxt = (cur == B) ? A : B;
    np = nl;
    span *= 2;
  }
  for (int c = threadIdx.x; c < tW; c += blockDim.x) a.roots[(int64_t)t * tW + c] = cur[c];
  phi2_mark(a, 0, 7);
}
__global__ __launch_bounds__(1024) void k_phi2_tree(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (!phi2_chain(a)) return;
  extern __shared__ __attribute__((aligned(16))) uint16_t st[];
  __shared__ int sglo[kPhi2MaxG];                     // window start of each group's first item (of cluster)
  phi2_tree_body(a, blockIdx.x, st, sglo);
}

// One wave: group g's items from start drift e0 (lane i = item j0 + i), the drift of each
// lane the group start plus the extra uniforms of the lanes before it, in fixed-point rounds
// (each round fixes every lane up to the next rejection); the mask words around the group's
// drifts prefetched in registers.  Writes sapos; false when a lane leaves its window.
__device__ __forceinline__ bool phi2_walk_group(const PhiArgs& a, int t, int j0, int ni, int64_t e0, int64_t* sapos,
                                                int64_t* total) {
  const int lane = threadIdx.x & 63;
  const int nw = a.nw, tW = a.tW;
  const bool act = lane < ni;
  const int64_t k = (int64_t)t * a.d + j0 + lane;
  const int64_t lo = act ? phi_lo(k, a.rate, a.sdev) : 0;
  const uint64_t* row = a.maskd + k * nw;
  const int q0 = act ? (int)max((int64_t)0, (e0 - lo) >> 6) : 0;
  uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  if (act) {
    w0 = q0 < nw ? row[q0] : 0ull;
    w1 = q0 + 1 < nw ? row[q0 + 1] : 0ull;
    w2 = q0 + 2 < nw ? row[q0 + 2] : 0ull;
    w3 = q0 + 3 < nw ? row[q0 + 3] : 0ull;
  }
  int64_t dl = e0;
  int ex = 0, tot = 0;
  for (;;) {
    bool bad = false;
    ex = 0;
    if (act) {
      const int64_t off = dl - lo;
      if (off < 0 || off >= tW) {
        bad = true;
      } else {
        const int q = (int)(off >> 6), sh = (int)(off & 63);
        uint64_t lw, hw;
        const int r = q - q0;
        if (r >= 0 && r + 1 <= 3) {
          lw = r == 0 ? w0 : r == 1 ? w1 : w2;
          hw = r == 0 ? w1 : r == 1 ? w2 : w3;
        } else {
          lw = row[q];
          hw = row[q + 1];
        }
        const uint64_t win = sh ? (lw >> sh) | (hw << (64 - sh)) : lw;
        const uint64_t acc = win & 0x5555555555555555ull;
        if (!acc) bad = true;
        else ex = __builtin_ctzll(acc);
      }
    }
    if (__ballot(bad)) return false;
    const int before = wave_excl_scan(ex, &tot);
    const int64_t nd = e0 + before;
    const bool changed = act && nd != dl;
    dl = nd;
    if (!__ballot(changed)) break;
  }
  if (act) sapos[j0 + lane] = (int64_t)t * 3 * a.d + a.d + 2 * (int64_t)(j0 + lane) + dl + ex;
  *total = tot;
  return true;
}

__global__ __launch_bounds__(1024) void k_phi2_values(PhiArgs a) {
  if (gate_closed(a.gate)) return;
  if (a.raw_ptr) a.raw = *a.raw_ptr;
  extern __shared__ __attribute__((aligned(16))) uint8_t wl[];
  __shared__ uint64_t tabs[512];
  __shared__ double red[4 * 16];
  __shared__ double wmx[16], wmn[16];
  __shared__ int sbad, slast;
  const int t = blockIdx.x, d = a.d, G = a.G, gs = a.gs, tW = a.tW;
  uint16_t* stb = reinterpret_cast<uint16_t*>(wl);
  int64_t* sgs = reinterpret_cast<int64_t*>(wl + align16((size_t)G * tW * 2));            // [G + 1] group starts
  double* wtab = reinterpret_cast<double*>(reinterpret_cast<uint8_t*>(sgs) + align16((size_t)(G + 1) * 8));
  int64_t* sapos = reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(wtab) + align16((size_t)2 * d * 8));
  uint8_t* spick = reinterpret_cast<uint8_t*>(sapos) + align16((size_t)d * 8);
  uint16_t* sroot = reinterpret_cast<uint16_t*>(spick + align16((size_t)d));   // [t + 1][tW] cluster tables
  __shared__ int64_t sclo[kPhi2MaxT];                  // window start of each cluster up to t
  __shared__ int sglo3[kPhi2MaxG];                     // window start of each of its groups
  phi2_mark(a, 0, 11);
  const bool on = phi2_chain(a);
  for (int i = threadIdx.x; i < 512; i += blockDim.x) tabs[i] = a.gtab[i];
  if (threadIdx.x == 0) {
    if (!on) phi_set_status(a, kPhiOff);
    sbad = !on || phi_get_status(a) != 0;
  }
  __syncthreads();
  if (!sbad) {
    phi2_stage_u16(stb, a.gtab2 + (int64_t)t * G * tW, G * tW);
    phi2_stage_u16(sroot, a.roots, (t + 1) * tW);
    for (int u = threadIdx.x; u <= t; u += blockDim.x) sclo[u] = phi_lo((int64_t)u * d, a.rate, a.sdev);
    for (int g = threadIdx.x; g < G; g += blockDim.x) sglo3[g] = (int)phi_lo((int64_t)t * d + (int64_t)g * gs, a.rate, a.sdev);
    for (int j = threadIdx.x; j < d; j += blockDim.x) spick[j] = (uint8_t)(a.det[(int64_t)t * d + j] - 1);
    __syncthreads();
    if (threadIdx.x == 0) {
      // the cluster's start drift: the clusters before it from drift 0 (their tables, k_phi2_tree);
      // the last cluster's end is the update's consumption
      int64_t e = 0;
      for (int u = 0; u <= t && !sbad; ++u) {
        if (u == t) a.dts[t] = e;
        if (u == t && t != a.T - 1) break;
        const int64_t c = e - sclo[u];
        const uint16_t v = (c >= 0 && c < tW) ? sroot[(size_t)u * tW + c] : kPhiBad;
        if (v == kPhiBad) sbad = 1;
        else e += v;
      }
      if (!sbad && t == a.T - 1) {
        const int64_t cons = (int64_t)a.T * 3 * d + e;
        if (cons + 1 > a.span) phi_set_status(a, kPhiShort);
        *(int64_t*)(a.status + 2) = cons;
        if (a.pos_out) *a.pos_out = *a.pos_in + a.sweep_len + cons;
      }
      // the groups' start drifts from the cluster's
      e = a.dts[t];
      for (int g = 0; g <= G && !sbad; ++g) {
        sgs[g] = e;
        if (g == G) break;
        const int64_t c = e - sglo3[g];
        const uint16_t v = (c >= 0 && c < tW) ? stb[(size_t)g * tW + c] : kPhiBad;
        if (v == kPhiBad) {
          sbad = 1;
          break;
        }
        e += v;
      }
    }
    __syncthreads();
    phi2_mark(a, 0, 12);
    if (!sbad) {
      const int wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
      for (int g = wid; g < G; g += nwv) {
        const int j0 = g * gs, ni = min(gs, d - j0);
        int64_t tot = 0;
        const bool ok = phi2_walk_group(a, t, j0, ni, sgs[g], sapos, &tot);
        // the walk must end where the group's table says it does
        if ((!ok || sgs[g] + tot != sgs[g + 1]) && (threadIdx.x & 63) == 0) atomicOr(&sbad, 1);
      }
    }
    __syncthreads();
    phi2_mark(a, 0, 13);
    if (sbad) {
      if (threadIdx.x == 0) phi_set_status(a, kPhiWindow);
    } else {
      // (the labels / counts k_phi2_group copied to the device)
      phi_values_body(a, t, spick, sapos, wtab, tabs, tabs + 256, red, wmx, wmn, &sbad, a.lab_dev);
    }
    phi2_mark(a, 0, 14);
  }
  // the last workgroup hands the status and the consumption to the host
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0)
    slast = __hip_atomic_fetch_add(&a.ctr[1], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (!slast) return;
  __threadfence();
  __shared__ int scode, smti;
  __shared__ int64_t soff;
  if (threadIdx.x == 0) {
    scode = phi_get_status(a);
    smti = 0;
    if (scode == 0 && a.state_host) {
      // the block of the position after the update's draws, relative to `raw`
      const uint32_t lo = (uint32_t)__hip_atomic_load(a.status + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t hi = (uint32_t)__hip_atomic_load(a.status + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t cons = (int64_t)(((uint64_t)hi << 32) | lo);
      const int mt = (int)((a.mti_pos - 1 + cons) % 624) + 1;
      const int64_t off = cons - mt;
      if (a.mti_pos >= 1 && a.mti_pos <= 624 && cons > 0 && off >= -a.raw_back && off + 624 <= a.nraw) {
        smti = mt;
        soff = off;
      }
    }
  }
  __syncthreads();
  if (smti) {
    for (int i = threadIdx.x; i < 624; i += blockDim.x) a.state_host[i] = a.raw[soff + i];
  }
  if (a.state_host && threadIdx.x == 0) a.state_host[624] = smti;
  if (a.chain_out && threadIdx.x == 0) {
    const uint32_t lo = (uint32_t)__hip_atomic_load(a.status + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t hi = (uint32_t)__hip_atomic_load(a.status + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.chain_out->end = a.pos0 + (int64_t)(((uint64_t)hi << 32) | lo);
    // (complete with its stream state: a device-side go needs no host adoption, PipeAuto)
    a.chain_out->ok = scode == 0 && smti != 0 ? 1 : 0;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (a.tdbg) a.tdbg[15] = wall_clock64();
  __hip_atomic_store(&a.ctr[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.status_host) {
    const int code = scode;
    const int lo32 = __hip_atomic_load(a.status + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int hi32 = __hip_atomic_load(a.status + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.status_host[1] = 0;
    a.status_host[2] = code ? 0 : lo32;
    a.status_host[3] = code ? 0 : hi32;
    __threadfence_system();
    __hip_atomic_store(a.status_host, code, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

size_t phi2_group_lds_bytes(int gs, int nw, double rate) { return phi2_group_lds(gs, nw, rate); }
size_t phi2_tree_lds_bytes(int T, int G, int tW) { return phi2_tree_lds(T, G, tW); }
size_t phi2_values_lds_bytes(int d, int G, int tW, int T) { return phi2_values_lds(d, G, tW, T); }

hipError_t launch_phi2(const PhiArgs& a, hipStream_t s, hipEvent_t before_values) {
  const int64_t items = (int64_t)a.T * a.d;
  if (items <= 0) return hipSuccess;
  if (a.gs < 1 || a.gs > 64 || a.G != (a.d + a.gs - 1) / a.gs || a.G > kPhi2MaxG || a.T > kPhi2MaxT || a.tW < 64 ||
      a.tW != 64 * (a.nw - 1) || a.tW >= 65535 || a.gen <= 0 || !a.gtab2 || !a.roots || !a.ctr || !a.dts || !a.maskd ||
      !a.lab_dev)
    return hipErrorInvalidValue;
  const size_t l1 = phi2_group_lds(a.gs, a.nw, a.rate), l2 = phi2_tree_lds(a.T, a.G, a.tW),
               l3 = phi2_values_lds(a.d, a.G, a.tW, a.T);
  if (l1 > 150 * 1024 || l2 > 150 * 1024 || l3 > 150 * 1024) return hipErrorInvalidValue;
  static const int th1 = [] {
    const char* e = std::getenv("HDPM_PHI2_GROUP_THREADS");
    const int v = e ? std::atoi(e) : 512;
    return v >= 128 && v <= 512 && v % 64 == 0 ? v : 512;   // (wave 0 prepares, the others compute logits)
  }();
  // The per-cluster kernels beside the sweep's prepass: a workgroup starts only where a CU has
  // room for all of its waves, and the prepass's small workgroups take every slot that frees,
  // so short rows (d <= 256: the tree's and the values' work fits few waves) run in 4-wave
  // workgroups (C5 6,522 -> 7,559 it/s, C3 10,847 -> 11,891 with the device update); wide
  // rows keep 16 waves (C4 6,753 against 5,314 at 4).  HDPM_PHI2_TREE_THREADS /
  // HDPM_PHI2_VALUES_WAVES / HDPM_PHI2_GROUP_THREADS override (testing).
  static const int th2e = [] {
    const char* e = std::getenv("HDPM_PHI2_TREE_THREADS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 64 && v <= 1024 && v % 64 == 0 ? v : 0;
  }();
  static const int w3e = [] {
    const char* e = std::getenv("HDPM_PHI2_VALUES_WAVES");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : 0;
  }();
  const bool narrow = a.d <= 256;
  const int th2 = th2e ? th2e : narrow ? 256 : 1024;
  const int w3 = w3e ? w3e : narrow ? std::min(4, a.wpb) : a.wpb;
  HDPM_LAUNCH(k_phi2_group, dim3((unsigned)(a.T * a.G)), dim3(th1), l1, s, a);
  HDPM_LAUNCH(k_phi2_tree, dim3((unsigned)a.T), dim3(th2), l2, s, a);
  if (before_values) {
    const hipError_t e = hipStreamWaitEvent(s, before_values, 0);
    if (e != hipSuccess) return e;
  }
  HDPM_LAUNCH(k_phi2_values, dim3((unsigned)a.T), dim3(64 * w3), l3, s, a);
  return hipGetLastError();
}

// dynamic LDS of k_phi_cwalk (cluster image + a pick row per wave) and k_phi_values
// (cluster image + tables, positions, picks)
size_t phi_cwalk_lds(int d, int nw, int wpb) { return phi_cwalk_image(d, nw) + 0 * (size_t)wpb; }
int phi_ilp() { return kPhiIlp; }
size_t phi_values_lds(int d, int nw) { return phi_cluster_lds(d, nw) + (size_t)d * (16 + 8 + 1); }

size_t phi_tree_lds_bytes(int SB, int nw, int W) { return phi_tree_lds(SB, nw, W); }
size_t phi_values2_lds_bytes(int d, int nb, int T, int W, int nw) { return phi_values2_lds(d, nb, T, W, nw); }

// tree mode (a.tree != nullptr): k_phi_prep (+ logits) -> k_phi_masks -> k_phi_tree ->
// k_phi_tree_top (segments above one workgroup) -> k_phi_values2; else the per-start-drift
// walks: k_phi_prep -> k_phi_masks -> k_phi_cwalk -> k_phi_chain -> k_phi_values
hipError_t launch_phi(const PhiArgs& a, hipStream_t s) {
  const int64_t items = (int64_t)a.T * a.d;
  if (items <= 0) return hipSuccess;
  if (a.nw < 1 || a.wpb < 1 || a.wpb > 16) return hipErrorInvalidValue;
  const int nprep = (int)((items + 255) / 256);
  const int nlog = (int)std::min<int64_t>(1024, (a.span + 255) / 256);
  HDPM_LAUNCH(k_phi_prep, dim3((unsigned)(nprep + nlog)), dim3(256), 0, s, a, nprep);
  // one wave per (candidate, mask word): enough workgroups for every fixed pick's item in one
  // pass (the loop covers the extra candidates of uniform-dependent picks)
  const int64_t mwaves = items * a.nw;
  HDPM_LAUNCH(k_phi_masks, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(32768, (mwaves + 3) / 4))),
                     dim3(256), 0, s, a);
  if (a.tree) {
    if (a.tW < 64 || a.tSB < 1 || a.tS < 1 || a.tnb < 1) return hipErrorInvalidValue;
    HDPM_LAUNCH(k_phi_tree, dim3((unsigned)(a.T * a.tS)), dim3(1024), phi_tree_lds(a.tSB, a.nw, a.tW), s, a);
    if (a.tS > 1) HDPM_LAUNCH(k_phi_tree_top, dim3((unsigned)a.T), dim3(1024), 0, s, a);
    if (a.S == 1 && a.Wc >= 1 && a.groups >= 1) {
      // clusters with a pick that depends on the uniform: their root tables by the walks
      const int wthreads = std::min(1024, ((a.Wc + kPhiIlp * a.groups - 1) / (kPhiIlp * a.groups) + 63) / 64 * 64);
      HDPM_LAUNCH(k_phi_cwalk, dim3((unsigned)(a.T * a.groups)), dim3(wthreads), phi_cwalk_lds(a.d, a.nw, 16),
                         s, a);
    }
    HDPM_LAUNCH(k_phi_values2, dim3((unsigned)a.T), dim3(64 * a.wpb), phi_values2_lds(a.d, a.tnb, a.T, a.tW, a.nw),
                       s, a);
    return hipGetLastError();
  }
  if (a.Wc < 1 || a.groups < 1) return hipErrorInvalidValue;
  const int wthreads = std::min(1024, ((a.Wc + kPhiIlp * a.groups - 1) / (kPhiIlp * a.groups) + 63) / 64 * 64);
  HDPM_LAUNCH(k_phi_cwalk, dim3((unsigned)(a.T * a.S * a.groups)), dim3(wthreads), phi_cwalk_lds(a.d, a.nw, 16),
                     s, a);
  const int64_t nF = (int64_t)a.T * a.S * a.Wc;
  HDPM_LAUNCH(k_phi_chain, dim3(1), dim3(1024), nF <= 16384 ? (size_t)nF * 4 : 0, s, a);
  HDPM_LAUNCH(k_phi_values, dim3((unsigned)a.T), dim3(64 * a.wpb), phi_values_lds(a.d, a.nw), s, a);
  return hipGetLastError();
}

}  // namespace hdpm
