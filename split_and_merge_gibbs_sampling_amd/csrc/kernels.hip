// kernels.hip -- gfx950 kernels of the hdpm Neal-8 sweep.
//
// Hot path (BASELINE north_star):
//   k_prepass   N x (K+m) Hamming log-likelihood matrix (exact, reference summation
//               order, code/neal8.cpp:40-92) + per-point certainty classification.
//   k_resolve   the sequential reassignment (n8:95-159) for the points whose draw is
//               not already decided, in index order, with exact R/Rcpp draw semantics.
//   k_relabel / k_hist / k_loglik   sufficient statistics for update_phi
//               (cf:535-590) and compute_loglikelihood (cf:379-401).
//
// Bit-exactness: every per-attribute dhamming value comes from host tables computed
// with glibc in the reference expression; the device only selects and adds them in
// j order (built with -ffp-contract=off), so each log-likelihood is bit-identical to
// the reference's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstdio>

#include "glibc_math.hpp"
#include "kernels.hpp"

namespace hdpm {

// Compute units of the current device, queried once per device (grids of persistent kernels;
// several contexts of one process may sit on different devices)
int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int c = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (c <= 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    __atomic_store_n(&cache[dev], c, __ATOMIC_RELAXED);
  }
  return c;
}

// Device copies of glibc's exp / log tables: every exp and log whose result decides a draw
// (n8:95, sm:209-210, sm:150-158) runs glibc's algorithm (glibc_math.hpp), so the device's
// probabilities are the host libm's bit for bit and the reference's cumulative compare
// `rU <= p[j]` cannot flip on an ulp (ocml's exp differs from glibc's in the last place).
namespace devtab {
#define HDPM_GLIBC_TABLE __constant__
#include "glibc_tables.inc"
#undef HDPM_GLIBC_TABLE
}  // namespace devtab

template <bool kOcml = false>
__device__ __forceinline__ double dexp(double x) {
  if constexpr (kOcml) return exp(x);   // testing only: the pre-glibc behaviour
  else return glibc::exp_r(x, devtab::kGlibcExpTab);
}
template <bool kOcml = false>
__device__ __forceinline__ double dlog(double x) {
  if constexpr (kOcml) return log(x);
  else return glibc::log_r(x, devtab::kGlibcLogTab);
}

__device__ __forceinline__ double raw_to_unif(uint32_t y) {
  const double i2_32m1 = 2.328306437080797e-10;
  double x = (double)y * 2.3283064365386963e-10;
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

// sample(P, 1, FALSE)[0] - 1 with one uniform (Rcpp EmpiricalSample, n8:66).
__device__ __forceinline__ int64_t pick_entry(uint32_t y, int64_t P) {
  return (int64_t)((int)((double)(int)P * raw_to_unif(y) + 1)) - 1;
}

// Latent entries far below the point's clusters (k_exact_rows_lv, lbound).  A latent whose
// log-weight is at least 40 below the best cluster's changes no draw whatever its exact value:
// its exp(v - max) < 2^-57 of the partial sum it is added to (the clusters come first in index
// order, n8:95-96), so sum(probs), FixupProb's sum and every other probability keep their bits,
// and it sorts behind entries whose cumulative sum reaches 1 - E 2^-52 > the largest uniform
// (1 - 2^-33): it can be taken as -inf (probability 0).  The exact rows store such a latent's
// head bound (kLatMargin below, which covers a snapshot draw's radius cap kSpecRadCap twice) and
// flag it; a reader that finds it no longer 40 below computes the exact sum (latent_exact).
constexpr double kLatMargin = 56.0;
constexpr double kSpecRadCap = 8.0;
// n8:47-49 for one latent entry, attribute order (bit-exact with the exact-rows sums); one lane
__device__ __noinline__ double latent_exact(const uint8_t* codes_t, int nq, int D, const uint8_t* pcodes,
                                            const double* ptab, int64_t i, int64_t pe) {
  const uint8_t* cc = pcodes + pe * (int64_t)(nq * 16);
  const double* tl = ptab + pe * 2 * (int64_t)D;
  double acc = 0.0;
  for (int j = 0; j < D; ++j) {
    const uint8_t x = codes_t[tiled_offset(i, j, nq)];
    acc += tl[2 * j + (x != cc[j] ? 1 : 0)];
  }
  return acc;
}

__device__ __forceinline__ int a_code(const uint8_t* codes_t, int64_t i, int j, int nq) {
  return codes_t[tiled_offset(i, j, nq)];
}

__device__ __forceinline__ bool byte_differs(const uint4& dx, int b) {
  const uint32_t w = b < 4 ? dx.x : b < 8 ? dx.y : b < 12 ? dx.z : dx.w;
  return ((w >> ((b & 3) * 8)) & 0xffu) != 0u;
}

// Register-staged codes of one point (NQR chunks of 16 bytes); NQR == 0 -> reload.
template <int NQR>
struct PointCodes {
  uint4 r[NQR > 0 ? NQR : 1];
  const uint8_t* base;
  int64_t i;
  int nq;
  __device__ __forceinline__ void load(const uint8_t* codes_t, int64_t i_, int nq_) {
    base = codes_t; i = i_; nq = nq_;
    if constexpr (NQR > 0) {
#pragma unroll
      for (int q = 0; q < NQR; ++q) r[q] = *(const uint4*)(codes_t + tiled_offset(i, q * 16, nq));
    }
  }
  __device__ __forceinline__ uint4 chunk(int q) const {
    if constexpr (NQR > 0) return r[q];
    else return *(const uint4*)(base + tiled_offset(i, q * 16, nq));
  }
};

// Exact log-likelihood of the point against a wave-uniform table (existing cluster).
template <int NQR>
__device__ __forceinline__ double ll_uniform(const PointCodes<NQR>& x, int d, const uint8_t* __restrict__ cc,
                                             const double* __restrict__ tab) {
  double ll = 0.0;
  auto body = [&](int q) {
    const uint4 xq = x.chunk(q);
    const uint4 cq = *(const uint4*)(cc + q * 16);
    const uint4 dx = make_uint4(xq.x ^ cq.x, xq.y ^ cq.y, xq.z ^ cq.z, xq.w ^ cq.w);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int j = q * 16 + b;
      if (j < d) {
        const double ta = tab[2 * j], tb = tab[2 * j + 1];
        ll += byte_differs(dx, b) ? tb : ta;
      }
    }
  };
  if constexpr (NQR > 0) {
#pragma unroll
    for (int q = 0; q < NQR; ++q) body(q);
  } else {
    for (int q = 0; q < x.nq; ++q) body(q);
  }
  return ll;
}

// Exact log-likelihood against a per-lane table (latent pool entry): only the selected
// half of each (match, mismatch) pair is fetched.
template <int NQR>
__device__ __forceinline__ double ll_lane(const PointCodes<NQR>& x, int d, const uint8_t* cc,
                                          const double* tab, int* hamming) {
  double ll = 0.0;
  int h = 0;
  auto body = [&](int q) {
    const uint4 xq = x.chunk(q);
    const uint4 cq = *(const uint4*)(cc + q * 16);
    const uint4 dx = make_uint4(xq.x ^ cq.x, xq.y ^ cq.y, xq.z ^ cq.z, xq.w ^ cq.w);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int j = q * 16 + b;
      if (j < d) {
        const int mis = byte_differs(dx, b) ? 1 : 0;
        h += mis;
        ll += tab[2 * j + mis];
      }
    }
  };
  if constexpr (NQR > 0) {
#pragma unroll
    for (int q = 0; q < NQR; ++q) body(q);
  } else {
    for (int q = 0; q < x.nq; ++q) body(q);
  }
  if (hamming) *hamming = h;
  return ll;
}


// Certainty by the draw's uniform (n8:95-102).  With the own cluster ahead of every other of
// the E entries by at least mg in log-weight, the max is the own entry (exp(0) = 1), revsort
// puts it first, and its computed probability after the sums and FixupProb is at least
// 1 / (1 + (E - 1) e^-mg) up to ~(2E + 10) ulps of rounding; Rcpp's ProbSampleReplace picks
// the first entry iff rU <= that probability.  So a point whose categorical uniform lies
// below the bound (shrunk by 1e-12 relative, and mg by 1e-6) stays whatever the exact rows
// -- no exact row is needed even though the margin is far below T.  E <= 200 keeps the
// Walker alias out of reach (only the own entry has n p > 0.1).
__device__ __forceinline__ bool stay_by_uniform(double mg, uint32_t raw_cat, int E) {
  if (!(mg > 1e-6) || E > 200) return false;
  const double pl = 1.0 / (1.0 + (double)(E - 1) * exp(-(mg - 1e-6)));
  return raw_to_unif(raw_cat) <= pl * (1.0 - 1e-12);
}

// The same test out of line, for kernels at their register limit: inlined, the exp's
// polynomial constants were hoisted out of k_prepass_wide's chunk loop into VGPRs and spilled
// (29 MB of scratch writes per C4 launch at 4 waves/SIMD).
__device__ __attribute__((noinline)) bool stay_by_uniform_call(double mg, uint32_t raw_cat, int E) {
  return stay_by_uniform(mg, raw_cat, E);
}

// Margin, row position and the ordered compaction of the block's uncertain points (the
// block's kBlock points are threads 0..kBlock-1 of its NT; the others pass active = false).
template <int NT = kBlock>
__device__ __forceinline__ void prepass_finish(const PrepassArgs& a, int64_t i, bool active, int own_cnt, double mg) {
  const int tid = threadIdx.x;
  const bool uncertain =
      active && !(own_cnt >= 2 && (mg > a.thresh ||
                                   stay_by_uniform(mg - a.dmax2, a.raw[i * (a.m + 1) + a.m], a.K + a.m)));
  if (active) a.margin[i] = mg;

  // ordered compaction of the uncertain points of this block
  __shared__ int s_wcnt[NT / kWave];
  const int lane = tid & 63, wv = tid >> 6;
  const unsigned long long bal = __ballot(uncertain);
  const int pre = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) s_wcnt[wv] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / kWave; ++w) {
    off += w < wv ? s_wcnt[w] : 0;
    tot += s_wcnt[w];
  }
  const int row = blockIdx.x * kBlock + off + pre;
  if (active) a.rowpos[i] = uncertain ? row : -1;
  if (uncertain) a.list[row] = (int)i;
  if (tid == 0) a.cnt[blockIdx.x] = tot;

}

// ------------------------------------------------------------------ prepass
// Uniform (wave-invariant) load through the constant address space -> scalar loads.
template <class T>
__device__ __forceinline__ T ldu(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

template <bool U>
__device__ __forceinline__ uint64_t ldw(const uint64_t* p) {
  if constexpr (U) return ldu(p);
  else return *p;
}

__device__ __forceinline__ double as_f64(uint64_t u) { return __longlong_as_double((long long)u); }

// Upper bound on latent entry pe's ll for point i from its pool-entry head (kernels.hpp
// "Pool-entry heads"; the prepass's latent bound), one lane
__device__ __forceinline__ double latent_head_ub(const PrepassArgs& a, int64_t i, int64_t pe) {
  const int W = a.wb * a.Ws, HS = head_stride(a.wb, a.Ws);
  const uint64_t* h = a.pool_head + pe * HS;
  int H = 0;
  for (int w = 0; w < a.Ws; ++w) {
    uint64_t m = 0;
    for (int b = 0; b < a.wb; ++b) m |= a.xbs[packed_offset(i, b * a.Ws + w, W)] ^ h[b * a.Ws + w];
    H += __popcll(m);
  }
  const uint64_t p0 = h[W], p1 = h[W + 1];
  const double A = (double)__uint_as_float((uint32_t)p0), dmn = (double)__uint_as_float((uint32_t)(p0 >> 32));
  const double sa = (double)__uint_as_float((uint32_t)p1), sb = (double)__uint_as_float((uint32_t)(p1 >> 32));
  double low = dmn * (double)H;
  if (H >= a.head_ha) low = fmax(low, sa + dmn * (double)(H - a.head_ha));
  if (H >= a.head_hb) low = fmax(low, sb + dmn * (double)(H - a.head_hb));
  return A - low + kBoundEps * (1.0 + fabs(A) + low);
}

// A draw's log-weights v[0..E) (clusters, then latents) whose latent columns flagged in lmv hold
// head bounds: each such latent is -inf (probability 0) while its bound is kLatNegligible below
// the best cluster, else its exact sum (latent_exact).  Latent 0 of a singleton is the point's
// own cluster (n8:65-75), never flagged.
template <int EM>
__device__ __forceinline__ void latent_fix(const uint8_t* codes_t, int nq, int D, ParamTables pool,
                                           const uint32_t* raw, int64_t P, double logfac, double (&v)[EM], int K,
                                           int E, unsigned int lmv, bool single, int64_t i, int m, double negl) {
  double mxc = -INFINITY;
#pragma unroll
  for (int e = 0; e < EM; ++e) mxc = e < K ? fmax(mxc, v[e]) : mxc;
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const int l = e - K;
    if (e >= K && e < E && ((lmv >> l) & 1u) && !(l == 0 && single)) {
      if (v[e] <= mxc - negl) {
        v[e] = -INFINITY;
      } else {
        const int64_t pe = pick_entry(raw[i * (m + 1) + l], P);
        v[e] = logfac + latent_exact(codes_t, nq, D, pool.codes, pool.tab, i, pe);
      }
    }
  }
}

// Mismatch mask M (one bit per attribute) of bit-sliced rows x and record codes, and H.
template <int WB, int WS, bool U>
__device__ __forceinline__ int mismatch_mask(const uint64_t (&x)[WB * WS], const uint64_t* rec, uint64_t (&M)[WS]) {
  int H = 0;
#pragma unroll
  for (int w = 0; w < WS; ++w) {
    uint64_t m = 0;
#pragma unroll
    for (int b = 0; b < WB; ++b) m |= x[b * WS + w] ^ ldw<U>(rec + b * WS + w);
    M[w] = m;
    H += __popcll(m);
  }
  return H;
}

// Sq = sum_b 2^b popc(M & plane_b)
template <int WB, int WS, bool U>
__device__ __forceinline__ int penalty_sum(const uint64_t (&M)[WS], const uint64_t* rec) {
  int Sq = 0;
#pragma unroll
  for (int w = 0; w < WS; ++w)
#pragma unroll
    for (int b = 0; b < kQ; ++b) Sq += __popcll(M[w] & ldw<U>(rec + (WB + b) * WS + w)) << b;
  return Sq;
}

// A whole record gathered with 16-B loads into registers.
template <int RW>
__device__ __forceinline__ void load_record(const uint64_t* rec, uint64_t (&R)[RW]) {
  static_assert(RW % 2 == 0, "records are 16-B aligned");
  const uint4* r4 = (const uint4*)rec;
#pragma unroll
  for (int k = 0; k < RW / 2; ++k) {
    const uint4 v = r4[k];
    R[2 * k] = ((uint64_t)v.y << 32) | v.x;
    R[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
  }
}

// Register-record versions (constant indices into R).
template <int WB, int WS, int RW>
__device__ __forceinline__ int mismatch_r(const uint64_t (&x)[WB * WS], const uint64_t (&R)[RW], uint64_t (&M)[WS]) {
  int H = 0;
#pragma unroll
  for (int w = 0; w < WS; ++w) {
    uint64_t m = 0;
#pragma unroll
    for (int b = 0; b < WB; ++b) m |= x[b * WS + w] ^ R[b * WS + w];
    M[w] = m;
    H += __popcll(m);
  }
  return H;
}
template <int WB, int WS, int RW>
__device__ __forceinline__ int penalty_r(const uint64_t (&M)[WS], const uint64_t (&R)[RW]) {
  int Sq = 0;
#pragma unroll
  for (int w = 0; w < WS; ++w)
#pragma unroll
    for (int b = 0; b < kQ; ++b) Sq += __popcll(M[w] & R[(WB + b) * WS + w]) << b;
  return Sq;
}

// Per-label summary for the prepass's cluster loop (one level of independent scalar loads
// per label instead of the label -> slot -> record / count -> logn chain):
// csum[l] = [record of slot_of_label[l] (bw words), logn[count], slot].
__global__ void k_cluster_summary(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {     // memset dispatches less per sweep
    if (a.zero) *a.zero = 0;
    if (a.wide_ctr) {
      a.wide_ctr[0] = 0;
      a.wide_ctr[1] = 0;
      a.wide_ctr[2] = 0;
    }
  }
  const int sw = a.bw + 2;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < a.K * sw; e += gridDim.x * blockDim.x) {
    const int l = e / sw, w = e - l * sw;
    const int s = a.slot_of_label[l];
    uint64_t v;
    if (w < a.bw) v = a.slot_bnd[(int64_t)s * a.bw + w];
    else if (w == a.bw) v = (uint64_t)__double_as_longlong(a.logn[a.counts[s]]);
    else v = (uint64_t)s;
    a.csum[e] = v;
  }
}

// Bounds-first prepass: every point gets rigorous bounds on its K + m log-weights from
// Hamming popcounts of bit-sliced rows; only points whose draw is not provably "stay" get
// exact rows.
//   own cluster (count >= 2): precise lower bound lo (penalty planes, record gathered);
//   other clusters: crude upper bound A - dmin H from the codes alone (scalar loads),
//     refined with the planes only in waves where some lane's crude bound could still
//     stop the point from being certain (ub > lo - thresh);
//   latent entries: precise upper bound from their pool record (16-B gathers, all m in
//     flight together when the records are small).
// margin = lo - max(ub) is a lower bound on how far the own cluster leads every other
// entry; the point is certain when it exceeds `thresh`.
// Upper bound on a latent entry's log-weight from its head (kernels.hpp "Pool-entry
// heads"); lanes whose head bound does not clear `cut` gather the full record and take
// the precise bound as well.
template <int WB, int WS>
__device__ __forceinline__ double latent_ub_head(const PrepassArgs& a, const uint64_t (&x)[WB * WS],
                                                 const uint64_t (&Hd)[WB * WS + 2], int64_t e, double cut) {
  constexpr int RW = (WB + kQ) * WS + 4, SC = (WB + kQ) * WS, HW = WB * WS + 2;
  uint64_t M[WS];
  const int H = mismatch_r<WB, WS, HW>(x, Hd, M);
  const uint64_t p0 = Hd[HW - 2], p1 = Hd[HW - 1];
  const double A = (double)__uint_as_float((uint32_t)p0), dmn = (double)__uint_as_float((uint32_t)(p0 >> 32));
  const double sa = (double)__uint_as_float((uint32_t)p1), sb = (double)__uint_as_float((uint32_t)(p1 >> 32));
  double low = dmn * (double)H;
  if (H >= a.head_ha) low = fmax(low, sa + dmn * (double)(H - a.head_ha));
  if (H >= a.head_hb) low = fmax(low, sb + dmn * (double)(H - a.head_hb));
  double ub = a.logfac + (A - low + kBoundEps * (1.0 + fabs(A) + low));
  if (ub > cut) {
    uint64_t R[RW];
    load_record<RW>(a.pool_bnd + e * a.bw, R);
    const int Sq = penalty_r<WB, WS, RW>(M, R);
    const double Af = as_f64(R[SC]), dl = as_f64(R[SC + 1]);
    const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
    ub = fmin(ub, a.logfac + (Af - pmin + kBoundEps * (1.0 + fabs(Af) + pmax)));
  }
  return ub;
}

template <int WB, int WS, bool HEAD>
__global__ __launch_bounds__(kBlock) void k_prepass(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  constexpr int WR = WB * WS;                  // row words
  constexpr int RW = (WB + kQ) * WS + 4;       // record words
  constexpr int SC = (WB + kQ) * WS;           // record scalars: A, delta, dmin, scale
  constexpr int NPF = HEAD ? 3 : RW <= 16 ? 3 : RW <= 32 ? 2 : 1;   // pool records in flight
  constexpr int LW = HEAD ? WR + 2 : RW;       // words gathered first per latent pick
  constexpr int HS = head_stride(WB, WS);      // head stride (words)
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)a.p0 + (int64_t)blockIdx.x * kBlock + tid;
  const bool active = i < a.n;
  const int64_t ii = active ? i : (int64_t)a.n - 1;
  uint64_t x[WR];
#pragma unroll
  for (int q = 0; q < WR; ++q) x[q] = a.xbs[packed_offset(ii, q, WR)];
  const int own = a.c[ii];
  const int own_cnt = a.counts[own];
  const uint32_t* raw = a.raw + ii * (a.m + 1);
  double mg = -INFINITY;
  if (own_cnt >= 2) {
    // the first latent records' gathers go out first: their latency overlaps the
    // own-cluster bound and the cluster loop
    uint64_t Rp[NPF][LW];
    int64_t pe[NPF];
    auto gather = [&](int u, int l) {
      pe[u] = pick_entry(raw[l], a.P);
      if constexpr (HEAD) load_record<LW>(a.pool_head + pe[u] * HS, Rp[u]);
      else load_record<LW>(a.pool_bnd + pe[u] * a.bw, Rp[u]);
    };
#pragma unroll
    for (int u = 0; u < NPF; ++u)
      if (u < a.m) gather(u, u);
    uint64_t M[WS];
    double lo;
    {
      uint64_t R[RW];
      load_record<RW>(a.slot_bnd + (int64_t)own * a.bw, R);
      const int H = mismatch_r<WB, WS, RW>(x, R, M);
      const int Sq = penalty_r<WB, WS, RW>(M, R);
      const double A = as_f64(R[SC]), dl = as_f64(R[SC + 1]);
      const double pmax = dl * (double)(Sq + H);
      lo = a.logn[own_cnt - 1] + (A - pmax - kBoundEps * (1.0 + fabs(A) + pmax));
    }
    const double cut = lo - a.thresh;        // an entry whose ub stays below this cannot matter
    double ubmax = -INFINITY;
    for (int l = 0; l < a.K; ++l) {
      const uint64_t* bd = a.csum + (int64_t)l * (RW + 2);
      const int s = (int)ldu(bd + RW + 1);
      const int H = mismatch_mask<WB, WS, true>(x, bd, M);
      const double A = as_f64(ldu(bd + SC)), dmin = as_f64(ldu(bd + SC + 2)), scale = as_f64(ldu(bd + SC + 3));
      const double lg = as_f64(ldu(bd + RW));
      double ub = lg + (A - dmin * (double)H + kBoundEps * (1.0 + scale));
      const bool need = s != own && ub > cut;
      if (__ballot(need)) {
        const int Sq = penalty_sum<WB, WS, true>(M, bd);
        const double dl = as_f64(ldu(bd + SC + 1));
        const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
        ub = fmin(ub, lg + (A - pmin + kBoundEps * (1.0 + fabs(A) + pmax)));
      }
      if (s != own) ubmax = fmax(ubmax, ub);
    }
    for (int l0 = 0; l0 < a.m; l0 += NPF) {
      if (l0 > 0) {
#pragma unroll
        for (int u = 0; u < NPF; ++u)
          if (l0 + u < a.m) gather(u, l0 + u);
      }
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        if constexpr (HEAD) {
          if (l0 + u < a.m) ubmax = fmax(ubmax, latent_ub_head<WB, WS>(a, x, Rp[u], pe[u], cut));
        } else if (l0 + u < a.m) {
          const int H = mismatch_r<WB, WS, RW>(x, Rp[u], M);
          const int Sq = penalty_r<WB, WS, RW>(M, Rp[u]);
          const double A = as_f64(Rp[u][SC]), dl = as_f64(Rp[u][SC + 1]);
          const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
          ubmax = fmax(ubmax, a.logfac + (A - pmin + kBoundEps * (1.0 + fabs(A) + pmax)));
        }
      }
    }
    mg = lo - ubmax;
  }
  prepass_finish(a, i, active, own_cnt, mg);
}

// Generic width (planes wider than 4 words, or wide codes): rows and records read from
// memory as needed.
__global__ __launch_bounds__(kBlock) void k_prepass_generic(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)a.p0 + (int64_t)blockIdx.x * kBlock + tid;
  const bool active = i < a.n;
  const int64_t ii = active ? i : (int64_t)a.n - 1;
  const int WB = a.wb, WS = a.Ws, WR = WB * WS, SC = (WB + kQ) * WS;
  const int own = a.c[ii];
  const int own_cnt = a.counts[own];
  const uint32_t* raw = a.raw + ii * (a.m + 1);
  auto bounds = [&](const uint64_t* rec, int& H, int& Sq) {
    H = 0;
    Sq = 0;
    for (int w = 0; w < WS; ++w) {
      uint64_t m = 0;
      for (int b = 0; b < WB; ++b) m |= a.xbs[packed_offset(ii, b * WS + w, WR)] ^ rec[b * WS + w];
      H += __popcll(m);
      for (int b = 0; b < kQ; ++b) Sq += __popcll(m & rec[(WB + b) * WS + w]) << b;
    }
  };
  double mg = -INFINITY;
  if (own_cnt >= 2) {
    int H, Sq;
    const uint64_t* ro = a.slot_bnd + (int64_t)own * a.bw;
    bounds(ro, H, Sq);
    const double A = as_f64(ro[SC]), dl = as_f64(ro[SC + 1]);
    const double pmax = dl * (double)(Sq + H);
    const double lo = a.logn[own_cnt - 1] + (A - pmax - kBoundEps * (1.0 + fabs(A) + pmax));
    double ubmax = -INFINITY;
    auto upper = [&](const uint64_t* rec, double base) {
      int h, sq;
      bounds(rec, h, sq);
      const double AA = as_f64(rec[SC]), d2 = as_f64(rec[SC + 1]);
      const double pm = d2 * (double)(sq + h);
      return base + (AA - d2 * (double)sq + kBoundEps * (1.0 + fabs(AA) + pm));
    };
    for (int l = 0; l < a.K; ++l) {
      const int s = a.slot_of_label[l];
      if (s != own) ubmax = fmax(ubmax, upper(a.slot_bnd + (int64_t)s * a.bw, a.logn[a.counts[s]]));
    }
    for (int l = 0; l < a.m; ++l) ubmax = fmax(ubmax, upper(a.pool_bnd + pick_entry(raw[l], a.P) * a.bw, a.logfac));
    mg = lo - ubmax;
  }
  prepass_finish(a, i, active, own_cnt, mg);
}

// Wide layouts (kernels.hpp wide_fits; C4: d = 784, wb = 4, Ws = 13 -- a 416-B row, 864-B
// records): the same bounds as k_prepass, but a point is worked on by a 16-lane group, lane
// w holding plane word w (and w + 16) of every bit-plane, so each record is read once per
// point with coalesced 8-B loads (a 104-B run per plane) and H / Sq are summed across the
// group with DPP row operations (one DPP row = one group).  Persistent workgroups of 16
// groups walk 16-point chunks (chunk c = blockIdx + k gridDim: no tail of a second wave of
// workgroups), staging each chunk's rows, labels, counts and raw draws in LDS while the
// previous chunk is computed (register prefetch); the cluster summaries are staged once per
// workgroup.  Latent picks gather the entry's head (codes + the four floats, 448 B at C4); a
// group whose head bound does not clear `cut` reads the record's penalty planes too.  Each
// chunk is its own list block (kWideChunk points: cnt[c], list rows c * kWideChunk + q).
constexpr int kWideThreads = 256;           // 16 groups of 16 lanes
constexpr int kWideChunk = kWideThreads / 16;

// Sum over the 16 lanes of a DPP row (every lane gets the total).
__device__ __forceinline__ int row_sum16(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);   // row_ror:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);   // row_ror:8
  return v;
}

// Record arrays in HBM are read through buffer resources: one 32-bit lane offset per
// record (entry * stride + 8 w) and the plane offsets in the scalar offset operand, so a
// record costs one VGPR of addressing instead of a 64-bit address per plane word.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
  const int nrec = (int)min(bytes, (int64_t)0x7fffffff);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ uint64_t bload(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0);
  return ((uint64_t)v[1] << 32) | v[0];
}

// A point's row in a 16-lane group: lane w holds word w (and w + 16) of each bit-plane.
// `ld(k, q)` returns the lane's word w + 16 k of a record at the wave-uniform word offset q.
template <int WB, int NW>
struct WideRow {
  uint64_t x[NW][WB];
  int WS;
  bool val[NW];                              // w + 16 k < WS
  template <class LD>
  __device__ __forceinline__ int mismatch(LD ld, uint64_t (&M)[NW]) const {
    int h = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      uint64_t m = 0;
#pragma unroll
      for (int b = 0; b < WB; ++b) m |= x[k][b] ^ ld(k, b * WS);
      m = val[k] ? m : 0ull;
      M[k] = m;
      h += __popcll(m);
    }
    return row_sum16(h);
  }
  // Sq = sum_b 2^b popc(M & plane_b), planes at word offsets (WB + b) WS
  template <class LD>
  __device__ __forceinline__ int penalty(LD ld, const uint64_t (&M)[NW]) const {
    int s = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
      for (int b = 0; b < kQ; ++b) s += __popcll(M[k] & ld(k, (WB + b) * WS)) << b;
    return row_sum16(s);
  }
};

// Dynamic LDS of k_prepass_wide: two chunks' rows [2][16][wb Ws + 1], and (CL) the cluster
// summaries [K][bw + 2].
constexpr int kWidePf = kWideRowMax * kWideChunk / kWideThreads;   // row words per thread prefetched
constexpr int kWideMaxM1 = 16;              // m + 1 <= 16: a chunk's raw draws fit one wave's lanes x 4
__host__ __device__ inline size_t wide_rows_words(int wb, int Ws) { return (size_t)kWideChunk * (wb * Ws + 1); }
size_t prepass_wide_lds_bytes(int wb, int Ws, int m, int K, int bw, bool cl) {
  (void)m;
  return 8 * (2 * wide_rows_words(wb, Ws) + (cl ? (size_t)K * (bw + 2) : 0));
}
// byte offsets of the record arrays must fit the buffer instructions' 32-bit offsets
bool prepass_wide_offsets_fit(const PrepassArgs& a) {
  const int64_t hs = head_stride(a.wb, a.Ws);
  return a.m + 1 <= kWideMaxM1 && a.P * (int64_t)std::max<int64_t>(a.bw, hs) * 8 + 4096 < 0x7fffffff;
}

// Waves per SIMD the compiler must fit: 4 (128 VGPRs) for C4's layout (wb 4, one word per
// lane; 121 VGPRs with two heads in flight, no spills), measured 46.5 against 48.5 us at its
// natural 3 (profiles/r05/wide_prepass); the other layouts keep the allocation they need.
template <int WB, int NW>
constexpr int wide_min_waves() { return WB == 4 && NW == 1 ? 4 : 1; }

template <int WB, int NW, bool CL>
__global__ __launch_bounds__(kWideThreads, (wide_min_waves<WB, NW>())) void k_prepass_wide(PrepassArgs a, int nchunks, int claim) {
  if (!pipe_gate(a)) return;
  extern __shared__ uint64_t s_dyn[];
  __shared__ double s_mg[2][kWideChunk];
  __shared__ int s_oc[2][kWideChunk];
  __shared__ int s_own[2][kWideChunk];
  __shared__ uint32_t s_raw[2][kWideChunk * kWideMaxM1];
  const int WS = a.Ws, WR = WB * WS, RS = WR + 1, SC = (WB + kQ) * WS, HS = head_stride(WB, WS);
  const int bw = a.bw, cw = a.bw + 2;
  uint64_t* s_rows0 = s_dyn;                 // two row buffers: chunk c reads one while c + grid is staged
  uint64_t* s_cs = s_dyn + 2 * wide_rows_words(WB, WS);
  const int tid = threadIdx.x, g = tid >> 4, w = tid & 15, m1 = a.m + 1;
  const int w8 = 8 * w;
  const __amdgpu_buffer_rsrc_t r_slot = make_rsrc(a.slot_bnd, (int64_t)(a.S + 2) * bw * 8);
  const __amdgpu_buffer_rsrc_t r_pool = make_rsrc(a.pool_bnd, a.P * bw * 8);
  const __amdgpu_buffer_rsrc_t r_head = make_rsrc(a.pool_head, a.P * HS * 8);
  const __amdgpu_buffer_rsrc_t r_csum = make_rsrc(a.csum, (int64_t)a.K * cw * 8);
  if constexpr (CL) {
    for (int e = tid; e < a.K * cw; e += kWideThreads) s_cs[e] = a.csum[e];
  }
  // the next chunk's rows, label / count and raw draws, in registers until staged
  uint64_t pf[kWidePf];
  int pf_own = 0, pf_oc = 0;
  uint32_t pf_raw[4];
  auto fetch = [&](int c) {
    const int64_t i0 = (int64_t)a.p0 + (int64_t)c * kWideChunk;
    // (32-bit point indices: n < 2^31; 64-bit forms of them were kept live across the loop)
    const int ip = min((int)i0 + (tid & (kWideChunk - 1)), a.n - 1);
    const uint64_t* rowp = a.xbs + ((int64_t)(ip >> 6) * WR) * 64 + (ip & 63);
#pragma unroll
    for (int r = 0; r < kWidePf; ++r) {
      const int e = tid + r * kWideThreads;
      if (e < kWideChunk * WR) pf[r] = rowp[(e / kWideChunk) * 64];
    }
    if (tid < kWideChunk) {
      pf_own = a.c[min(i0 + tid, (int64_t)a.n - 1)];
      pf_oc = a.counts[pf_own];
    }
    if (tid < 64) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = tid + 64 * r;
        const int64_t ie = i0 * m1 + e;
        pf_raw[r] = (e < kWideChunk * m1 && ie < (int64_t)a.n * m1) ? a.raw[ie] : 0u;
      }
    }
  };
  auto stage = [&](int par) {
#pragma unroll
    for (int r = 0; r < kWidePf; ++r) {
      const int e = tid + r * kWideThreads;
      if (e < kWideChunk * WR) s_rows0[par * wide_rows_words(WB, WS) + (e & (kWideChunk - 1)) * RS + e / kWideChunk] = pf[r];
    }
    if (tid < kWideChunk) {
      s_own[par][tid] = pf_own;
      s_oc[par][tid] = pf_oc;
    }
    if (tid < 64) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (tid + 64 * r < kWideChunk * m1) s_raw[par][tid + 64 * r] = pf_raw[r];
    }
  };
  // chunks c = blockIdx.x + k gridDim.x, two ahead.  claim != 0: claimed from a counter
  // (k_cluster_summary zeroes it) instead, so a workgroup that starts late leaves its share to
  // the others -- but every claim is a same-address device atomic, and at C4 (4,400 chunks on
  // 1,024 workgroups) they took the kernel from 50 to 80 us (profiles/r04/r5)
  __shared__ int s_cl[2];
  if (tid == 0) {
    s_cl[0] = claim ? atomicAdd(a.wide_ctr, 1) : (int)blockIdx.x;
    s_cl[1] = claim ? atomicAdd(a.wide_ctr, 1) : (int)(blockIdx.x + gridDim.x);
  }
  __syncthreads();
  int c = s_cl[0];
  if (c < nchunks) {
    fetch(c);
    stage(0);
  }
  WideRow<WB, NW> xr;
  xr.WS = WS;
#pragma unroll
  for (int k = 0; k < NW; ++k) xr.val[k] = w + 16 * k < WS;
  int par = 0;
  // the chunk's margins, row positions and ordered compaction (one list block per chunk), by
  // wave 0 at the top of the next iteration (one barrier per chunk)
  auto finish = [&](int cf, int pf_) {
    const int64_t f0 = (int64_t)a.p0 + (int64_t)cf * kWideChunk;
    const int fn = (int)min((int64_t)kWideChunk, (int64_t)a.n - f0);
    const bool on = tid < fn;
    const double mgp = on ? s_mg[pf_][tid] : -INFINITY;
    const int ocp = on ? s_oc[pf_][tid] : 0;
    // the categorical draw from the chunk's staged draws (still in buffer pf_: the next chunk
    // is staged there only after this); a global load here held the other waves at the barrier
    const bool uncertain =
        on && !(ocp >= 2 && (mgp > a.thresh ||
                             stay_by_uniform_call(mgp - a.dmax2, s_raw[pf_][(on ? tid : 0) * m1 + a.m], a.K + a.m)));
    const int64_t i = f0 + tid;
    if (on) a.margin[i] = mgp;
    const unsigned long long bal = __ballot(uncertain);
    const int row = cf * kWideChunk + __popcll(bal & ((1ull << tid) - 1ull));
    if (on) a.rowpos[i] = uncertain ? row : -1;
    if (uncertain) a.list[row] = (int)i;
    if (tid == 0) a.cnt[cf] = __popcll(bal);
  };
  int cprev = -1;
  int it = 0;
#pragma unroll 1
  for (; c < nchunks; par ^= 1, ++it) {
    __syncthreads();                          // the chunk is staged; the previous chunk's margins are in
    if (cprev >= 0 && tid < 64) finish(cprev, par ^ 1);
    // the next chunk (claimed an iteration ago); claim the one after it
    const int cn = s_cl[(it + 1) & 1];
    if (tid == 0) s_cl[it & 1] = cn < nchunks ? (claim ? atomicAdd(a.wide_ctr, 1) : cn + (int)gridDim.x) : nchunks;
    if (cn < nchunks) fetch(cn);
    const int64_t i0 = (int64_t)a.p0 + (int64_t)c * kWideChunk;
    const int npts = (int)min((int64_t)kWideChunk, (int64_t)a.n - i0);
    const bool act = g < npts;
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
      for (int b = 0; b < WB; ++b)
        xr.x[k][b] = xr.val[k] ? s_rows0[par * wide_rows_words(WB, WS) + g * RS + b * WS + w + 16 * k] : 0ull;
    const int own = s_own[par][g];
    const int own_cnt = s_oc[par][g];
    double mg = -INFINITY;
    if (act && own_cnt >= 2) {                // group-uniform
      const uint32_t* raw = s_raw[par] + g * m1;
      // the first latent heads' gathers go out first (their latency overlaps the own-cluster
      // bound and the cluster loop)
      constexpr int LW = WB * NW;
      constexpr int NPF = LW <= 2 ? 3 : LW <= 8 ? 2 : 1;   // heads in flight (register budget: 4 waves at wb 4)
      uint64_t Hd[NPF][LW + 2];
      int pe[NPF];                            // entry of the pick
      const bool heads = a.pool_head != nullptr;
      auto gather = [&](int u, int l) {
        const int e = (int)pick_entry(raw[l], a.P);
        pe[u] = e;
        if (heads) {
          const int hb = e * HS * 8;
#pragma unroll
          for (int k = 0; k < NW; ++k)
#pragma unroll
            for (int b = 0; b < WB; ++b) Hd[u][k * WB + b] = bload(r_head, hb + w8 + 128 * k, 8 * b * WS);
          Hd[u][LW] = bload(r_head, hb, 8 * WR);
          Hd[u][LW + 1] = bload(r_head, hb, 8 * (WR + 1));
        }
      };
#pragma unroll
      for (int u = 0; u < NPF; ++u)
        if (u < a.m) gather(u, u);
      uint64_t M[NW];
      double lo;
      // the own cluster's record: its copy among the cluster summaries in LDS (CL; a lane per
      // summary, 16 at a time), so no global-memory latency precedes the cluster loop; the
      // slot's record otherwise
      int lown = -1;
      if constexpr (CL) {
        for (int l0 = 0; l0 < a.K; l0 += 16) {
          const int l = l0 + w;
          const unsigned long long hb = __ballot(l < a.K && (int)s_cs[l * cw + bw + 1] == own);
          const unsigned gb = (unsigned)(hb >> (16 * (g & 3))) & 0xFFFFu;
          if (gb) {
            lown = l0 + __ffs((int)gb) - 1;
            break;
          }
        }
      }
      if (lown >= 0) {
        const uint64_t* rec = s_cs + lown * cw;
        auto ld = [&](int k, int q) { return rec[q + w + 16 * k]; };
        const int H = xr.mismatch(ld, M);
        const int Sq = xr.penalty(ld, M);
        const double A = as_f64(rec[SC]), dl = as_f64(rec[SC + 1]);
        const double pmax = dl * (double)(Sq + H);
        lo = a.logn[own_cnt - 1] + (A - pmax - kBoundEps * (1.0 + fabs(A) + pmax));
      } else {
        const int ob = own * bw * 8;
        auto ld = [&](int k, int q) { return bload(r_slot, ob + w8 + 128 * k, 8 * q); };
        const int H = xr.mismatch(ld, M);
        const int Sq = xr.penalty(ld, M);
        const double A = as_f64(bload(r_slot, ob, 8 * SC)), dl = as_f64(bload(r_slot, ob, 8 * (SC + 1)));
        const double pmax = dl * (double)(Sq + H);
        lo = a.logn[own_cnt - 1] + (A - pmax - kBoundEps * (1.0 + fabs(A) + pmax));
      }
      const double cut = lo - a.thresh;
      double ubmax = -INFINITY;
#pragma unroll 1
      for (int l = 0; l < a.K; ++l) {
        // wave-uniform record: LDS (CL) or the csum buffer
        auto ldc = [&](int q) -> uint64_t {
          if constexpr (CL) return s_cs[l * cw + q];
          else return bload(r_csum, 0, 8 * (l * cw + q));
        };
        auto ld = [&](int k, int q) -> uint64_t {
          if constexpr (CL) return s_cs[l * cw + q + w + 16 * k];
          else return bload(r_csum, w8 + 128 * k, 8 * (l * cw + q));
        };
        const int s = (int)ldc(bw + 1);
        if (s == own) continue;               // group-uniform
        const int H = xr.mismatch(ld, M);
        const double A = as_f64(ldc(SC)), dmin = as_f64(ldc(SC + 2)), scale = as_f64(ldc(SC + 3));
        const double lg = as_f64(ldc(bw));
        double ub = lg + (A - dmin * (double)H + kBoundEps * (1.0 + scale));
        if (ub > cut) {
          const int Sq = xr.penalty(ld, M);
          const double dl = as_f64(ldc(SC + 1));
          const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
          ub = fmin(ub, lg + (A - pmin + kBoundEps * (1.0 + fabs(A) + pmax)));
        }
        ubmax = fmax(ubmax, ub);
      }
#pragma unroll 1
      for (int l0 = 0; l0 < a.m; l0 += NPF) {
        if (l0 > 0) {
#pragma unroll
          for (int u = 0; u < NPF; ++u)
            if (l0 + u < a.m) gather(u, l0 + u);
        }
#pragma unroll
        for (int u = 0; u < NPF; ++u) {
          if (l0 + u >= a.m) continue;
          const int rb = pe[u] * bw * 8;
          auto ldr = [&](int k, int q) { return bload(r_pool, rb + w8 + 128 * k, 8 * q); };
          double ub;
          if (heads) {
            int h = 0;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
              uint64_t mm = 0;
#pragma unroll
              for (int b = 0; b < WB; ++b) mm |= xr.x[k][b] ^ Hd[u][k * WB + b];
              mm = xr.val[k] ? mm : 0ull;
              M[k] = mm;
              h += __popcll(mm);
            }
            const int H = row_sum16(h);
            const uint64_t p0 = Hd[u][LW], p1 = Hd[u][LW + 1];
            const double A = (double)__uint_as_float((uint32_t)p0), dmn = (double)__uint_as_float((uint32_t)(p0 >> 32));
            const double sa = (double)__uint_as_float((uint32_t)p1), sb = (double)__uint_as_float((uint32_t)(p1 >> 32));
            double low = dmn * (double)H;
            if (H >= a.head_ha) low = fmax(low, sa + dmn * (double)(H - a.head_ha));
            if (H >= a.head_hb) low = fmax(low, sb + dmn * (double)(H - a.head_hb));
            ub = a.logfac + (A - low + kBoundEps * (1.0 + fabs(A) + low));
            if (ub > cut) {
              const int Sq = xr.penalty(ldr, M);
              const double Af = as_f64(bload(r_pool, rb, 8 * SC)), dl = as_f64(bload(r_pool, rb, 8 * (SC + 1)));
              const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
              ub = fmin(ub, a.logfac + (Af - pmin + kBoundEps * (1.0 + fabs(Af) + pmax)));
            }
          } else {
            const int H = xr.mismatch(ldr, M);
            const int Sq = xr.penalty(ldr, M);
            const double Af = as_f64(bload(r_pool, rb, 8 * SC)), dl = as_f64(bload(r_pool, rb, 8 * (SC + 1)));
            const double pmin = dl * (double)Sq, pmax = dl * (double)(Sq + H);
            ub = a.logfac + (Af - pmin + kBoundEps * (1.0 + fabs(Af) + pmax));
          }
          ubmax = fmax(ubmax, ub);
        }
      }
      mg = lo - ubmax;
    }
    if (w == 0) s_mg[par][g] = mg;
    // the next chunk into the other buffers (wave 0 stages its labels / draws only after it
    // finished the previous chunk from them, above)
    if (cn < nchunks) stage(par ^ 1);
    cprev = c;
    c = cn;
  }
  __syncthreads();
  if (cprev >= 0 && tid < 64) finish(cprev, par ^ 1);
}

// Workgroups of k_prepass_wide in flight on the whole GPU (persistent grid).
template <class F>
static int wide_grid(F kern, size_t lds, int want) {
  const int cus = device_cus();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kWideThreads, lds) != hipSuccess || per <= 0) per = 1;
  if (want > 0) per = std::min(per, want);
  // HDPM_WIDE_WGS: workgroups per CU (A/B of the persistent grid)
  static const int ovr = [] {
    const char* e = std::getenv("HDPM_WIDE_WGS");
    return e ? std::atoi(e) : 0;
  }();
  if (ovr > 0 && ovr <= 32) per = ovr;
  return cus * per;
}

int prepass_list_block(const PrepassArgs& a) {
  return (a.wide && wide_fits(a.wb, a.Ws) && prepass_wide_offsets_fit(a)) ? kWideChunk : kBlock;
}

// Block offsets of the prepass lists and the dense, index-ordered list of uncertain rows
// (row = list block * its points (kBlock, or kWideChunk) + position), so the serial resolver reads it 64 at a time
// instead of walking every block count.  One workgroup of 1024 threads.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_list_scan(const int* __restrict__ cnt, int nblocks, int lblock,
                                                           int* __restrict__ dense, int* __restrict__ total) {
  __shared__ int s_sum[kScanThreads / kWave];
  const int tid = threadIdx.x;
  const int chunk = (nblocks + kScanThreads - 1) / kScanThreads;
  const int b0 = min(nblocks, tid * chunk), b1 = min(nblocks, b0 + chunk);
  int mine = 0;
  for (int b = b0; b < b1; ++b) mine += cnt[b];
  // block-wide exclusive scan of `mine`
  const int lane = tid & 63, wv = tid >> 6;
  int inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_sum[wv] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / kWave; ++w) {
    base += w < wv ? s_sum[w] : 0;
    all += s_sum[w];
  }
  int off = base + inc - mine;
  for (int b = b0; b < b1; ++b) {
    const int c = cnt[b];
    for (int q = 0; q < c; ++q) dense[off + q] = b * lblock + q;
    off += c;
  }
  if (tid == 0) *total = all;
}

// Long lists (~1M rows from a random start): the block offsets by one workgroup, then the
// dense list written by a wave per list block, coalesced (k_list_scan's per-thread runs of
// scattered stores cost ~0.3 ms at 1M rows).
__global__ __launch_bounds__(kScanThreads) void k_list_offsets(const int* __restrict__ cnt, int nblocks,
                                                              int* __restrict__ boff, int* __restrict__ total) {
  __shared__ int s_sum[kScanThreads / kWave];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int chunk = (nblocks + kScanThreads - 1) / kScanThreads;
  const int b0 = min(nblocks, tid * chunk), b1 = min(nblocks, b0 + chunk);
  int mine = 0;
  for (int b = b0; b < b1; ++b) mine += cnt[b];
  int inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_sum[wv] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / kWave; ++w) {
    base += w < wv ? s_sum[w] : 0;
    all += s_sum[w];
  }
  int off = base + inc - mine;
  for (int b = b0; b < b1; ++b) {
    boff[b] = off;
    off += cnt[b];
  }
  if (tid == 0) *total = all;
}

// (rq: also the resolver's per-point records (row, point, slot, categorical draw), which
// k_exact_rows_mass reads instead of walking row -> point -> label itself)
__global__ __launch_bounds__(256) void k_list_fill(PrepassArgs a, int want_rq) {
  if (!pipe_gate(a)) return;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= a.nlb) return;
  const int n = a.cnt[b], o = a.boff[b], m1 = a.m + 1;
  for (int q = lane; q < n; q += kWave) {
    const int row = b * a.lblock + q;
    a.dense[o + q] = row;
    if (want_rq) {
      const int i = a.list[row];
      a.rq[o + q] = make_int4(row, i, a.c[i], (int)a.raw[(int64_t)i * m1 + m1 - 1]);
    }
  }
}

// ------------------------------------------------------------------ resolver
// One wave walks the sweep in index order.  State (counts, label<->slot maps, the log
// counts logn[cnt] and logn[cnt - 1] per slot) lives in LDS, so a decision touches global
// memory only for its exact row, which is prefetched one point ahead into an LDS double
// buffer, and its label / categorical draw, which are loaded 64 points at a time.
// The resolver is a single wave: LDS ops of one wave complete in order, so a
// compiler-ordering point plus an LDS wait replaces the workgroup barrier (and, unlike
// __syncthreads, leaves prefetched global loads in flight).
__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct RShared {
  int K, nslots, status, next, restart, moves, exact, checked, pick, src, nstruct, aborted;
  double dnow, sum;
  double dvmax;        // max over slots of |logn[count] - logn[snapshot count]|
  double pad;
  long long tsub[8];   // diagnostics (resolver profiling)
  int bgo, bq;         // block mode: continue flag, next dense-list position
};
constexpr int kRSharedBytes = 192;
static_assert(sizeof(RShared) <= kRSharedBytes, "RShared");

// Block mode (k_resolve_blk, one wave, for a chain far from convergence: most points
// uncertain): the next kBlk listed points are drawn together, one lane per point, in the
// state at the block start (the reference's draw run literally per lane, revsort included);
// then, still in parallel, each point's draw is kept while no log-weight of it has moved by
// its radius -- a bound from the count changes of the points before it in the block -- and
// the block commits its points up to the first draw that is not kept or the first
// structural move (case 2 relabels, cases 3 / 4 take a new slot and end the launch, both
// processed by the serial path).  A block's first draw is always kept.
constexpr int kBlk = 64;
constexpr int kRqWin = 512;

struct RState {
  RShared* sh;
  int lcap, emax;
  int* cnt;     // [lcap]
  int* snap;    // [lcap]
  int* sol;     // [lcap] slot_of_label
  int* los;     // [lcap] label_of_slot
  double* l1;   // [lcap] logn[cnt]
  double* l0;   // [lcap] logn[cnt - 1]
  double* val;  // [emax]
  double* p;    // [emax]
  double* row;  // [2][emax] exact rows (double buffer)
  int* perm;    // [emax]
  uint64_t* ltab;   // glibc's log table (logn[c] = log(c) on the device, bit for bit)
  // block mode only (nullptr otherwise):
  double* sl1;  // [lcap] logn[snapshot count]
  double* sl0;  // [lcap] logn[snapshot count - 1]
  double* bp;   // [64 entries][64 lanes] per-lane draw scratch (probabilities)
  int* bperm;   // [64][64] per-lane revsort indices
  int* bcmin;   // [kWave] lower bounds on the slot counts during a block's walk
  int4* brq;    // [kRqWin] window of the listed points' inputs {row, point, slot, draw}
};

// LIST mode stages the exact rows of each 64 listed points in LDS ahead of their decisions
// (one load round trip per 64 points instead of one per exact decision) when a row has at
// most kTileCols columns; row stride odd (no bank aliasing between the lanes' rows).
constexpr int kTileCols = 95;
__host__ __device__ inline int resolve_tile_stride(int ncol) { return ncol | 1; }
__host__ __device__ inline size_t resolve_lds_bytes(int lcap, int m, int blocks, int ncol = 0) {
  const size_t emax = (size_t)lcap + (size_t)m;
  size_t b = kRSharedBytes + emax * 4 * sizeof(double) + (size_t)lcap * 2 * sizeof(double) + (size_t)lcap * 4 * sizeof(int) +
             emax * sizeof(int);
  b = (b + 15) & ~(size_t)15;
  b += 256 * sizeof(uint64_t);
  b += (size_t)lcap * 2 * sizeof(double);      // the snapshot's log counts (sl1, sl0)
  if (blocks)
    b += 64 * kWave * (sizeof(double) + sizeof(int)) + kWave * sizeof(int) + 16 + kRqWin * sizeof(int4);
  else if (ncol > 0 && ncol <= kTileCols)
    b += (size_t)kWave * resolve_tile_stride(ncol) * sizeof(double);
  return b;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ double slot_drift(const RState& st, const double* logn, int s) {
  const int a = st.snap[s], b = st.cnt[s];
  if (a >= 2) {
    if (b < 2) return INFINITY;
    return fabs(st.l0[s] - (st.sl0 ? st.sl0[s] : logn[a - 1]));   // logn[b - 1] - logn[a - 1]
  }
  if (a == 1) return b == 0 ? 0.0 : st.l1[s];
  return INFINITY;
}

// |logn[count] - logn[snapshot count]| of slot s (inf when either count is 0)
__device__ __forceinline__ double count_drift(const RState& st, const double* logn, int s) {
  const int a = st.snap[s], b = st.cnt[s];
  if (a == b) return 0.0;
  if (a < 1 || b < 1) return INFINITY;
  return fabs(st.l1[s] - (st.sl1 ? st.sl1[s] : logn[a]));
}



// lane 0: record a reassignment for the incremental frequency tables
__device__ __forceinline__ void log_move(const ResolveArgs& a, int& nlog, int64_t i, int from, int to) {
  if (a.mlog) {
    a.mlog[3 * nlog] = (int)i;
    a.mlog[3 * nlog + 1] = from;
    a.mlog[3 * nlog + 2] = to;
    ++nlog;
  }
}

// logn[c] = log((double) c) as the host's table holds it (glibc's algorithm, LDS table)
__device__ __forceinline__ double logn_dev(const RState& st, int c) {
  return c <= 0 ? -INFINITY : glibc::log_r((double)c, st.ltab);
}

// lane 0: slot s's count changed -> refresh its log-count cache.  A count moves by one per
// reassignment, so one of the two values is the other's old one; the new one is computed
// (no dependent global load on the resolver's serial path).
__device__ __forceinline__ void set_count(const RState& st, const double* logn, int s, int c) {
  (void)logn;
  const int old = st.cnt[s];
  st.cnt[s] = c;
  if (c == old) return;
  if (c == old - 1) {
    st.l1[s] = st.l0[s];
    st.l0[s] = logn_dev(st, c - 1);
  } else if (c == old + 1) {
    st.l0[s] = st.l1[s];
    st.l1[s] = logn_dev(st, c);
  } else {
    st.l1[s] = logn_dev(st, c);
    st.l0[s] = logn_dev(st, c - 1);
  }
}

// Serial revsort (R sort.c) on lane 0.
__device__ void dev_revsort(double* a0, int* ib0, int n) {
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

// R's revsort on one lane's column of a [n][kWave] LDS array (a0, ib0 point at the lane's
// entry 0; entry e at e * kWave): the same operations as dev_revsort.
__device__ void lane_revsort(double* a0, int* ib0, int n) {
  if (n <= 1) return;
  auto A = [&](int x) -> double& { return a0[(x - 1) * kWave]; };
  auto B = [&](int x) -> int& { return ib0[(x - 1) * kWave]; };
  int l = (n >> 1) + 1, ir = n, i, j, ii;
  double ra;
  for (;;) {
    if (l > 1) {
      l = l - 1;
      ra = A(l);
      ii = B(l);
    } else {
      ra = A(ir);
      ii = B(ir);
      A(ir) = A(1);
      B(ir) = B(1);
      if (--ir == 1) {
        A(1) = ra;
        B(1) = ii;
        return;
      }
    }
    i = l;
    j = l << 1;
    while (j <= ir) {
      if (j < ir && A(j) > A(j + 1)) ++j;
      if (ra > A(j)) {
        A(i) = A(j);
        B(i) = B(j);
        j += (i = j);
      } else {
        j = ir + 1;
      }
    }
    A(i) = ra;
    B(i) = ii;
  }
}

// Walker's alias draw (Rcpp sugar WalkerSample, R random.c walker_ProbSampleReplace) for
// n > 200 effective categories, serial on one lane: q holds the FixupProb-normalised
// probabilities (overwritten with the table), w is scratch packing the alias (low 16 bits)
// and the small/large work list HL (high 16 bits) of each entry; n < 65536.  One uniform u:
// rU = u n, k = (int) rU, k if rU < q[k] + k else alias[k].  Same operations as the host's
// walker_table / sample_prob1_pick (rmath.hpp) and the oracle.
__device__ int dev_walker(double* q, int* w, int n, double u) {
  auto hl = [&](int pos) { return (int)((unsigned)w[pos] >> 16); };
  auto set_hl = [&](int pos, int v) { w[pos] = (int)(((unsigned)w[pos] & 0xffffu) | ((unsigned)v << 16)); };
  auto set_a = [&](int i, int v) { w[i] = (int)(((unsigned)w[i] & 0xffff0000u) | (unsigned)v); };
  for (int i = 0; i < n; i++) w[i] = i;
  int h = -1, l = n;
  for (int i = 0; i < n; i++) {
    q[i] = q[i] * n;
    if (q[i] < 1.) set_hl(++h, i); else set_hl(--l, i);
  }
  if (h >= 0 && l < n) {
    for (int k = 0; k < n - 1; k++) {
      const int i = hl(k), j = hl(l);
      set_a(i, j);
      q[j] += q[i] - 1;
      if (q[j] < 1.) l++;
      if (l >= n) break;
    }
  }
  for (int i = 0; i < n; i++) q[i] += i;
  const double rU = u * n;
  const int k = (int)rU;
  return rU < q[k] ? k : (w[k] & 0xffff);
}

__device__ __forceinline__ double readlane_f64(double x, int l) {
  const uint64_t u = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// The n8:95-102 draw from the log-weights pv (entry e in lane e % 64 of register e / 64,
// E entries), categorical uniform rU.  Returns the drawn index in [0, E) or -status.
// The reference's left-to-right reductions -- the max, sum(probs) (n8:96) and Rcpp
// FixupProb's sum of the positive entries -- run in index order over readlane'd values,
// so they round exactly as on the CPU.  The loops run over E rounded up to 8 with padding
// entries -inf / 0.0, which leave a max or a non-negative running sum unchanged.  Counts,
// the maximum's position and ties come from ballots; ties or a draw past the maximum take
// R's revsort on lane 0 (LDS scratch lp / lperm, result through *lpick).
//
// With `rad` (the snapshot draws of k_exact_rows), *rad receives a radius: the draw is
// unchanged when every log-weight moves by less than *rad (normalised probabilities then
// move by factors within exp(+-2 rad)): the chosen entry keeps its place in revsort's order
// (ratios to its neighbours) and the uniform stays inside its cumulative interval.  0 when
// no such bound is kept (ties, the Walker threshold in reach).
template <int RE, bool kOcml = false>
__device__ int decide_values(double (&pv)[RE], int E, double rU, double* lp, int* lperm, int* lpick,
                             double* rad = nullptr) {
  if (rad) *rad = 0.0;
  const int lane = threadIdx.x & 63;
  E = __builtin_amdgcn_readfirstlane(E);
  const int E8 = (E + 7) & ~7;
  auto scan = [&](double acc, auto f) -> double {
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const int lim = min(kWave, E8 - r * kWave);
      for (int e0 = 0; e0 < lim; e0 += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = f(acc, readlane_f64(pv[r], e0 + k));
      }
    }
    return acc;
  };
#pragma unroll
  for (int r = 0; r < RE; ++r)
    if (r * kWave + lane >= E) pv[r] = -INFINITY;
  // max is order-free: a butterfly instead of the sequential scan
  double mx = pv[0];
#pragma unroll
  for (int r = 1; r < RE; ++r) mx = fmax(mx, pv[r]);
  mx = wave_max(mx);
#pragma unroll
  for (int r = 0; r < RE; ++r) pv[r] = (r * kWave + lane < E) ? dexp<kOcml>(pv[r] - mx) : 0.0;  // n8:95
  const double sum = scan(0.0, [](double s, double x) { return s + x; });
#pragma unroll
  for (int r = 0; r < RE; ++r) pv[r] = pv[r] / sum;                                             // n8:96
  const double s2 = scan(0.0, [](double s, double x) { return s + (x > 0 ? x : 0.0); });       // FixupProb
  if (!(s2 > 0)) return -3;  // kProb: no positive probability
  int nc = 0;
#pragma unroll
  for (int r = 0; r < RE; ++r) {
    const bool in = r * kWave + lane < E;
    pv[r] = in ? pv[r] / s2 : 0.0;
    nc += __popcll(__ballot(in && (double)E * pv[r] > 0.1));
  }
  if (nc > 200) {          // Walker's alias method (Rcpp sample() with > 200 categories)
#pragma unroll
    for (int r = 0; r < RE; ++r)
      if (r * kWave + lane < E) lp[r * kWave + lane] = pv[r];
    wave_sync();
    if (lane == 0) *lpick = dev_walker(lp, lperm, E, rU);
    wave_sync();
    return *lpick;
  }
  double pmax = pv[0];
#pragma unroll
  for (int r = 1; r < RE; ++r) pmax = fmax(pmax, pv[r]);
  pmax = wave_max(pmax);
  int ties = 0, amax = -1;
#pragma unroll
  for (int r = 0; r < RE; ++r) {
    const unsigned long long b = __ballot(r * kWave + lane < E && pv[r] == pmax);
    ties += __popcll(b);
    if (amax < 0 && b) amax = r * kWave + __ffsll((long long)b) - 1;
  }
  // Unique maximum drawn: revsort puts it first, cumsum[0] = pmax.
  if (ties == 1 && rU <= pmax) {
    if (rad && E <= 200) {
      double p2 = -1.0;
#pragma unroll
      for (int r = 0; r < RE; ++r)
        if (r * kWave + lane < E && r * kWave + lane != amax) p2 = fmax(p2, pv[r]);
      p2 = wave_max(p2);
      const double r1 = p2 > 0 ? 0.5 * log(pmax / p2) : INFINITY;
      *rad = fmax(0.0, fmin(r1, 0.5 * log(pmax / rU)) - 1e-9);
    }
    return amax;
  }
  // Positive entries with distinct values: revsort (a heapsort) leaves them in plain
  // descending order, so an entry's position is its rank, and the cumulative sums run
  // over that order with the serial loop's additions.  Ties among positive entries, or a
  // draw past the last positive entry (it would land among the zeros, whose order is
  // heapsort's tie handling), take the serial revsort below.
  if (ties == 1) {
    int rank[RE];
    bool tie = false;
#pragma unroll
    for (int r = 0; r < RE; ++r) rank[r] = 0;
#pragma unroll
    for (int r2 = 0; r2 < RE; ++r2) {
      const int lim = min(kWave, E - r2 * kWave);
      for (int l = 0; l < lim; ++l) {
        const double x = readlane_f64(pv[r2], l);
#pragma unroll
        for (int r = 0; r < RE; ++r) {
          rank[r] += x > pv[r] ? 1 : 0;
          tie |= x == pv[r] && pv[r] > 0 && (r2 != r || l != lane);
        }
      }
    }
    int npos = 0;
#pragma unroll
    for (int r = 0; r < RE; ++r) npos += __popcll(__ballot(r * kWave + lane < E && pv[r] > 0));
    if (!__ballot(tie)) {
#pragma unroll
      for (int r = 0; r < RE; ++r)
        if (r * kWave + lane < E && pv[r] > 0) {
          lp[rank[r]] = pv[r];
          lperm[rank[r]] = r * kWave + lane;
        }
      wave_sync();
      int pick = -1, jp = 0;
      double c = 0.0, cprev = 0.0;
      for (int j0 = 0; j0 < npos && pick < 0; j0 += 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = j0 + k < npos ? lp[j0 + k] : 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int j = j0 + k;
          if (pick >= 0 || j >= npos) break;
          cprev = c;
          c += v[k];
          if (j == E - 1 || rU <= c) { pick = lperm[j]; jp = j; }
        }
      }
      if (rad && pick >= 0 && E <= 200) {
        const double pj = lp[jp];
        double r = INFINITY;
        if (jp > 0) r = fmin(r, fmin(0.5 * log(lp[jp - 1] / pj), 0.5 * log(rU / cprev)));
        if (jp + 1 < npos) r = fmin(r, 0.5 * log(pj / lp[jp + 1]));
        if (jp != E - 1) r = fmin(r, 0.5 * log(c / rU));
        *rad = fmax(0.0, r - 1e-9);
      }
      wave_sync();   // lp / lperm are reused by the next decision
      if (pick >= 0) return pick;
    }
  }
#pragma unroll
  for (int r = 0; r < RE; ++r)
    if (r * kWave + lane < E) lp[r * kWave + lane] = pv[r];
  wave_sync();
  if (lane == 0) {
    for (int e = 0; e < E; ++e) lperm[e] = e + 1;
    dev_revsort(lp, lperm, E);
    for (int e = 1; e < E; ++e) lp[e] += lp[e - 1];
    int j;
    for (j = 0; j < E - 1; j++)
      if (rU <= lp[j]) break;
    *lpick = lperm[j] - 1;
  }
  wave_sync();
  return *lpick;
}

// Exact n8:40-102 decision for a point whose exact row is Lr (LDS), own slot `own`, in the
// resolver's current state.  Returns the drawn index in [0, K+m) or -status.
template <int RE>
__device__ int exact_decision_reg(const ResolveArgs& a, const RState& st, int K, const double* Lr, int own, double rU) {
  const int lane = threadIdx.x & 63;
  K = __builtin_amdgcn_readfirstlane(K);
  own = __builtin_amdgcn_readfirstlane(own);
  const int E = K + a.m;
  const bool singleton = st.cnt[own] == 1;
  double pv[RE];
#pragma unroll
  for (int r = 0; r < RE; ++r) {
    const int e = r * kWave + lane;
    double v = -INFINITY;
    if (e < K) {
      const int s = st.sol[e];
      // logn[cnt - (s == own)] + ll; logn[0] = -inf covers the emptied singleton
      v = (s == own ? st.l0[s] : st.l1[s]) + Lr[s];
    } else if (e < E) {
      const int l = e - K;
      v = a.logfac + ((l == 0 && singleton) ? Lr[own] : Lr[a.S + l]);
    }
    pv[r] = v;
  }
  return decide_values<RE>(pv, E, rU, st.p, st.perm, &st.sh->pick);
}

// LDS path for more than 256 entries.
__device__ int exact_decision_lds(const ResolveArgs& a, const RState& st, int K, const double* Lr, int own,
                                  double rU) {
  const int lane = threadIdx.x & 63;
  const int E = K + a.m;
  const bool singleton = st.cnt[own] == 1;
  double mx = -INFINITY;
  for (int e = lane; e < E; e += kWave) {
    double v;
    if (e < K) {
      const int s = st.sol[e];
      v = (s == own ? st.l0[s] : st.l1[s]) + Lr[s];
    } else {
      const int l = e - K;
      v = a.logfac + ((l == 0 && singleton) ? Lr[own] : Lr[a.S + l]);
    }
    st.val[e] = v;
    mx = fmax(mx, v);
  }
  mx = wave_max(mx);
  for (int e = lane; e < E; e += kWave) st.p[e] = dexp(st.val[e] - mx);
  wave_sync();
  if (lane == 0) {
    double sum = 0.0;
    for (int e = 0; e < E; ++e) sum += st.p[e];
    st.sh->sum = sum;
  }
  wave_sync();
  const double sum = st.sh->sum;
  for (int e = lane; e < E; e += kWave) st.p[e] = st.p[e] / sum;
  wave_sync();
  if (lane == 0) {
    double s2 = 0.0;
    for (int e = 0; e < E; ++e) if (st.p[e] > 0) s2 += st.p[e];
    st.sh->sum = s2;
  }
  wave_sync();
  const double s2 = st.sh->sum;
  if (!(s2 > 0)) return -3;
  int nc = 0;
  for (int e = lane; e < E; e += kWave) {
    const double q = st.p[e] / s2;
    st.p[e] = q;
    nc += ((double)E * q > 0.1) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o);
  wave_sync();
  if (nc > 200) {          // Walker's alias method
    if (lane == 0) st.sh->pick = dev_walker(st.p, st.perm, E, rU);
    wave_sync();
    return st.sh->pick;
  }
  if (lane == 0) {
    for (int e = 0; e < E; ++e) st.perm[e] = e + 1;
    dev_revsort(st.p, st.perm, E);
    for (int e = 1; e < E; ++e) st.p[e] += st.p[e - 1];
    int j;
    for (j = 0; j < E - 1; j++)
      if (rU <= st.p[j]) break;
    st.sh->pick = st.perm[j] - 1;
  }
  wave_sync();
  return st.sh->pick;
}

__device__ int exact_decision(const ResolveArgs& a, const RState& st, int K, const double* Lr, int own, double rU) {
  const int E = __builtin_amdgcn_readfirstlane(K) + a.m;
  if (E <= kWave) return exact_decision_reg<1>(a, st, K, Lr, own, rU);
  if (E <= 4 * kWave) return exact_decision_reg<4>(a, st, K, Lr, own, rU);
  return exact_decision_lds(a, st, K, Lr, own, rU);
}

__device__ void copy_pool_params(const ResolveArgs& a, int64_t e, int s) {
  const int lane = threadIdx.x & 63;
  const int dp = a.dp;
  for (int b = lane; b < dp; b += kWave) a.slot_codes[(int64_t)s * dp + b] = a.pool.codes[e * dp + b];
  for (int b = lane; b < 2 * a.d; b += kWave) a.slot_tab[(int64_t)s * 2 * a.d + b] = a.pool.tab[e * 2 * a.d + b];
  for (int b = lane; b < a.bw; b += kWave) a.slot_bnd[(int64_t)s * a.bw + b] = a.pool_bnd[e * a.bw + b];
}

// The snapshot draw of an uncertain point from its row (acc_r: entry e in lane e % 64 of
// register e / 64), with the resolver's exact decision (one wave).
template <int RE>
__device__ void exact_rows_decide(const PrepassArgs& a, int q, int64_t i, const uint32_t* raw, double (&acc_r)[RE],
                                  double* lp, int* lperm, int* lpick) {
  const int lane = threadIdx.x & 63;
  const int E = a.K + a.m;
  {
    if (!a.spec) return;
    // n8:40-94 in the snapshot state: logn[count - (slot == own)] + ll for the clusters,
    // log(gamma / m) + ll for the latents (the singleton's first latent is its own cluster)
    const int own = __builtin_amdgcn_readfirstlane(a.c[i]);
    const int own_cnt = a.counts[own];
    double ll_own = 0.0;
    double pv[RE];
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const int e = r * kWave + lane;
      int s = -1;
      if (e < a.K) s = a.slot_of_label[e];
      const unsigned long long bo = __ballot(s == own);
      if (bo) ll_own = readlane_f64(acc_r[r], __ffsll((long long)bo) - 1);
      double v = -INFINITY;
      if (e < a.K) v = a.logn[a.counts[s] - (s == own ? 1 : 0)] + acc_r[r];
      pv[r] = v;
    }
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const int e = r * kWave + lane;
      if (e >= a.K && e < E) {
        const int l = e - a.K;
        pv[r] = a.logfac + ((l == 0 && own_cnt == 1) ? ll_own : acc_r[r]);
      }
    }
    double rad = 0.0;
    const int pick = decide_values<RE>(pv, E, raw_to_unif(raw[a.m]), lp, lperm, lpick, &rad);
    if (lane == 0) {
      a.spec[q] = pick >= 0 ? pick : -1;
      a.spec_rad[q] = rad;
    }
  }
}

// Exact rows of the uncertain points: one wave per point (grid-stride over the dense
// list), lane e computes entry e's log-likelihood, adding its per-attribute dhamming
// values in attribute order -- the reference's summation order (n8:47-49), so every row
// is bit-exact.  The point's codes are wave-uniform (scalar loads); each lane reads its
// entry's codes 16 at a time and gathers the 32 table values of two chunks before adding
// them, so the loads overlap.
//
// Speculation: the same wave then draws the point in the snapshot state (the counts and
// slots every row of this round was built against) with the resolver's exact decision.
// While no earlier point of the round has moved, the resolver's state IS the snapshot,
// so it takes these draws as they are; after the first move it decides on its own.
template <int RE>
__device__ void exact_rows_point(const PrepassArgs& a, int q, int row, double* lp, int* lperm, int* lpick) {
  const int lane = threadIdx.x & 63;
  const int E = a.K + a.m;
  const int dp = a.nq * 16;
  const int64_t i = a.list[row];
  const uint32_t* raw = a.raw + i * (a.m + 1);
  double* Lr = a.L + (int64_t)row * (a.S + a.m);
  auto entry_ll = [&](int r) -> double {
      const int e = r * kWave + lane;
      const bool on = e < E;
      const uint8_t* cc;
      const double* tab;
      int col;
      if (e < a.K) {
        const int s = a.slot_of_label[e];
        cc = a.slots.codes + (int64_t)s * dp;
        tab = a.slots.tab + (int64_t)s * 2 * a.d;
        col = s;
      } else {
        const int64_t pe = pick_entry(raw[on ? e - a.K : 0], a.P);
        cc = a.pool.codes + pe * dp;
        tab = a.pool.tab + pe * 2 * a.d;
        col = a.S + (e - a.K);
      }
      double acc = 0.0;
      for (int c0 = 0; c0 < a.nq; c0 += 2) {
        double t[32];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = c0 + h;
          uint4 xc = make_uint4(0, 0, 0, 0);
          if (c < a.nq) {
            const uint32_t* xp = (const uint32_t*)(a.codes_t + tiled_offset(i, c * 16, a.nq));
            xc = make_uint4(ldu(xp), ldu(xp + 1), ldu(xp + 2), ldu(xp + 3));
          }
          const uint4 cq = (on && c < a.nq) ? *(const uint4*)(cc + c * 16) : make_uint4(0, 0, 0, 0);
          const uint4 dx = make_uint4(xc.x ^ cq.x, xc.y ^ cq.y, xc.z ^ cq.z, xc.w ^ cq.w);
#pragma unroll
          for (int b = 0; b < 16; ++b) {
            const int j = c * 16 + b;
            t[h * 16 + b] = (on && j < a.d) ? tab[2 * j + (byte_differs(dx, b) ? 1 : 0)] : 0.0;
          }
        }
#pragma unroll
        for (int u = 0; u < 32; ++u)
          if ((c0 * 16 + u) < a.d) acc += t[u];
      }
      if (on) Lr[col] = acc;
      return acc;
  };
  double acc_r[RE > 0 ? RE : 1];
  if constexpr (RE > 0) {
#pragma unroll
    for (int r = 0; r < RE; ++r) acc_r[r] = entry_ll(r);
  } else {
    for (int r = 0; r < (E + kWave - 1) / kWave; ++r) (void)entry_ll(r);
  }
  if constexpr (RE > 0) exact_rows_decide<RE>(a, q, i, raw, acc_r, lp, lperm, lpick);
}

// Independent waves per workgroup (no block-level barrier): a sweep whose points are all
// certain costs one small grid of early exits, not one workgroup per prepass block.
constexpr int kExactWaves = 4;
__global__ __launch_bounds__(kWave * kExactWaves) void k_exact_rows(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  const int total = *a.dense_total;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q0 = blockIdx.x * kExactWaves + wv;
  if (q0 >= total) return;
  __shared__ double lp_w[kExactWaves][4 * kWave];
  __shared__ int lperm_w[kExactWaves][4 * kWave];
  __shared__ int lpick_w[kExactWaves];
  double* lp = lp_w[wv];
  int* lperm = lperm_w[wv];
  int* lpick = &lpick_w[wv];
  const int E = a.K + a.m;
  for (int q = q0; q < total; q += gridDim.x * kExactWaves) {
    const int row = a.dense[q];
    if (lane == 0) {   // the resolver's per-point inputs, in list order
      const int64_t i = a.list[row];
      a.rq[q] = make_int4(row, (int)i, a.c[i], (int)a.raw[i * (a.m + 1) + a.m]);
    }
    if (E <= kWave) exact_rows_point<1>(a, q, row, lp, lperm, lpick);
    else if (E <= 4 * kWave) exact_rows_point<4>(a, q, row, lp, lperm, lpick);
    else {
      exact_rows_point<0>(a, q, row, lp, lperm, lpick);
      if (a.spec && lane == 0) a.spec[q] = -1;
    }
  }
}

// Workgroup per point, when the point's E x D table values fit in LDS: the 256 threads
// gather them all at once (codes 4 attributes at a time, then the selected table value),
// so a row costs one round of gather latency instead of D / 32; wave 0 then adds each
// entry's values in attribute order (the reference's summation order, bit-exact) and
// draws the snapshot decision.  Dynamic LDS: exact_wg_lds_bytes.
constexpr int kExactWgThreads = 256;
constexpr size_t kExactWgLdsMax = 64 * 1024;
__host__ __device__ inline size_t exact_wg_lds_bytes(int E, int d, int dp) {
  return (size_t)E * (d + 1) * 8 + (size_t)E * 16 + (size_t)E * 4 + (size_t)dp + 16;
}

// k_list_scan inside the exact-rows workgroups (one launch less per round): every workgroup
// scans the list blocks' counts in kExactWgThreads chunks (exclusive offsets in s_off);
// workgroup 0 also writes the dense list and its length, which the resolver reads.
__device__ int exact_dense_scan(const PrepassArgs& a, int* s_off) {
  __shared__ int s_w[kExactWgThreads / kWave];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int chunk = (a.nlb + kExactWgThreads - 1) / kExactWgThreads;
  const int b0 = min(a.nlb, t * chunk), b1 = min(a.nlb, b0 + chunk);
  int mine = 0;
  for (int b = b0; b < b1; ++b) mine += a.cnt[b];
  int inc = mine;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) s_w[wv] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kExactWgThreads / kWave; ++w) {
    base += w < wv ? s_w[w] : 0;
    all += s_w[w];
  }
  const int off0 = base + inc - mine;
  s_off[t] = off0;
  if (t == 0) s_off[kExactWgThreads] = all;
  if (blockIdx.x == 0) {
    int off = off0;
    for (int b = b0; b < b1; ++b) {
      const int c = a.cnt[b];
      for (int q = 0; q < c; ++q) a.dense[off + q] = b * a.lblock + q;
      off += c;
    }
    if (t == 0) *a.dense_total = all;
  }
  __syncthreads();
  return all;
}
// row of dense position q: the thread chunk whose offsets hold q, then its blocks
__device__ int exact_dense_row(const PrepassArgs& a, const int* s_off, int q) {
  int lo = 0, hi = kExactWgThreads - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s_off[mid + 1] > q) hi = mid;
    else lo = mid + 1;
  }
  const int chunk = (a.nlb + kExactWgThreads - 1) / kExactWgThreads;
  int b = lo * chunk, off = s_off[lo];
  for (;; ++b) {
    const int c = a.cnt[b];
    if (q < off + c) return b * a.lblock + (q - off);
    off += c;
  }
}

template <int RE>
__global__ __launch_bounds__(kExactWgThreads) void k_exact_rows_wg(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  __shared__ int s_off[kExactWgThreads + 1];
  const int total = a.exact_scan ? *a.dense_total : exact_dense_scan(a, s_off);
  if ((int)blockIdx.x >= total) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double lp[4 * kWave];
  __shared__ int lperm[4 * kWave];
  __shared__ int lpick;
  const int E = a.K + a.m, D = a.d, dp = a.nq * 16, RS = D + 1;   // odd row stride: no bank aliasing
  double* vals = (double*)smem;                                    // [E][RS]
  const uint8_t** ecode = (const uint8_t**)(vals + (size_t)E * RS);
  const double** etab = (const double**)(ecode + E);
  int* ecol = (int*)(etab + E);
  uint8_t* xc = (uint8_t*)(ecol + E);
  const int t = threadIdx.x, lane = t & 63;
  const int nj4 = (D + 3) >> 2;
  for (int q = blockIdx.x; q < total; q += gridDim.x) {
    const int row = a.exact_scan ? a.dense[q] : exact_dense_row(a, s_off, q);
    const int64_t i = a.list[row];
    const uint32_t* raw = a.raw + i * (a.m + 1);
    if (t == 0) a.rq[q] = make_int4(row, (int)i, a.c[i], (int)raw[a.m]);   // the resolver's inputs
    for (int e = t; e < E; e += kExactWgThreads) {
      if (e < a.K) {
        const int s = a.slot_of_label[e];
        ecode[e] = a.slots.codes + (int64_t)s * dp;
        etab[e] = a.slots.tab + (int64_t)s * 2 * D;
        ecol[e] = s;
      } else {
        const int64_t pe = pick_entry(raw[e - a.K], a.P);
        ecode[e] = a.pool.codes + pe * dp;
        etab[e] = a.pool.tab + pe * 2 * D;
        ecol[e] = a.S + (e - a.K);
      }
    }
    for (int j = t; j < dp; j += kExactWgThreads) xc[j] = a.codes_t[tiled_offset(i, j, a.nq)];
    __syncthreads();
    for (int f = t; f < E * nj4; f += kExactWgThreads) {
      const int e = f / nj4, j0 = (f - e * nj4) * 4;
      const uint32_t dx = *(const uint32_t*)(ecode[e] + j0) ^ *(const uint32_t*)(xc + j0);
      const double* tb = etab[e];
      double v[4];
#pragma unroll
      for (int b = 0; b < 4; ++b)
        v[b] = (j0 + b < D) ? tb[2 * (j0 + b) + (((dx >> (8 * b)) & 0xffu) ? 1 : 0)] : 0.0;
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (j0 + b < D) vals[e * RS + j0 + b] = v[b];
    }
    __syncthreads();
    if (t < kWave) {
      double acc_r[RE];
      double* Lr = a.L + (int64_t)row * (a.S + a.m);
#pragma unroll
      for (int r = 0; r < RE; ++r) {
        const int e = r * kWave + lane;
        double acc = 0.0;
        if (e < E) {
          const double* vr = vals + e * RS;
          for (int j = 0; j < D; ++j) acc += vr[j];
          Lr[ecol[e]] = acc;
        }
        acc_r[r] = acc;
      }
      exact_rows_decide<RE>(a, q, i, raw, acc_r, lp, lperm, &lpick);
    }
    __syncthreads();   // the LDS staging is reused by the next point
  }
}

// The resolver's per-launch context (shared by k_resolve and k_resolve_blk): the point
// decisions and state updates run on one wave (lane 0 writes the shared state).
struct RCtx {
  const ResolveArgs& a;
  const RState& st;
  RShared& S;
  int lane, ncol, scap;
  int nlog;    // running move-log length (uniform across the wave)
  bool prof;
  __device__ bool process(int64_t i, int row, int own, uint32_t rawU, int spec, double srad, bool given = false,
                          const double* rowp = nullptr);
  __device__ bool verify(int64_t lo, int64_t hi, double dn_over = -1.0, const int* cmin = nullptr);
};

// Decide point i (exact row in LDS at Lr) and apply n8:107-159.  Returns false to stop
// the sweep here.
__device__ __forceinline__ bool RCtx::process(int64_t i, int row, int own, uint32_t rawU, int spec, double srad, bool given,
                                              const double* rowp) {
  const int K = S.K;
  const long long tq0 = prof ? wall_clock64() : 0;
  // The snapshot draw holds while nothing has moved in this launch, and after moves while
  // the slots and labels are those of the snapshot and no log-weight of the point has
  // moved by its radius: the others' by at most dvmax, its own slot's (count - 1) by du.
  // `given`: block mode, the caller has checked the draw against its block start.
  bool use_spec = given || (spec >= 0 && S.moves == 0);
  if (spec >= 0 && !use_spec && S.nstruct == 0) {
    const int sa = st.snap[own], sb = st.cnt[own];
    const double du = sa == sb ? 0.0 : (sa >= 2 && sb >= 2 ? fabs(st.l0[own] - st.sl0[own]) : INFINITY);
    use_spec = fmax(S.dvmax, du) < srad;
  }

  int pick = spec;
  if (!use_spec) {   // the point's exact row: staged in LDS (LIST mode), else loaded now
    if (!rowp) {
      const double* src = a.L + (int64_t)row * ncol;
      for (int c = lane; c < ncol; c += kWave) st.row[c] = src[c];
      if (a.lmask) {       // latent columns holding head bounds: their exact sums (latent_exact)
        const unsigned int lmv = a.lmask[row];
        if (lane < a.m && ((lmv >> lane) & 1u))
          st.row[a.S + lane] = latent_exact(a.codes_t, a.nq, a.d, a.pool.codes, a.pool.tab, i,
                                            pick_entry(a.raw[i * (a.m + 1) + lane], a.P));
      }
      wave_sync();
      rowp = st.row;
    }
    pick = exact_decision(a, st, K, rowp, own, raw_to_unif(rawU));
  }
  const long long tq1 = prof ? wall_clock64() : 0;
  if (prof && lane == 0) S.tsub[4] += tq1 - tq0;
  if (lane == 0) {
    if (!use_spec) S.exact++;
    // a pipelined sweep stops before its first decision that is not "stay" (nothing changed)
    const bool stay = pick >= 0 && ((pick < K && st.cnt[own] != 1 && st.sol[pick] == own) ||
                                    (pick >= K && st.cnt[own] == 1 && pick == K));
    if (a.dry && !stay) { S.status = kDryStop; S.next = (int)i; }
    else if (pick < 0) { S.status = -pick; S.next = (int)i; }
    else {
      const int ownlab = st.los[own];
      if (pick < K) {
        const int ns = st.sol[pick];
        if (st.cnt[own] != 1) {                                   // case 1
          if (ns != own) {
            a.c[i] = ns; set_count(st, a.logn, own, st.cnt[own] - 1); set_count(st, a.logn, ns, st.cnt[ns] + 1);
            S.moves++;
            log_move(a, nlog, i, own, ns);
            S.dnow = fmax(S.dnow, fmax(slot_drift(st, a.logn, own), slot_drift(st, a.logn, ns)));
            S.dvmax = fmax(S.dvmax, fmax(count_drift(st, a.logn, own), count_drift(st, a.logn, ns)));
          }
        } else {                                                  // case 2
          int target = ns;
          if (pick == ownlab) {           // the own (-inf) cluster was drawn
            if (ownlab == K - 1) { S.status = 1; S.next = (int)i; }
            target = st.sol[K - 1];
          }
          if (S.status == 0) {
            a.c[i] = target; set_count(st, a.logn, own, st.cnt[own] - 1);
            set_count(st, a.logn, target, st.cnt[target] + 1);
            S.moves++;
            log_move(a, nlog, i, own, target);
            const int last = st.sol[K - 1];
            st.los[own] = -1;
            if (ownlab != K - 1) { st.sol[ownlab] = last; st.los[last] = ownlab; }
            st.sol[K - 1] = -1;
            S.K = K - 1;
            S.nstruct++;
            S.dnow = fmax(S.dnow, fmax(slot_drift(st, a.logn, own), slot_drift(st, a.logn, target)));
          }
        }
      } else {
        const int l = pick - K;
        const bool single = st.cnt[own] == 1;
        if (!single || l != 0) {                                  // case 3 / case 4 (new params)
          if (S.nslots >= st.lcap || S.nslots >= scap) { S.status = 5; S.next = (int)i; }
          else {
            const int ns = S.nslots;
            S.nslots = ns + 1;
            if (!single) {                                        // case 3
              st.sol[K] = ns; st.los[ns] = K; S.K = K + 1;
              set_count(st, a.logn, own, st.cnt[own] - 1);
            } else {                                              // case 4
              st.sol[ownlab] = ns; st.los[ns] = ownlab; st.los[own] = -1;
              set_count(st, a.logn, own, 0);
            }
            set_count(st, a.logn, ns, 1);
            st.snap[ns] = 0;
            a.c[i] = ns;
            log_move(a, nlog, i, own, ns);
            S.src = (int)pick_entry(a.raw[i * (a.m + 1) + l], a.P);
            a.slot_src[ns] = S.src;
            S.moves++;
            S.restart = 1;
            S.next = (int)i + 1;
          }
        }
        // case 4 with latent 0 (the singleton's own parameters): nothing changes.
      }
    }
  }
  wave_sync();
  if (prof && lane == 0) S.tsub[6] += wall_clock64() - tq1;
  if (S.restart && S.status == 0) {
    const int ns = S.nslots - 1;
    copy_pool_params(a, S.src, ns);
    if (a.freq)   // the new slot's frequency table starts empty (the logged move fills it)
      for (int e = lane; e < a.fstride; e += kWave) a.freq[(int64_t)ns * a.fstride + e] = 0u;
  }
  return S.status == 0 && !S.restart;
}

// Once the drift exceeds dmax, the unlisted (certain at the snapshot) points between two
// listed ones are re-tested before the next listed point is decided: the n8 sequence is
// unchanged, and a point that is no longer certain stops the launch for the host to
// recompute bounds from there.  Returns false on such a point.
// (Block mode passes dn_over, a bound on the drift over a block's walk, and cmin, lower
// bounds on the counts during it.)
__device__ __forceinline__ bool RCtx::verify(int64_t lo, int64_t hi, double dn_over, const int* cmin) {
  if (lane == 0) S.checked = 1;
  const double dn = dn_over >= 0.0 ? dn_over : S.dnow;
  const int* cn = cmin ? cmin : st.cnt;
  constexpr int U = 4;     // chunks of 64 points whose inputs are loaded together
  for (int64_t base0 = lo; base0 < hi; base0 += U * kWave) {
    int rp[U], cj[U];
    double mgv[U];
    uint32_t rwv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = base0 + u * kWave + lane;
      const bool in = j < hi;
      rp[u] = in ? a.rowpos[j] : 0;
      mgv[u] = in ? a.margin[j] : 0.0;
      rwv[u] = in ? a.raw[j * (a.m + 1) + a.m] : 0u;
      cj[u] = in ? a.c[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = base0 + u * kWave + lane;
      bool fail = false;
      if (j < hi && rp[u] < 0) {
        const double mg = mgv[u] - 2.0 * dn;
        fail = !((mg > a.T || stay_by_uniform(mg, rwv[u], a.K + a.m)) && cn[cj[u]] >= 2);
      }
      const unsigned long long bal = __ballot(fail);
      if (bal) {
        if (lane == 0) { S.restart = 1; S.next = (int)(base0 + u * kWave + __ffsll((long long)bal) - 1); }
        wave_sync();
        return false;
      }
    }
  }
  return true;
}

__device__ __forceinline__ void resolve_layout(const ResolveArgs& a, RState& st, unsigned char* smem, bool blocks) {
  st.lcap = a.lcap;
  st.emax = a.lcap + a.m;
  st.sh = (RShared*)smem;
  st.val = (double*)(smem + kRSharedBytes);
  st.p = st.val + st.emax;
  st.row = st.p + st.emax;
  st.l1 = st.row + 2 * st.emax;
  st.l0 = st.l1 + st.lcap;
  st.cnt = (int*)(st.l0 + st.lcap);
  st.snap = st.cnt + st.lcap;
  st.sol = st.snap + st.lcap;
  st.los = st.sol + st.lcap;
  st.perm = st.los + st.lcap;
  // offsets from smem (not integer casts of the pointers): the arrays stay LDS pointers for
  // the compiler (ds_read, not flat loads that the LDS wait counter would also wait for)
  auto up16 = [&](const void* q) { return smem + ((((const unsigned char*)q - smem) + 15) & ~(ptrdiff_t)15); };
  st.ltab = (uint64_t*)up16(st.perm + st.emax);
  st.bp = nullptr;
  st.bperm = nullptr;
  st.bcmin = nullptr;
  st.brq = nullptr;
  // the snapshot's log counts in LDS (drift tests without global loads on the serial path)
  st.sl1 = (double*)(st.ltab + 256);
  st.sl0 = st.sl1 + st.lcap;
  if (blocks) {
    st.bp = st.sl0 + st.lcap;
    st.bperm = (int*)(st.bp + 64 * kWave);
    st.bcmin = st.bperm + 64 * kWave;
    st.brq = (int4*)up16(st.bcmin + kWave);
  }
}

// all threads: the launch's state in LDS
__device__ __forceinline__ void resolve_init(const ResolveArgs& a, const RState& st) {
  RShared& S = *st.sh;
  for (int e = threadIdx.x; e < 256; e += blockDim.x) st.ltab[e] = devtab::kGlibcLogTab[e];
  for (int s = threadIdx.x; s < st.lcap; s += blockDim.x) {
    const int v = s < a.nslots ? a.counts[s] : 0;
    st.cnt[s] = v;
    st.snap[s] = v;
    st.l1[s] = a.logn[v];
    st.l0[s] = v > 0 ? a.logn[v - 1] : -INFINITY;
    st.los[s] = s < a.nslots ? a.label_of_slot[s] : -1;
    st.sol[s] = s < a.K ? a.slot_of_label[s] : -1;
    if (st.sl1) { st.sl1[s] = st.l1[s]; st.sl0[s] = st.l0[s]; }
  }
  if (threadIdx.x == 0) {
    S.K = a.K; S.nslots = a.nslots; S.status = 0; S.next = a.n; S.restart = 0;
    S.moves = 0; S.exact = 0; S.checked = 0; S.dnow = 0.0; S.dvmax = 0.0; S.nstruct = 0; S.aborted = 0;
    S.bgo = 1; S.bq = 0;
    for (int k = 0; k < 8; ++k) S.tsub[k] = 0;
  }
  __syncthreads();
}

// all threads: write the state back, the host summary and the control block
__device__ __forceinline__ void resolve_finish(const ResolveArgs& a, const RState& st, int nlog, const long long* tp,
                                               bool prof) {
  RShared& S = *st.sh;
  const int scap = a.scap;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  // write back
  for (int s = threadIdx.x; s < S.nslots; s += blockDim.x) { a.counts[s] = st.cnt[s]; a.label_of_slot[s] = st.los[s]; }
  for (int s = threadIdx.x; s < S.K; s += blockDim.x) a.slot_of_label[s] = st.sol[s];
  // summary for the host (label -> slot, counts, pool sources), read with the control block
  __syncthreads();
  for (int s = threadIdx.x; s < scap; s += blockDim.x) {
    a.summary[s] = s < S.K ? st.sol[s] : -1;
    a.summary[scap + s] = s < S.nslots ? st.cnt[s] : 0;
    a.summary[2 * scap + s] = s < S.nslots ? a.slot_src[s] : -1;
  }
  if (wv != 0) return;
  if (prof && lane == 0) {
    for (int k = 0; k < 7; ++k) a.prof[k] = tp[k];
    a.prof[7] = wall_clock64();
    for (int k = 0; k < 8; ++k) a.prof[8 + k] = S.tsub[k];
  }
  if (lane == 0 && a.mcount) *a.mcount = nlog;
  if (lane == 0) {
    ResolveCtl c;
    c.next = S.next; c.status = S.status; c.restart = S.restart; c.K = S.K; c.nslots = S.nslots;
    c.moves = S.moves; c.exact = S.exact; c.checked = S.checked;
    c.listed = *a.dense_total;
    c.aborted = S.aborted;
    c.uncertain = a.uncertain ? *a.uncertain : -1;
    *a.ctl = c;
  }
}

__global__ __launch_bounds__(kWave) void k_resolve(ResolveArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  RState st;
  resolve_layout(a, st, smem, false);
  RShared& S = *st.sh;
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool prof = a.prof != nullptr;
  if (prof) tp[0] = wall_clock64();
  resolve_init(a, st);
  RCtx R{a, st, S, lane, a.S + a.m, a.scap, a.mcount ? *a.mcount : 0, prof};
  const int ncol = R.ncol;
  const int tstride = resolve_tile_stride(ncol);
  // LIST mode's row tile after the layout's last array (resolve_lds_bytes)
  double* tile = (ncol <= kTileCols && !a.force_exact) ? st.sl0 + st.lcap : nullptr;
  bool go = true;
  int64_t start_checked = -1;
if (!a.force_exact) {
  // LIST mode: only the prepass's uncertain points need work while drift <= dmax.  The
  // dense list, the points' labels, draws and snapshot draws are read 64 at a time; the
  // points whose snapshot draw still holds and keeps them in their cluster change
  // nothing and are passed over with one ballot; the others are decided in order (exact
  // rows loaded only for the points that need an exact decision).
  const int total = *a.dense_total;
  if (prof) tp[1] = wall_clock64();
  int64_t vfrom = a.p0;   // unlisted points [vfrom, next listed point) not yet re-tested
  constexpr int kB = 4;   // chunks of 64 points whose inputs are loaded together
  for (int qb = 0; qb < total && go; qb += kB * kWave) {
    long long tb = prof ? wall_clock64() : 0;
    int4 rqv[kB];
    int spv[kB];
    double srv[kB];
#pragma unroll
    for (int b = 0; b < kB; ++b) {
      const int qq = qb + b * kWave + lane;
      const bool in = qq < total;
      rqv[b] = in ? a.rq[qq] : make_int4(0, 0, 0, 0);
      spv[b] = (in && a.spec) ? a.spec[qq] : -1;
      srv[b] = (in && a.spec) ? a.spec_rad[qq] : 0.0;
    }
    if (prof) tp[3] += wall_clock64() - tb;
#pragma unroll
    for (int b = 0; b < kB; ++b) {
    const int q0 = qb + b * kWave;
    if (q0 >= total || !go) break;
    const int lim = min(kWave, total - q0);
    const int rw = rqv[b].x, li = rqv[b].y, ci = rqv[b].z;
    const uint32_t ru = (uint32_t)rqv[b].w;
    const int sp = spv[b];
    const double sr = srv[b];
    if (tile) {        // every lane its point's exact row, all loads in flight together
      const double* src = a.L + (int64_t)rw * ncol;
      double* dst = tile + lane * tstride;
      for (int c0 = 0; c0 < ncol; c0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (lane < lim && c0 + u < ncol) ? src[c0 + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (c0 + u < ncol) dst[c0 + u] = v[u];
      }
      wave_sync();
    }
    int q = 0;
    while (q < lim && go) {
      long long t0 = prof ? wall_clock64() : 0;
      bool stays = false;
      if (lane >= q && lane < lim && sp >= 0 && sp < S.K && st.cnt[ci] != 1 && st.sol[sp] == ci) {
        const int sa = st.snap[ci], sb = st.cnt[ci];
        const double du = sa == sb ? 0.0 : (sa >= 2 && sb >= 2 ? fabs(st.l0[ci] - st.sl0[ci]) : INFINITY);
        stays = S.moves == 0 || (S.nstruct == 0 && fmax(S.dvmax, du) < sr);
      }
      const unsigned long long todo = __ballot(lane >= q && lane < lim && !stays);
      if (!todo) break;
      q = __ffsll((long long)todo) - 1;
      const int64_t i = __shfl(li, q);
      const long long tv = prof ? wall_clock64() : 0;
      if (S.dnow > a.dmax && !R.verify(vfrom, i)) { go = false; break; }
      if (prof && lane == 0) { S.tsub[5] += wall_clock64() - tv; S.tsub[7] += i - vfrom; }
      go = R.process(i, __shfl(rw, q), __shfl(ci, q), (uint32_t)__shfl((int)ru, q), __shfl(sp, q), __shfl(sr, q),
                     false, tile ? tile + q * tstride : nullptr);
      vfrom = i + 1;
      ++q;
      if (prof) {
        tp[4] += wall_clock64() - t0;
        tp[6] += 1;
      }
    }
    }
  }
  if (go && S.status == 0 && !S.restart && S.dnow > a.dmax) (void)R.verify(vfrom, a.n);
} else {
  start_checked = a.p0;
}
// CHECKED mode: every remaining point is re-tested against the current drift.
if (start_checked >= 0 && S.status == 0 && !S.restart) {
  if (lane == 0) S.checked = 1;
  for (int64_t base = start_checked; base < a.n; base += kWave) {
    const int64_t i = base + lane;
    bool unc = false;
    int ci = 0;
    if (i < a.n) {
      ci = a.c[i];
      const double mg = a.margin[i] - 2.0 * S.dnow;
      unc = a.force_exact ||
            !((mg > a.T || stay_by_uniform(mg, a.raw[i * (a.m + 1) + a.m], a.K + a.m)) && st.cnt[ci] >= 2);
    }
    unsigned long long bal = __ballot(unc);
    bool stop = false;
    while (bal) {
      const int q = __ffsll((long long)bal) - 1;
      const int row = a.rowpos[base + q];
      if (row < 0) {
        // certain at the snapshot but not under the current drift, and no exact row:
        // stop here and let the host recompute bounds from this point
        if (lane == 0) { S.restart = 1; S.next = (int)(base + q); }
        wave_sync();
        stop = true;
        break;
      }
      if (!R.process(base + q, row, __shfl(ci, q), a.raw[(base + q) * (a.m + 1) + a.m], -1, 0.0)) { stop = true; break; }
      // drift may have grown: re-test the remaining lanes
      bool u2 = false;
      if (lane > q && i < a.n) {
        const double mg = a.margin[i] - 2.0 * S.dnow;
        u2 = a.force_exact ||
             !((mg > a.T || stay_by_uniform(mg, a.raw[i * (a.m + 1) + a.m], a.K + a.m)) && st.cnt[ci] >= 2);
      }
      bal = __ballot(u2);
    }
    if (stop) break;
  }
}
  resolve_finish(a, st, R.nlog, tp, prof);
}

// The n8:95-102 draw of this lane's point from its E log-weights w (LDS column: entry e at
// w[e * kWave]), run literally: max, exp, sum, normalise, FixupProb, revsort, cumulative
// compare (n8:95-102 with Rcpp's sample()), the same operations as decide_values.  *rad: as
// decide_values' radius (the draw holds while every log-weight moves by less), 0 when no
// bound is kept (ties among the positive probabilities, a draw past them).  Returns the
// index or -status.  The column is overwritten (p), perm is the lane's index column.
__device__ int decide_lane(double* w, int* perm, int E, double rU, double* rad) {
  *rad = 0.0;
  double mx = w[0];
  for (int e = 1; e < E; ++e) mx = fmax(mx, w[e * kWave]);
  for (int e = 0; e < E; ++e) w[e * kWave] = dexp(w[e * kWave] - mx);                     // n8:95
  double sum = 0.0;
  for (int e = 0; e < E; ++e) sum += w[e * kWave];
  for (int e = 0; e < E; ++e) w[e * kWave] = w[e * kWave] / sum;                          // n8:96
  double s2 = 0.0;                                                                         // FixupProb
  for (int e = 0; e < E; ++e) { const double x = w[e * kWave]; s2 += x > 0 ? x : 0.0; }
  if (!(s2 > 0)) return -3;
  double pmax = -1.0, p2 = -1.0;
  int amax = -1, ties = 0, npos = 0;
  for (int e = 0; e < E; ++e) {
    const double x = w[e * kWave] / s2;
    w[e * kWave] = x;
    npos += x > 0 ? 1 : 0;
    if (x > pmax) { p2 = pmax; pmax = x; amax = e; ties = 1; }
    else if (x == pmax) ++ties;
    else if (x > p2) p2 = x;
  }
  if (ties == 1 && rU <= pmax) {          // revsort puts the unique maximum first
    const double r1 = p2 > 0 ? 0.5 * log(pmax / p2) : INFINITY;
    *rad = fmax(0.0, fmin(r1, 0.5 * log(pmax / rU)) - 1e-9);
    return amax;
  }
  for (int e = 0; e < E; ++e) perm[e * kWave] = e + 1;
  lane_revsort(w, perm, E);
  // the reference's cumulative sums in sorted order (in place there; the same additions
  // in a register here, so w keeps the sorted probabilities for the radius)
  double c = 0.0, cprev = 0.0;
  int j;
  for (j = 0; j < E - 1; ++j) {
    cprev = c;
    c += w[j * kWave];
    if (rU <= c) break;
  }
  if (j == E - 1) { cprev = c; c += w[j * kWave]; }
  const int pick = perm[j * kWave] - 1;
  // radius: the pick keeps its place among the positive entries (strictly between its
  // neighbours) and rU its interval (as decide_values)
  if (j < npos) {
    const double pj = w[j * kWave];
    double r = INFINITY;
    bool ok = true;
    if (j > 0) {
      const double pprev = w[(j - 1) * kWave];
      ok &= pprev > pj;
      r = fmin(r, fmin(0.5 * log(pprev / pj), 0.5 * log(rU / cprev)));
    }
    if (j + 1 < npos) {
      const double pnext = w[(j + 1) * kWave];
      ok &= pj > pnext;
      r = fmin(r, 0.5 * log(pj / pnext));
    }
    if (j != E - 1) r = fmin(r, 0.5 * log(c / rU));
    if (ok) *rad = fmax(0.0, r - 1e-9);
  }
  return pick;
}

// Block mode (see kBlk): one wave, launched when the previous launch listed at least
// kResolveBlkMin uncertain points and K + m <= 64, nslots <= 64 (lane = block point, and
// lane = slot in the walk).
__global__ __launch_bounds__(kWave) void k_resolve_blk(ResolveArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  RState st;
  resolve_layout(a, st, smem, true);
  RShared& S = *st.sh;
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool prof = a.prof != nullptr;
  if (prof) tp[0] = wall_clock64();
  resolve_init(a, st);
  RCtx R{a, st, S, lane, a.S + a.m, a.scap, a.mcount ? *a.mcount : 0, prof};
  const int ncol = R.ncol;
  const int total = *a.dense_total;
  int64_t vfrom = a.p0;   // unlisted points [vfrom, next listed point) not yet re-tested
  bool go = true;
  if (prof) tp[1] = wall_clock64();
  const unsigned long long below = (1ull << lane) - 1ull;
  int rq_lo = 0, rq_hi = 0;
  for (int qb = 0; qb < total && go;) {
    const long long tb = prof ? wall_clock64() : 0;
    const int nb = min(kBlk, total - qb);
    const int K = S.K, E = K + a.m;
    const bool inb = lane < nb;
    // ---- the block's draws, lane k = point qb + k, in the state at the block start; the
    // points' inputs come through an LDS window of kRqWin list positions
    if (qb + nb > rq_hi) {
      rq_lo = qb;
      rq_hi = min(total, qb + kRqWin);
      for (int q = lane; q < rq_hi - rq_lo; q += kWave) st.brq[q] = a.rq[rq_lo + q];
      wave_sync();
    }
    const int4 r = inb ? st.brq[qb - rq_lo + lane] : make_int4(0, 0, 0, 0);
    const int own = r.z;
    const bool single = inb && st.cnt[own] == 1;
    double* wcol = st.bp + lane;
    int* pcol = st.bperm + lane;
    if (inb) {
      // the row entries 16 at a time (loads in flight together), then the log-weights
      const double* Lr = a.L + (int64_t)r.x * ncol;
      const double lo = Lr[own];
      for (int e0 = 0; e0 < E; e0 += 16) {
        double x[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const int e = e0 + t;
          x[t] = e < E ? Lr[e < K ? st.sol[e] : a.S + e - K] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const int e = e0 + t;
          if (e < K) {
            const int sl = st.sol[e];
            wcol[e * kWave] = (sl == own ? st.l0[sl] : st.l1[sl]) + x[t];
          } else if (e < E) {
            wcol[e * kWave] = a.logfac + ((e == K && single) ? lo : x[t]);
          }
        }
      }
    }
    double rad = 0.0;
    int pick = -1;
    if (inb) {
      const double rU = raw_to_unif((uint32_t)r.w);
      pick = decide_lane(wcol, pcol, E, rU, &rad);
    }
    if (prof) tp[3] += wall_clock64() - tb;
    const long long tw = prof ? wall_clock64() : 0;
    // ---- classification in the block-start state (a kept point has its own count unchanged,
    // so its state at its turn is this one): stay, case-1 move own -> tgt, or structural
    bool mover = false, structural = false;
    int tgt = own;
    if (inb) {
      if (pick < 0) structural = true;
      else if (pick < K) {
        const int ns = st.sol[pick];
        if (!single) { mover = ns != own; tgt = ns; }
        else structural = true;                                             // case 2
      } else {
        structural = !(single && pick == K);                                // cases 3 / 4 (new params)
      }
    }
    // whether LIST mode would have had to decide the point itself (its snapshot draw from
    // k_exact_rows no longer held): the host's choice between the two modes
    bool list_exact = true;
    if (inb && a.spec) {
      const int sp = a.spec[qb + lane];
      if (sp >= 0) {
        const int sa = st.snap[own], sb = st.cnt[own];
        const double du0 = sa == sb ? 0.0 : (sa >= 2 && sb >= 2 ? fabs(st.l0[own] - st.sl0[own]) : INFINITY);
        list_exact = !(S.moves == 0 || (S.nstruct == 0 && fmax(S.dvmax, du0) < a.spec_rad[qb + lane]));
      }
    }
    const unsigned long long smask = __ballot(structural);
    const int ks0 = smask ? __ffsll((long long)smask) - 1 : nb;
    const unsigned long long mvm = __ballot(mover) & (ks0 >= 64 ? ~0ull : ((1ull << ks0) - 1ull));
    // slots the block's moves touch
    unsigned long long touch = mover && lane < ks0 ? ((1ull << own) | (1ull << tgt)) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) touch |= __shfl_xor(touch, o);
    const int cs = lane < S.nslots ? st.cnt[lane] : 0;     // block-start counts (lane = slot)
    // ---- the walk in parallel: count changes before each point, from the moves before it;
    // |log(c + d) - log(c)| <= |d| / min(c, c + d) bounds the drift of a count's log (fp32,
    // integers below 2^24 exact, the factor covers the division's rounding)
    auto bound = [](int d, int c) -> float {
      if (d == 0) return 0.0f;
      const int mn = min(c, c + d);
      return mn <= 0 ? INFINITY : (float)abs(d) / (float)mn * 1.000001f;
    };
    float Dk = 0.0f, du = 0.0f;
    for (unsigned long long t = touch; t; t &= t - 1) {
      const int sl = __ffsll((long long)t) - 1;
      const unsigned long long in = __ballot(mover && tgt == sl) & mvm, out = __ballot(mover && own == sl) & mvm;
      const int d = __popcll(in & below) - __popcll(out & below);
      const int c = __builtin_amdgcn_readlane(cs, sl);
      Dk = fmaxf(Dk, bound(d, c));
      if (own == sl) du = bound(d, c - 1);
    }
    const bool keep = lane == 0 || (double)fmaxf(Dk, du) < rad;
    const unsigned long long bad = __ballot(inb && !keep);
    const int kstop = bad ? __ffsll((long long)bad) - 1 : nb;
    int kc = min(kstop, ks0);
    bool serial_next = ks0 < kstop;
    // unlisted points before the last kept one: re-tested with a bound on the drift and
    // lower bounds on the counts over the walk (their turn comes during it)
    if (kc > 0) {
      const int64_t ilast = __shfl(r.y, kc - 1);
      const unsigned long long ltk = kc >= 64 ? ~0ull : ((1ull << kc) - 1ull);
      const float Dall = wave_max(lane < kc ? (double)Dk : 0.0);
      if (S.dnow + (double)Dall > a.dmax) {
        int co = 0;
        for (unsigned long long t = touch; t; t &= t - 1) {
          const int sl = __ffsll((long long)t) - 1;
          const int nout = __popcll(__ballot(mover && own == sl) & mvm & ltk);
          if (lane == sl) co = nout;
        }
        if (lane < S.nslots) st.bcmin[lane] = cs - co;
        wave_sync();
        if (!R.verify(vfrom, ilast, S.dnow + (double)Dall, st.bcmin)) {
          const int64_t u = S.next;     // the launch stops at the first failing unlisted point
          kc = __popcll(__ballot(lane < kc && (int64_t)r.y < u));
          go = false;
          serial_next = false;
        }
      }
    }
    // ---- commit the kept points together: labels, move log, counts, drifts
    const unsigned long long ltk = kc >= 64 ? ~0ull : ((1ull << kc) - 1ull);
    const bool cm = lane < kc && mover;
    const unsigned long long mm = __ballot(cm);
    if (cm) {
      a.c[r.y] = tgt;
      if (a.mlog) {
        const int q = R.nlog + __popcll(mm & below);
        a.mlog[3 * q] = r.y;
        a.mlog[3 * q + 1] = own;
        a.mlog[3 * q + 2] = tgt;
      }
    }
    if (a.mlog) R.nlog += __popcll(mm);
    int dl = 0;
    for (unsigned long long t = touch; t; t &= t - 1) {
      const int sl = __ffsll((long long)t) - 1;
      const int d = __popcll(__ballot(mover && tgt == sl) & mvm & ltk) - __popcll(__ballot(mover && own == sl) & mvm & ltk);
      if (lane == sl) dl = d;
    }
    double sd = 0.0, cd = 0.0;
    if (lane < S.nslots && dl != 0) {
      const int c = cs + dl;
      st.cnt[lane] = c;
      st.l1[lane] = logn_dev(st, c);
      st.l0[lane] = logn_dev(st, c - 1);
      sd = slot_drift(st, a.logn, lane);
      cd = count_drift(st, a.logn, lane);
    }
    sd = wave_max(sd);
    cd = wave_max(cd);
    const int lex = __popcll(__ballot(lane < kc && list_exact));
    if (lane == 0) {
      S.moves += __popcll(mm);
      S.exact += lex;
      S.dnow = fmax(S.dnow, sd);
      S.dvmax = fmax(S.dvmax, cd);
    }
    if (kc > 0) vfrom = (int64_t)__shfl(r.y, kc - 1) + 1;
    int done = kc;
    wave_sync();
    // ---- a structural point (case 2, 3 or 4) in turn: the serial path
    if (serial_next && go) {
      const int64_t i = __shfl(r.y, kc);
      if (S.dnow > a.dmax && !R.verify(vfrom, i)) go = false;
      else {
        go = R.process(i, __shfl(r.x, kc), __shfl(own, kc), (uint32_t)__shfl(r.w, kc), __shfl(pick, kc), 0.0, true);
        R.nlog = __builtin_amdgcn_readfirstlane(R.nlog);
        vfrom = i + 1;
        ++done;
        if (lane == 0 && __shfl(list_exact ? 1 : 0, kc)) S.exact++;
      }
    }
    qb += done;
    if (prof) { tp[4] += wall_clock64() - tw; tp[6] += done; tp[5] += 1; }
  }
  if (go && S.status == 0 && !S.restart && S.dnow > a.dmax) (void)R.verify(vfrom, a.n);
  resolve_finish(a, st, R.nlog, tp, prof);
}

// ------------------------------------------------------------------ fixed-point resolver
// k_resolve_fp (kFpThreads threads, one listed point per thread) walks the dense list in
// chunks of kFpThreads positions.  A chunk's outcomes are a fixed point: every point draws in
// the state left by the outcomes of the chunk's points before it (the launch's committed
// state plus their case-1 moves), and the draws are repeated -- for the points after the
// first outcome that changed -- until no outcome changes.  Point k's state depends only on
// the points before it, so after round r the first r outcomes are final, and the fixed point
// is the n8 walk's sequence of decisions (code/neal8.cpp:40-160, in index order).
// A point's draw is its snapshot draw (k_exact_rows) while no log-weight of it has moved by
// its radius (decide_values), else the n8:95-102 draw on its own lane (fp_draw).  Outcomes:
// stay, case-1 move, or stop -- cases 2-4, an error, or a pick among equal probabilities
// (revsort's order decides those): the chunk commits its points before the first stop and
// the stop goes through the serial path (RCtx::process on wave 0), then the next chunk
// starts behind it.  Unlisted points between listed ones are re-tested against the drift
// after the moves before them, as in k_resolve.  Needs K + m <= 64 and lcap <= 64.
#ifndef HDPM_FP_THREADS
#define HDPM_FP_THREADS 512     // build parameter for A/B (8 waves: two per SIMD; 256: C2 -10%, C5 random-20 -26%)
#endif
constexpr int kFpThreads = HDPM_FP_THREADS;
constexpr int kFpWaves = kFpThreads / kWave;
constexpr int kFpFallback = -1000;

struct FpShared {
  int wc[kFpWaves][kWave];          // slot counts at each wave's first point
  int wd[kFpWaves][kWave];          // each wave's net count change per slot
  double wsd[kFpWaves];
  int wstop[kFpWaves], wchg[kFpWaves], wmov[kFpWaves], wfresh[kFpWaves], wneed[kFpWaves];
  int dlist[kFpThreads];            // chunk positions whose draw is made this round (compacted)
  int dpick[kFpThreads];            // ... and their picks
  long long wev[kFpWaves];          // diagnostics: each wave's evaluation ticks in a round
  uint64_t etab[256];               // glibc's exp table (fp_draw)
  int cmo[kWave];                   // moves out of each slot in the chunk
  int cmin[kWave];                  // lower bounds on the counts during the chunk
  int pi[kFpThreads];               // point of each chunk position
  double dnl[kFpThreads];           // the walk's drift after each chunk position
  int nlog, go, ufail, stop_pick, stop_fresh, iters, pad0, pad1;
  int4 stop_rq;
  unsigned long long bin[kFpWaves][kWave];   // per wave and slot: the movers into the slot
  unsigned long long bout[kFpWaves][kWave];  // ... and out of it
};

__host__ __device__ inline size_t resolve_fp_lds_bytes(int lcap, int m) {
  return ((resolve_lds_bytes(lcap, m, 0, 0) + 15) & ~(size_t)15) + sizeof(FpShared);
}

// logn[c] from the host's table (the same glibc values logn_dev computes): independent loads
// the per-lane code issues together, instead of dependent log evaluations
// A load from global memory as such (a global_load, not a flat one: flat loads count
// against the LDS wait counter too, so every LDS wait would wait for them)
template <class T>
__device__ __forceinline__ T gld(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(1))) T*)p;
#else
  return *p;     // host pass: never called
#endif
}

__device__ __forceinline__ double fp_logn(const ResolveArgs& a, int c) { return c <= 0 ? -INFINITY : gld(a.logn + c); }

__device__ __forceinline__ double fp_wave_drift_bound(const ResolveArgs& a, const RState& st, const int* wc,
                                                      const unsigned long long* bin, const unsigned long long* bout,
                                                      int nsl) {
  const int s = threadIdx.x & 63;
  double b = 0.0;
  if (s < nsl) {
    const int lo = wc[s] - __popcll(bout[s]), hi = wc[s] + __popcll(bin[s]);
    const int a0 = st.snap[s];
    if (!(lo == a0 && hi == a0)) {
      const double d_oth = (a0 < 1 || lo < 1) ? INFINITY
                                               : fmax(fabs(fp_logn(a, hi) - st.sl1[s]), fabs(fp_logn(a, lo) - st.sl1[s]));
      const double d_own = (a0 < 2 || lo < 2)
                               ? INFINITY
                               : fmax(fabs(fp_logn(a, hi - 1) - st.sl0[s]), fabs(fp_logn(a, lo - 1) - st.sl0[s]));
      b = fmax(d_oth, d_own);
    }
  }
  return wave_max(b);
}

// slot_drift of slot s at count b (k_resolve's running drift after a move)
__device__ __forceinline__ double slot_drift_at(const ResolveArgs& a, const RState& st, int s, int b) {
  const int a0 = st.snap[s];
  if (a0 >= 2) return b < 2 ? INFINITY : fabs(fp_logn(a, b - 1) - st.sl0[s]);
  if (a0 == 1) return b == 0 ? 0.0 : fp_logn(a, b);
  return INFINITY;
}

// The n8:95-102 draw from the log-weights v[0..E) on this lane: the operations of
// decide_values (max, glibc exp, index-order sum, normalisation, FixupProb), then revsort's
// descending order walked group by group of equal values with the reference's cumulative
// sums; a pick inside a group of more than one entry (whose order is heapsort's) returns
// kFpFallback.  E <= EM <= 200 (no Walker tables).  Returns the index or -status.
// exp(x) for x = v - max <= 0 as fp_draw needs it: glibc's main path (exp_r's value for
// -512 < x <= 0, its |x| < 2^-54 path included), and 0 for x <= -512.  An entry with x <= -512
// has p < e^-512 < 2^-738 against a sum >= 1 (the maximum's exp(0) = 1), so the sums round
// the same whether it is added or not, every other probability keeps its bits, and it cannot
// be drawn: it sorts behind every entry with x > -512, and the cumulative sum over those
// reaches 1 - E 2^-52 before it, far above the largest uniform 1 - 2^-33 (raw_to_unif).  So
// the draw is the reference's for every input, with a third of exp_bf's operations.
__device__ __forceinline__ double fp_exp(double x, const uint64_t* T) {
  using namespace glibc;
  const uint64_t ix = asu(x);
  const uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
  const bool tiny = (int)(abstop - 0x3c9u) < 0;
  const double kd0 = __builtin_fma(x, kExpInvLn2N, kExpShift);
  const uint64_t ki = asu(kd0);
  const double kd = kd0 - kExpShift;
  double r = __builtin_fma(kd, kExpNegLn2hiN, x);
  r = __builtin_fma(kd, kExpNegLn2loN, r);
  const uint32_t i2 = 2u * (uint32_t)(ki & 127u);
  const uint64_t sbits = T[i2 + 1] + (ki << 45);
  const double p23 = __builtin_fma(r, kExpC3, kExpC2);
  const double rt = r + asd(T[i2]);
  const double r2 = r * r;
  const double p45 = __builtin_fma(r, kExpC5, kExpC4);
  const double t = __builtin_fma(p23, r2, rt);
  const double r4 = r2 * r2;
  const double tmp = __builtin_fma(r4, p45, t);
  const double scale = asd(sbits);
  const double y = __builtin_fma(scale, tmp, scale);
  return tiny ? x + 1.0 : (x > -512.0 ? y : 0.0);
}

// An upper bound, over the wave's lanes, of the drift the fixed-point evaluation computes per
// lane (the largest |log-count term now - at the snapshot| over the entries, n8:40-92): the
// count a lane sees for slot s lies in [wc - movers out of s, wc + movers into s] (the wave's
// movers before it), its own slot's term uses that count less one, and logn is monotone, so
// the extremes bound every lane.  Below a lane's radius the snapshot draw holds without the
// per-entry terms.  Lane = slot; every lane of the wave calls it.
struct FpShared;
__device__ __forceinline__ double fp_wave_drift_bound(const ResolveArgs& a, const RState& st, const int* wc,
                                                      const unsigned long long* bin, const unsigned long long* bout,
                                                      int nsl);

//
// With kRad, *rad receives a radius as decide_values' (0 when none is kept): the draw stands
// while every log-weight moves by less than it -- normalised probabilities then move by
// factors within exp(+-2 rad), so the picked entry keeps its rank (its ratios to the nearest
// larger and smaller values) and the uniform stays inside its cumulative interval; 1e-9 covers
// the reference's few ulps of rounding.
template <int EM, bool kRad = false>
__device__ int fp_draw(double (&v)[EM], int E, double rU, const uint64_t* etab, double* rad = nullptr) {
  if constexpr (kRad) *rad = 0.0;
  // branch-free over the EM slots (padding: exp(-inf) = 0 adds nothing to the sums), so
  // the exps' table loads are issued together
  double mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    v[e] = e < E ? v[e] : -INFINITY;
    mx = fmax(mx, v[e]);
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const double p = fp_exp(v[e] - mx, etab);                                 // n8:95
    v[e] = e < E ? p : 0.0;
  }
  double sum = 0.0;
#pragma unroll
  for (int e = 0; e < EM; ++e) sum += v[e];
  // The dominant entry drawn (most draws: a point that stays).  With one entry at the maximum
  // (exp 0 = 1; revsort puts it first) the reference's probability of it is
  // (1 / sum) / s2 with s2 = 1 to within E ulps, so it is at least (1 / sum)(1 - 1e-12), and
  // a uniform below that picks it: no normalisation or walk needed.
  {
    int nmax = 0, am = 0;
    double e2 = 0.0;
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const bool is1 = v[e] == 1.0;
      nmax += is1 ? 1 : 0;
      am = is1 ? e : am;
      e2 = (!is1 && v[e] > e2) ? v[e] : e2;
    }
    const double pl = (1.0 / sum) * (1.0 - 1e-12);
    if (nmax == 1 && rU <= pl) {
      if constexpr (kRad) {
        double r = 0.5 * log(pl / rU);
        const double p2u = (e2 / sum) * (1.0 + 1e-12);
        if (p2u > 0.0) r = fmin(r, 0.5 * log(pl / p2u));
        *rad = fmax(0.0, r - 1e-9);
      }
      return am;
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) v[e] = v[e] / sum;                           // n8:96
  double s2 = 0.0;                                                          // FixupProb
#pragma unroll
  for (int e = 0; e < EM; ++e) s2 += v[e] > 0 ? v[e] : 0.0;
  if (!(s2 > 0)) return -3;
#pragma unroll
  for (int e = 0; e < EM; ++e) v[e] = e < E ? v[e] / s2 : -1.0;
  double prev = INFINITY, c = 0.0;
  for (int j = 0; j < E;) {
    double cur = -1.0;
    int g = 0, idx = -1;
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const double x = v[e];
      const bool lt = x < prev;
      const bool gt = lt && x > cur, eq = lt && x == cur;
      cur = gt ? x : cur;
      idx = gt ? e : idx;
      g = gt ? 1 : (eq ? g + 1 : g);
    }
    if (g == 0) return kFpFallback;
    const double cb = c;      // cumulative before this group
    for (int k = 0; k < g; ++k, ++j) {
      c += cur;
      if (j == E - 1 || rU <= c) {
        if (g != 1) return kFpFallback;
        if constexpr (kRad) {
          if (rU <= c && cur > 0.0) {
            double nx = 0.0;   // the next smaller positive value
#pragma unroll
            for (int e = 0; e < EM; ++e) nx = (v[e] < cur && v[e] > nx) ? v[e] : nx;
            double r = 0.5 * log(c / rU);
            if (prev < INFINITY) r = fmin(r, 0.5 * log(prev / cur));
            if (nx > 0.0) r = fmin(r, 0.5 * log(cur / nx));
            if (cb > 0.0) r = fmin(r, 0.5 * log(rU / cb));
            *rad = fmax(0.0, r - 1e-9);
          }
        }
        return idx;
      }
    }
    prev = cur;
  }
  return kFpFallback;
}

// The draw of chunk position t (a point whose snapshot draw does not hold) in the state the
// round gives it -- the counts at its wave's first point plus the moves before it in its wave
// (ballot masks), n8:40-102 -- made by whichever lane the round's compacted list assigns it:
// the positions that draw are gathered into dense waves first, so a wave with one drawing lane
// no longer runs fp_draw for all 64 (the fixed-point resolvers' rounds, k_resolve_fp / _fpg).
template <int EM>
__device__ __forceinline__ int fp_draw_at(const ResolveArgs& a, const RState& st, FpShared* F, int t, int4 r, int K,
                                          int E, int ncol) {
  const int w = t >> 6;
  const unsigned long long bl = (1ull << (t & 63)) - 1ull;
  const int own = r.z;
  auto corr = [&](int sl) -> int { return __popcll(F->bin[w][sl] & bl) - __popcll(F->bout[w][sl] & bl); };
  const int cnow = F->wc[w][own] + corr(own);
  const bool single = cnow == 1;
  int sl[EM];
  double v[EM], x[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const int s = st.sol[e < K ? e : 0];
    sl[e] = s;
    const int c = F->wc[w][s] + corr(s) - (s == own ? 1 : 0);                  // n8:40-92
    v[e] = gld(a.logn + ((e < K && c > 0) ? c : 0));
  }
  const double* Lr = a.L + (int64_t)r.x * ncol;
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const int l = e - K;
    const int col = e < K ? sl[e] : (e < E ? ((l == 0 && single) ? own : a.S + l) : 0);
    x[e] = gld(Lr + col);
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) v[e] = e < K ? v[e] + x[e] : a.logfac + x[e];
  if (a.lmask) {
    const unsigned int lmv = gld(a.lmask + r.x);
    if (lmv) latent_fix<EM>(a.codes_t, a.nq, a.d, a.pool, a.raw, a.P, a.logfac, v, K, E, lmv, single, r.y, a.m,
                            a.lat_negl);
  }
  return fp_draw<EM>(v, E, raw_to_unif((uint32_t)r.w), F->etab);
}

// Every thread of the workgroup: positions with `need` set get their draws made in dense waves
// (fp_draw_at); returns this thread's pick (or -1 without need).
template <int EM>
__device__ __forceinline__ int fp_draws_compacted(const ResolveArgs& a, const RState& st, FpShared* F, bool need,
                                                  int q0, int K, int E, int ncol) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long nb = __ballot(need);
  if (lane == 0) F->wneed[wv] = __popcll(nb);
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kFpWaves; ++w) {
    base += w < wv ? F->wneed[w] : 0;
    tot += F->wneed[w];
  }
  if (need) F->dlist[base + __popcll(nb & ((1ull << lane) - 1ull))] = tid;
  __syncthreads();
  for (int k = tid; k < tot; k += kFpThreads) {
    const int t = F->dlist[k];
    F->dpick[t] = fp_draw_at<EM>(a, st, F, t, gld(a.rq + q0 + t), K, E, ncol);
  }
  __syncthreads();
  return need ? F->dpick[tid] : -1;
}

// The drift of a point's log-count terms from the snapshot's (n8:40-92: logn[count] per
// cluster, logn[count - 1] for its own) -- the quantity a snapshot draw's radius bounds -- as an
// upper bound from float logarithms plus their error (counts < 2^24 are exact in float; each
// log2 is within a few ulps, < 2e-6 at these magnitudes, so 3e-5 covers the difference).  The
// radius test needs only a bound, and this spares the EM table loads of the exact terms (the
// drawing lanes load them, fp_draw_at).
__device__ __forceinline__ double fdrift(int now, int snap) {
  if (now == snap) return 0.0;
  if (now < 1 || snap < 1) return INFINITY;
  return (double)fabsf(__log2f((float)now) - __log2f((float)snap)) * 0.6931471805599453 + 3e-5;
}
template <int EM, class CORR>
__device__ __forceinline__ double fp_lane_drift(const RState& st, const int* wc, CORR corr, int own, int cnow, int K) {
  double drift = 0.0;
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    if (e < K) {
      const int s = st.sol[e];
      const int a0 = st.snap[s];
      double d;
      if (s == own) d = a0 == cnow ? 0.0 : ((a0 >= 2 && cnow >= 2) ? fdrift(cnow - 1, a0 - 1) : INFINITY);
      else d = fdrift(wc[s] + corr(s), a0);
      drift = fmax(drift, d);
    }
  }
  return drift;
}

// Unlisted points in [lo, hi) re-tested as RCtx::verify does, each against the drift after
// the chunk positions before it (dnl[k] for the last position k < nk with pi[k] < j, dn0
// before any) and the count bounds cmin.  All threads; returns the first failing point
// (restart there) or hi.
__device__ int64_t fp_verify(const ResolveArgs& a, const RState& st, FpShared* F, int nk, double dn0, int64_t lo,
                             int64_t hi, const int* cmin) {
  RShared& S = *st.sh;
  if (threadIdx.x == 0) { F->ufail = INT_MAX; S.checked = 1; }
  __syncthreads();
  for (int64_t b = lo; b < hi; b += kFpThreads) {
    const int64_t j = b + threadIdx.x;
    if (j < hi && gld(a.rowpos + j) < 0) {
      int k0 = 0, k1 = nk;
      while (k0 < k1) {
        const int md = (k0 + k1) >> 1;
        if (F->pi[md] < j) k0 = md + 1; else k1 = md;
      }
      const double dn = k0 > 0 ? F->dnl[k0 - 1] : dn0;
      if (dn > a.dmax) {
        const double mg = gld(a.margin + j) - 2.0 * dn;
        if (!((mg > a.T || stay_by_uniform(mg, gld(a.raw + j * (a.m + 1) + a.m), a.K + a.m)) && cmin[gld(a.c + j)] >= 2))
          atomicMin(&F->ufail, (int)j);
      }
    }
    __syncthreads();
    if (F->ufail != INT_MAX) break;
  }
  const int u = F->ufail;
  __syncthreads();
  if (u == INT_MAX) return hi;
  if (threadIdx.x == 0) { S.restart = 1; S.next = u; }
  return u;
}

// wave 0: the chunk's stop (F->stop_*) decided and applied by the serial path.  Not inlined:
// the serial decision's registers stay out of the fixed-point loop's allocation.
__device__ __noinline__ void fp_stop(const ResolveArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  RState st;     // rebuilt here: passing the caller's would keep its arrays out of registers
  resolve_layout(a, st, smem, false);
  FpShared* F = (FpShared*)(smem + ((resolve_lds_bytes(a.lcap, a.m, 0, 0) + 15) & ~(size_t)15));
  RCtx R{a, st, *st.sh, lane, a.S + a.m, a.scap, F->nlog, false};
  const int4 rs = F->stop_rq;
  const int pk = F->stop_pick;
  const bool given = pk != kFpFallback;
  const bool ok = R.process(rs.y, rs.x, rs.z, (uint32_t)rs.w, given ? pk : -1, 0.0, given);
  if (lane == 0) {
    F->nlog = R.nlog;
    F->go = ok ? 1 : 0;
    if (given && F->stop_fresh) st.sh->exact++;
  }
}

template <int EM>
__global__ __launch_bounds__(kFpThreads) void k_resolve_fp(ResolveArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  RState st;
  resolve_layout(a, st, smem, false);
  RShared& S = *st.sh;
  FpShared* F = (FpShared*)(smem + ((resolve_lds_bytes(a.lcap, a.m, 0, 0) + 15) & ~(size_t)15));
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool prof = a.prof != nullptr;
  if (prof) tp[0] = wall_clock64();
  if (tid == 0) { F->nlog = a.mcount ? *a.mcount : 0; F->go = 1; F->iters = 0; }
  for (int e = tid; e < 256; e += kFpThreads) F->etab[e] = devtab::kGlibcExpTab[e];
  resolve_init(a, st);
  const int total = *a.dense_total;
  const int ncol = a.S + a.m;
  const int nsl = S.nslots;      // a launch that opens a slot ends with it
  int64_t vfrom = a.p0;
  bool go = true;
  int chunks = 0;
  long long t_a = 0;
  if (prof) tp[1] = wall_clock64();
  for (int q0 = 0; q0 < total && go;) {
    ++chunks;
    if (prof) t_a = wall_clock64();
    const int nc = min(kFpThreads, total - q0);
    const bool in = tid < nc;
    const int4 r = in ? gld(a.rq + q0 + tid) : make_int4(0, 0, 0, 0);
    const int own = r.z;
    const int sp = (in && a.spec) ? gld(a.spec + q0 + tid) : -1;
    const double sr = (in && a.spec) ? gld(a.spec_rad + q0 + tid) : 0.0;
    // (the categorical uniform: fp_draw_at reads it from the record)
    F->pi[tid] = in ? r.y : INT_MAX;
    const int K = S.K, E = K + a.m;
    const bool struct0 = S.nstruct == 0;
    int cls = 0, tgt = own, pick = -1, co = 0, ct = 0;   // cls: 0 stay, 1 case-1 move to tgt, 2 stop
    // The first round's guess: the snapshot draws' outcomes in the chunk-start state (any guess
    // converges to the same fixed point; a right one does so in one round instead of two;
    // debug bit 26 starts from "stay")
    if (in && struct0 && sp >= 0 && !(a.debug_fp & 1)) {
      const bool single0 = st.cnt[own] == 1;
      if (sp < K) {
        const int s2 = st.sol[sp];
        if (!single0) { cls = s2 != own ? 1 : 0; tgt = s2; }
        else cls = 2;
      } else {
        cls = (single0 && sp == K) ? 0 : 2;
      }
    }
    bool fresh = false;
    int chg = -1, fs = nc;
    bool conv = false;
    for (int it = 0; it <= kFpThreads + 1; ++it) {
      const long long tr0 = prof ? wall_clock64() : 0;
      // (1) the first stop of the current outcomes; each wave's net count changes before it
      const unsigned long long sbal = __ballot(in && cls == 2);
      if (lane == 0) F->wstop[wv] = sbal ? wv * kWave + __ffsll((long long)sbal) - 1 : kFpThreads;
      F->wd[wv][lane] = 0;
      __syncthreads();
      fs = nc;
      for (int w = 0; w < kFpWaves; ++w) fs = min(fs, F->wstop[w]);
      const bool mover = in && cls == 1 && tid < fs;
      if (mover) {
        atomicAdd(&F->wd[wv][own], -1);
        atomicAdd(&F->wd[wv][tgt], 1);
      }
      __syncthreads();
      // (2) the counts at each wave's first point (lane = slot)
      if (wv == 0) {
        int c = lane < nsl ? st.cnt[lane] : 0;
        for (int w = 0; w < kFpWaves; ++w) {
          F->wc[w][lane] = c;
          c += F->wd[w][lane];
        }
      }
      __syncthreads();
      const long long tr1 = prof ? wall_clock64() : 0;
      // (3) the wave's moves per slot it touches (ballot masks, zero for the others): a point's
      // count change of slot s from the moves before it in its wave is
      // popc(in & below) - popc(out & below)
      F->bin[wv][lane] = 0ull;
      F->bout[wv][lane] = 0ull;
      unsigned long long touch = mover ? ((1ull << own) | (1ull << tgt)) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) touch |= __shfl_xor(touch, o);
      for (unsigned long long t = touch; t; t &= t - 1) {
        const int sl = __ffsll((long long)t) - 1;
        const unsigned long long bi = __ballot(mover && tgt == sl), bo = __ballot(mover && own == sl);
        if (lane == 0) { F->bin[wv][sl] = bi; F->bout[wv][sl] = bo; }
      }
      wave_sync();
      auto corr = [&](int sl) -> int {
        return __popcll(F->bin[wv][sl] & below) - __popcll(F->bout[wv][sl] & below);
      };
      const long long tr2 = prof ? wall_clock64() : 0;
      // (4) the points after the first changed outcome draw again (all of them in round 0).
      // Branch-free entry loops: every LDS read and table / row load of a pass is issued
      // before its values are used.
      bool changed = false;
      long long tdraw = 0;
      bool ev2 = false, need = false;   // evaluated in full this round; its draw is made this round
      int cnow2 = 0;
      const bool evl = in && tid > chg && tid <= fs;
      const double wdb = (struct0 && a.spec) ? fp_wave_drift_bound(a, st, F->wc[wv], F->bin[wv], F->bout[wv], nsl)
                                             : INFINITY;
      if (evl && struct0 && sp >= 0 && wdb < sr) {
        // every entry's drift is below this point's radius: its snapshot draw holds
        const int cnow = F->wc[wv][own] + corr(own);
        const bool single = cnow == 1;
        const int np = sp;
        fresh = false;
        int ncl = 2, nt = own;
        if (np < K) {
          const int s2 = st.sol[np];
          if (!single) { ncl = s2 != own ? 1 : 0; nt = s2; }
        } else if (single && np == K) {
          ncl = 0;
        }
        const int ctn = F->wc[wv][nt] + corr(nt);
        changed = ncl != cls || (ncl == 1 && nt != tgt);
        cls = ncl;
        tgt = nt;
        pick = np;
        co = cnow;
        ct = ctn;
      } else if (evl) {
        ev2 = true;
        cnow2 = F->wc[wv][own] + corr(own);
        // the snapshot draw holds while every log-count term drifted less than its radius
        bool take_spec = false;
        if (struct0 && sp >= 0) {
          const double drift = fp_lane_drift<EM>(st, F->wc[wv], corr, own, cnow2, K);
          take_spec = drift == 0.0 || drift < sr;
        }
        need = !take_spec;
      }
      // the draws of this round, compacted into dense waves (fp_draws_compacted)
      const long long td0 = prof ? wall_clock64() : 0;
      const int dpk = fp_draws_compacted<EM>(a, st, F, need, q0, K, E, ncol);
      if (ev2) {
        const int cnow = cnow2;
        const bool single = cnow == 1;
        int np;
        if (!need) {
          np = sp;
          fresh = false;
        } else {
          np = dpk;
          fresh = true;
        }
        if (prof && need) tdraw = wall_clock64() - td0;
        int ncl = 2, nt = own;
        if (np >= 0) {
          if (np < K) {
            const int s2 = st.sol[np];
            if (!single) { ncl = s2 != own ? 1 : 0; nt = s2; }
          } else if (single && np == K) {
            ncl = 0;
          }
        }
        const int ctn = F->wc[wv][nt] + corr(nt);
        changed = ncl != cls || (ncl == 1 && nt != tgt);
        cls = ncl;
        tgt = nt;
        pick = np;
        co = cnow;
        ct = ctn;
      }
      const unsigned long long cbal = __ballot(changed);
      if (lane == 0) F->wchg[wv] = cbal ? wv * kWave + __ffsll((long long)cbal) - 1 : kFpThreads;
      if (prof) {
        const long long tr3 = wall_clock64();
        const int ne = __popcll(__ballot(evl)), nf = __popcll(__ballot(evl && fresh));
        const long long tdm = (long long)wave_max((double)tdraw);
        if (lane == 0) {
          F->wev[wv] = tr3 - tr2;
          atomicAdd((unsigned long long*)&S.tsub[5], (unsigned long long)tdm);
          atomicAdd((unsigned long long*)&S.tsub[6], (unsigned long long)ne);
          atomicAdd((unsigned long long*)&S.tsub[7], (unsigned long long)nf);
        }
        if (tid == 0) { S.tsub[2] += tr1 - tr0; S.tsub[3] += tr2 - tr1; }
      }
      __syncthreads();
      int c2 = kFpThreads;
      for (int w = 0; w < kFpWaves; ++w) c2 = min(c2, F->wchg[w]);
      if (tid == 0) F->iters++;
      if (prof && tid == 0) {
        long long mx = 0;
        for (int w = 0; w < kFpWaves; ++w) mx = max(mx, F->wev[w]);
        S.tsub[4] += mx;
      }
      if (c2 >= kFpThreads) { conv = true; break; }
      chg = c2;
    }
    if (!conv) {       // cannot happen (at most nc + 1 rounds); stop loudly
      if (tid == 0) { S.status = 5; S.next = F->pi[0]; }   // HDPM_E_ARG
      go = false;
      break;
    }
    if (prof) { const long long t = wall_clock64(); tp[3] += t - t_a; t_a = t; }
    // ---- the walk's drift after each position (running maximum from S.dnow), count bounds
    const bool mv = in && cls == 1 && tid < fs;
    double sd = mv ? fmax(slot_drift_at(a, st, own, co - 1), slot_drift_at(a, st, tgt, ct + 1)) : 0.0;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const double x = __shfl_up(sd, o);
      if (lane >= o) sd = fmax(sd, x);
    }
    if (lane == kWave - 1) F->wsd[wv] = sd;
    if (wv == 0) F->cmo[lane] = 0;
    __syncthreads();
    if (mv) atomicAdd(&F->cmo[own], 1);
    double dpre = S.dnow;
    for (int w = 0; w < wv; ++w) dpre = fmax(dpre, F->wsd[w]);
    F->dnl[tid] = fmax(sd, dpre);
    __syncthreads();
    if (wv == 0) {
      int mn = F->wc[0][lane];
      for (int w = 1; w < kFpWaves; ++w) mn = min(mn, F->wc[w][lane]);
      F->cmin[lane] = mn - F->cmo[lane];
    }
    __syncthreads();
    // ---- unlisted points before the first stop (or before the chunk's last point)
    int kc = fs;
    {
      const int64_t hi = fs < nc ? F->pi[fs] : F->pi[nc - 1];
      const double dtop = fs > 0 ? F->dnl[fs - 1] : S.dnow;
      if (dtop > a.dmax && hi > vfrom) {
        const int64_t u = fp_verify(a, st, F, fs, S.dnow, vfrom, hi, F->cmin);
        if (u < hi) {
          int k = 0;
          while (k < fs && F->pi[k] < u) ++k;
          kc = k;
          go = false;
        }
      }
    }
    // ---- commit the positions before kc: labels, move log, counts, drifts
    const bool cm = mv && tid < kc;
    const unsigned long long mmc = __ballot(cm);
    const unsigned long long fbal = __ballot(in && tid < kc && fresh);
    if (lane == 0) { F->wmov[wv] = __popcll(mmc); F->wfresh[wv] = __popcll(fbal); }
    if (wv == 0) F->wd[0][lane] = 0;
    __syncthreads();
    if (cm) {
      a.c[r.y] = tgt;
      if (a.mlog) {
        int q = F->nlog + __popcll(mmc & below);
        for (int w = 0; w < wv; ++w) q += F->wmov[w];
        a.mlog[3 * q] = r.y;
        a.mlog[3 * q + 1] = own;
        a.mlog[3 * q + 2] = tgt;
      }
      atomicAdd(&F->wd[0][own], -1);
      atomicAdd(&F->wd[0][tgt], 1);
    }
    __syncthreads();
    if (wv == 0) {
      double cd = 0.0;
      if (lane < nsl) {
        const int dl = F->wd[0][lane];
        if (dl != 0) {
          const int c = st.cnt[lane] + dl;
          st.cnt[lane] = c;
          st.l1[lane] = fp_logn(a, c);
          st.l0[lane] = fp_logn(a, c - 1);
        }
        cd = count_drift(st, a.logn, lane);
      }
      cd = wave_max(cd);
      if (lane == 0) {
        int nm = 0, nf = 0;
        for (int w = 0; w < kFpWaves; ++w) { nm += F->wmov[w]; nf += F->wfresh[w]; }
        S.moves += nm;
        S.exact += nf;
        if (kc > 0) S.dnow = fmax(S.dnow, F->dnl[kc - 1]);
        S.dvmax = fmax(S.dvmax, cd);
        if (a.mlog) F->nlog += nm;
      }
    }
    if (tid == fs) {
      F->stop_rq = r;
      F->stop_pick = pick;
      F->stop_fresh = fresh ? 1 : 0;
    }
    __syncthreads();
    if (prof) { const long long t = wall_clock64(); tp[4] += t - t_a; t_a = t; }
    if (!go) break;
    if (fs < nc) {
      // ---- the stop: the serial path in the committed state (that of its turn)
      const int4 rs = F->stop_rq;
      if (wv == 0) fp_stop(a);
      __syncthreads();
      go = F->go != 0;
      vfrom = (int64_t)rs.y + 1;
      q0 += fs + 1;
      if (prof) { tp[2] += wall_clock64() - t_a; tp[6] += 1; }
    } else {
      vfrom = (int64_t)F->pi[nc - 1] + 1;
      q0 += nc;
    }
    __syncthreads();
  }
  if (go && S.status == 0 && !S.restart && S.dnow > a.dmax) (void)fp_verify(a, st, F, 0, S.dnow, vfrom, a.n, st.cnt);
  // prof: [1] start of the walk, [2] stop ticks, [3] fixed-point rounds ticks, [4] drift /
  // re-test / commit ticks, [5] rounds, [6] stops; tsub[0] chunks, tsub[1] listed
  if (prof && tid == 0) { tp[5] = F->iters; S.tsub[0] = chunks; S.tsub[1] = total; }
  resolve_finish(a, st, F->nlog, tp, prof);
}

#include "resolve_fpg.inl"

// ------------------------------------------------------------------ end of sweep
// The sweep-end kernels are enqueued behind every resolver launch and read its control
// block: they act only when that launch finished the sweep, so the host need not wait for
// the resolver before issuing them.  A launch whose last point opened a cluster (case 3 /
// case 4 set `restart` with next = i + 1) has finished it too when i is the last point:
// `next >= n` alone decides (every restart that leaves work sets next < n).
__device__ __forceinline__ bool sweep_done(const ResolveCtl* ctl, int n) {
  return ctl->status == 0 && ctl->next >= n;
}

__global__ void k_relabel(int* c, const int* label_of_slot, int n, const ResolveCtl* ctl) {
  if (!sweep_done(ctl, n)) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = label_of_slot[c[i]];
}

// Incremental sufficient statistics: every logged reassignment moves the point's codes
// from one slot's frequency table to the other's (one wave per move, lanes over
// attributes).  Equivalent to recounting, at the cost of the moves.
__global__ __launch_bounds__(kWave) void k_apply_moves(const int* __restrict__ mlog, const int* __restrict__ mcount,
                                                      const uint8_t* __restrict__ codes_t, int d, int nq, int mmax,
                                                      unsigned int* freq, const ResolveCtl* ctl, int n) {
  if (!sweep_done(ctl, n)) return;
  const int nm = *mcount;
  const int fs = d * mmax;
  for (int q = blockIdx.x; q < nm; q += gridDim.x) {
    const int64_t i = mlog[3 * q];
    const int from = mlog[3 * q + 1], to = mlog[3 * q + 2];
    for (int j = threadIdx.x; j < d; j += kWave) {
      const int x = a_code(codes_t, i, j, nq) - 1;
      atomicSub(freq + (int64_t)from * fs + j * mmax + x, 1u);
      atomicAdd(freq + (int64_t)to * fs + j * mmax + x, 1u);
    }
  }
}

// The same with the deltas of the first ls slots accumulated in LDS per workgroup (a
// contiguous share of the move log each) and added once per changed counter: from a random
// start half the points move per sweep, and per-move global atomics on the few thousand
// counters of the tables serialised (3-4.6 ms per C5 sweep).  Moves of slots >= ls (past
// the LDS budget) update the global tables directly.
__global__ __launch_bounds__(256) void k_apply_moves_lds(const int* __restrict__ mlog, const int* __restrict__ mcount,
                                                        const uint8_t* __restrict__ codes_t, int d, int nq, int mmax,
                                                        unsigned int* freq, const ResolveCtl* ctl, int n, int ls) {
  if (!sweep_done(ctl, n)) return;
  const int nm = *mcount;
  const int per = (nm + (int)gridDim.x - 1) / (int)gridDim.x;
  const int q0 = (int)blockIdx.x * per, q1 = min(nm, q0 + per);
  if (q0 >= q1) return;
  extern __shared__ int dl[];          // [ls][d * mmax] count changes
  const int fs = d * mmax;
  for (int e = threadIdx.x; e < ls * fs; e += blockDim.x) dl[e] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nwv = blockDim.x >> 6;
  for (int q = q0 + wv; q < q1; q += nwv) {
    const int64_t i = mlog[3 * q];
    const int from = mlog[3 * q + 1], to = mlog[3 * q + 2];
    for (int j = lane; j < d; j += kWave) {
      const int off = j * mmax + a_code(codes_t, i, j, nq) - 1;
      if (from < ls) atomicSub(&dl[from * fs + off], 1);
      else atomicSub(freq + (int64_t)from * fs + off, 1u);
      if (to < ls) atomicAdd(&dl[to * fs + off], 1);
      else atomicAdd(freq + (int64_t)to * fs + off, 1u);
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < ls * fs; e += blockDim.x) {
    const int v = dl[e];
    if (v) atomicAdd(freq + e, (unsigned)v);
  }
}

// freq per label after the sweep: out[l] = freq[slot_of_label[l]].
__global__ void k_freq_gather(const unsigned int* __restrict__ freq, const int* __restrict__ sol, int fs,
                              unsigned int* __restrict__ out, const ResolveCtl* ctl, int n) {
  if (!sweep_done(ctl, n)) return;
  const int K = ctl->K;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)K * fs;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(e / fs);
    out[e] = freq[(int64_t)sol[l] * fs + (e - (int64_t)l * fs)];
  }
}

// After k_relabel: counts per label, identity slot maps (slot == label again).  One block.
__global__ __launch_bounds__(1024) void k_finish_sweep(int* counts, int* sol, int* los, int* src,
                                                      const ResolveCtl* ctl, int n) {
  if (!sweep_done(ctl, n)) return;
  const int K = ctl->K, nslots = ctl->nslots;
  extern __shared__ int fs[];
  int* c = fs;            // [nslots]
  int* m = fs + nslots;   // [K]
  for (int s = threadIdx.x; s < nslots; s += blockDim.x) c[s] = counts[s];
  for (int l = threadIdx.x; l < K; l += blockDim.x) m[l] = sol[l];
  __syncthreads();
  for (int l = threadIdx.x; l < K; l += blockDim.x) {
    counts[l] = c[m[l]];
    sol[l] = l;
    los[l] = l;
    src[l] = -1;
  }
}

// Cluster parameter upload (UploadLayout) from the staging buffer.  With `sum` (full uploads
// of entry r = label r = slot r, the pipelined sweep's), also k_cluster_summary's work for the
// round that follows: the per-label summaries straight from the staged records and counts,
// and its counter clears -- one launch fewer on the sweep's path.
struct ScatterSummary {
  uint64_t* csum;           // [nent][bw + 2]: record, logn[count], slot
  const double* logn;
  int* zero;                // cleared (nullable)
  int* wide_ctr;            // [3] cleared
};
__global__ void k_scatter_clusters(const uint8_t* __restrict__ stage, int nent, int dp, int d, int bw, int full,
                                   uint8_t* codes, double* tab, uint64_t* bnd, int* counts, int* sol, int* los,
                                   int* src, const int* gate, ScatterSummary sum) {
  if (gate_closed(gate)) return;
  const UploadLayout L = upload_layout(nent, dp, d, bw);
  const int* slot = (const int*)(stage + L.off_slot);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  if (sum.csum) {
    if (tid == 0) {
      if (sum.zero) *sum.zero = 0;
      sum.wide_ctr[0] = 0;
      sum.wide_ctr[1] = 0;
      sum.wide_ctr[2] = 0;
    }
    const int sw = bw + 2;
    const int* scount = (const int*)(stage + L.off_counts);
    for (int64_t q = tid; q < (int64_t)nent * sw; q += nth) {
      const int l = (int)(q / sw), w = (int)(q - (int64_t)l * sw);
      uint64_t v;
      if (w < bw) v = ((const uint64_t*)(stage + L.off_bnd))[(int64_t)l * bw + w];
      else if (w == bw) v = (uint64_t)__double_as_longlong(sum.logn[scount[l]]);
      else v = (uint64_t)l;
      sum.csum[q] = v;
    }
  }
  const int tw = 2 * d;
  for (int64_t q = tid; q < (int64_t)nent * tw; q += nth) {
    const int r = (int)(q / tw), o = (int)(q - (int64_t)r * tw);
    tab[(int64_t)slot[r] * tw + o] = ((const double*)(stage + L.off_tab))[q];
  }
  for (int64_t q = tid; q < (int64_t)nent * bw; q += nth) {
    const int r = (int)(q / bw), o = (int)(q - (int64_t)r * bw);
    bnd[(int64_t)slot[r] * bw + o] = ((const uint64_t*)(stage + L.off_bnd))[q];
  }
  for (int64_t q = tid; q < (int64_t)nent * dp; q += nth) {
    const int r = (int)(q / dp), o = (int)(q - (int64_t)r * dp);
    codes[(int64_t)slot[r] * dp + o] = stage[L.off_codes + q];
  }
  if (full)
    for (int64_t r = tid; r < nent; r += nth) {
      counts[r] = ((const int*)(stage + L.off_counts))[r];
      sol[r] = (int)r;
      los[r] = (int)r;
      src[r] = -1;
    }
}

__global__ __launch_bounds__(kBlock) void k_hist_global(HistArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / a.nq;
  const int q = (int)(t % a.nq);
  if (i >= a.n) return;
  const int k = a.label[i];
  if (a.mask && !a.mask[k]) return;
  for (int b = 0; b < 16; ++b) {
    const int j = q * 16 + b;
    if (j >= a.d) break;
    const int x = a.codes_t[tiled_offset(i, j, a.nq)];
    atomicAdd(a.freq + ((int64_t)k * a.d + j) * a.mmax + (x - 1), 1u);
  }
}

// freq from the packed rows.  A workgroup (16 waves, one per CU) owns a contiguous range
// of 64-point tiles and a slice of KC labels.  Per tile, lane p loads point p's packed row
// (coalesced) into its wave's LDS stage; then the wave walks the points with lanes over
// attributes: lane j reads field j of the point (broadcast read) and adds 1 to
// h[(k - k0) * mmax + x][j] with a non-returning LDS atomic (consecutive banks: no
// conflicts).  Points outside the slice count into a trash row, so the loop is
// branch-free and unrolled over 8 points to keep reads in flight.  Each workgroup writes
// its counters to `partial`; k_hist_reduce sums them into freq[k][j][x].
constexpr int kHistBlock = 1024;
constexpr int kHistUnroll = 8;
__global__ __launch_bounds__(kHistBlock) void k_hist_packed(HistArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int row = a.mmax * a.d;
  const int hsize = a.KC * row;
  const int halloc = hsize + row;                           // + trash row
  unsigned int* h = (unsigned int*)smem;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* stg = (uint64_t*)(smem + (((size_t)halloc * 4 + 15) / 16) * 16) + (size_t)wv * a.W * 64;
  for (int e = threadIdx.x; e < halloc; e += kHistBlock) h[e] = 0u;
  __syncthreads();
  const int k0 = blockIdx.y * a.KC;
  const int64_t ntiles = ((int64_t)a.n + 63) / 64;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_block;
  const int64_t t1 = min(ntiles, t0 + a.tiles_per_block);
  const int W = a.W, wb = a.wb, d = a.d;
  const uint64_t fmask = (1ull << wb) - 1ull;
  for (int64_t t = t0 + wv; t < t1; t += kHistBlock / kWave) {
    const int64_t i = t * 64 + lane;
    int kk = a.KC;
    if (i < a.n) {
      const int k = a.label[i];
      if ((!a.mask || a.mask[k]) && k >= k0 && k < k0 + a.KC) kk = k - k0;
    }
    const int kbase = kk * row;
    for (int q = 0; q < W; ++q) stg[q * 64 + lane] = i < a.n ? a.xpk[packed_offset(i, q, W)] : 0ull;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int jb = 0; jb < d; jb += 64) {
      const int j = jb + lane;
      const bool on = j < d;
      const int bit = (on ? j : 0) * wb;
      const uint64_t* sw = stg + (bit >> 6) * 64;
      const int sh = bit & 63;
      for (int p = 0; p < 64; p += kHistUnroll) {
        uint64_t w[kHistUnroll];
        int kb[kHistUnroll];
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
          w[u] = sw[p + u];
          kb[u] = __builtin_amdgcn_readlane(kbase, p + u);
        }
#pragma unroll
        for (int u = 0; u < kHistUnroll; ++u) {
          const int x = (int)((w[u] >> sh) & fmask);
          if (on) __hip_atomic_fetch_add(h + kb[u] + x * d + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();
  unsigned int* dst = a.partial + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * hsize;
  for (int e = threadIdx.x; e < hsize; e += kHistBlock) dst[e] = h[e];
}

// freq[k][j][x] += sum of a group of workgroup partials (freq zeroed first).
constexpr int kHistReduceSplit = 16;
__global__ __launch_bounds__(256) void k_hist_reduce(HistArgs a, int nbx) {
  const int hsize = a.KC * a.mmax * a.d;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= hsize) return;
  const int per = (nbx + kHistReduceSplit - 1) / kHistReduceSplit;
  const int b0 = blockIdx.z * per, b1 = min(nbx, b0 + per);
  if (b0 >= b1) return;
  const unsigned int* src = a.partial + (size_t)blockIdx.y * nbx * hsize + e;
  unsigned int s = 0;
  for (int b = b0; b < b1; ++b) s += src[(size_t)b * hsize];
  const int kk = e / (a.mmax * a.d), rem = e - kk * a.mmax * a.d;
  const int x = rem / a.d, j = rem - x * a.d;
  const int k = blockIdx.y * a.KC + kk;
  if (k < a.K && s) atomicAdd(a.freq + ((size_t)k * a.d + j) * a.mmax + x, s);
}

// compute_loglikelihood: exact per-point own-cluster log-likelihood (j order), then a
// compensated (two-sum) reduction; partial[2*block] = (hi, lo).
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

__global__ __launch_bounds__(kBlock) void k_loglik(LoglikArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double hi = 0.0, lo = 0.0;
  if (i < a.n) {
    const int k = a.label[i];
    const int dp = a.nq * 16;
    PointCodes<0> x;
    x.load(a.codes_t, i, a.nq);
    hi = ll_lane<0>(x, a.d, a.cl.codes + (int64_t)k * dp, a.cl.tab + (int64_t)k * 2 * a.d, nullptr);
  }
  // wave reduction with error terms
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double oh = __shfl_xor(hi, o), ol = __shfl_xor(lo, o);
    double s, e;
    two_sum(hi, oh, s, e);
    hi = s;
    lo = lo + ol + e;
  }
  __shared__ double sh[kBlock / kWave][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { sh[wv][0] = hi; sh[wv][1] = lo; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double H = 0.0, Lo = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) {
      double s, e;
      two_sum(H, sh[w][0], s, e);
      H = s;
      Lo += sh[w][1] + e;
    }
    a.partial[2 * blockIdx.x] = H;
    a.partial[2 * blockIdx.x + 1] = Lo;
  }
}

// Test/diagnostic kernel: L[k*ldL + i] and Hamming counts H[k*ldL + i] for K label tables.
__global__ __launch_bounds__(kBlock) void k_lmatrix(const uint8_t* codes_t, int n, int d, int nq,
                                                   ParamTables cl, int K, double* L, int* H, int64_t ldL) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int dp = nq * 16;
  PointCodes<0> x;
  x.load(codes_t, i, nq);
  for (int k = 0; k < K; ++k) {
    int h;
    const double ll = ll_lane<0>(x, d, cl.codes + (int64_t)k * dp, cl.tab + (int64_t)k * 2 * d, &h);
    L[(int64_t)k * ldL + i] = ll;
    H[(int64_t)k * ldL + i] = h;
  }
}

// ------------------------------------------------------------------ launchers
template <int WB, int WS, bool HEAD>
static hipError_t launch_prepass_t(const PrepassArgs& a, int nblocks, hipStream_t s) {
  HDPM_LAUNCH((k_prepass<WB, WS, HEAD>), dim3(nblocks), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <int WB>
static hipError_t launch_prepass_w(const PrepassArgs& a, int nblocks, hipStream_t s) {
  if (a.Ws == 2) {
    if (a.pool_head) return launch_prepass_t<WB, 2, true>(a, nblocks, s);
    return launch_prepass_t<WB, 2, false>(a, nblocks, s);
  }
  if constexpr (WB <= 4) {
    if (a.Ws == 4) {
      if (a.pool_head) return launch_prepass_t<WB, 4, true>(a, nblocks, s);
      return launch_prepass_t<WB, 4, false>(a, nblocks, s);
    }
  }
  if (a.wide && wide_fits(WB, a.Ws) && prepass_wide_offsets_fit(a)) {
    // cluster summaries in LDS while they fit beside the rows (9 KB at C4 with K = 10), for
    // the instances that keep it without spilling (wb Ws <= 64 leaves NW = 2 to wb <= 2)
    constexpr bool kClOk = WB == 1 || WB == 4;
    const bool cl = kClOk && prepass_wide_lds_bytes(WB, a.Ws, a.m, a.K, a.bw, true) <= 40 * 1024;
    const size_t lds = prepass_wide_lds_bytes(WB, a.Ws, a.m, a.K, a.bw, cl);
    const int nchunks = (a.n - a.p0 + kWideChunk - 1) / kWideChunk;
    auto go = [&](auto kern) {
      // (the same number of chunks for every workgroup -- 875 workgroups x 5 chunks at C4 instead of
      // 1,024 x 4-5 -- measured 54 against 47 us: the kernel wants every resident wave)
      const int grid = std::min(nchunks, wide_grid(kern, lds, a.wide_per_cu));
      // HDPM_WIDE_CLAIM=1: chunks claimed from a counter (A/B; see k_prepass_wide)
      static const int claim = [] {
        const char* e = std::getenv("HDPM_WIDE_CLAIM");
        return e ? std::atoi(e) : 0;
      }();
      HDPM_LAUNCH(kern, dim3(grid), dim3(kWideThreads), lds, s, a, nchunks, claim);
      return hipGetLastError();
    };
    if constexpr (WB <= 2) {
      if (a.Ws > 16) return cl ? go(k_prepass_wide<WB, 2, kClOk>) : go(k_prepass_wide<WB, 2, false>);
    }
    return cl ? go(k_prepass_wide<WB, 1, kClOk>) : go(k_prepass_wide<WB, 1, false>);
  }
  HDPM_LAUNCH(k_prepass_generic, dim3(nblocks), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// Exact rows when nearly every point is listed (a chain from a random start: ~1M per C5 sweep;
// the dense list comes from k_list_scan).  Persistent workgroups of 8 waves, a wave per point,
// lane e per entry (E <= 64).  The K clusters' codes and tables are staged in LDS once per
// workgroup; per point the wave gathers the m latent entries' selected table values (all
// lanes, every load of a batch in flight) into LDS, then lane e adds its entry's D values in
// attribute order (n8:47-49; bit-exact) from LDS and the wave draws the snapshot decision.
constexpr int kMassWaves = 8;
__host__ __device__ inline size_t exact_mass_lds_bytes(int K, int m, int d, int dp) {
  return (size_t)K * 2 * d * 8 + (size_t)kMassWaves * m * d * 8 + (size_t)K * dp + (size_t)kMassWaves * dp;
}

// exact_rows_decide with the launch's snapshot per entry in LDS: slot, count, log-counts
__device__ __forceinline__ void mass_decide(const PrepassArgs& a, int q, int own, double acc, uint32_t rawm,
                                            const int* s_sl, const int* s_cnt, const double* s_l0, const double* s_l1,
                                            double* lp, int* lperm, int* lpick) {
  const int lane = threadIdx.x & 63;
  const int K = a.K, E = K + a.m;
  const bool clu = lane < K;
  const int s = clu ? s_sl[lane] : -1;
  const unsigned long long bo = __ballot(clu && s == own);
  const int lo = bo ? __ffsll((long long)bo) - 1 : 0;
  const double ll_own = readlane_f64(acc, lo);
  const int own_cnt = __shfl(clu ? s_cnt[lane] : 0, lo);
  double v = -INFINITY;
  if (clu) v = (s == own ? s_l0[lane] : s_l1[lane]) + acc;                         // n8:40-92
  else if (lane < E) v = a.logfac + ((lane == K && own_cnt == 1) ? ll_own : acc);
  double pv[1] = {v};
  double rad = 0.0;
  const int pick = decide_values<1>(pv, E, raw_to_unif(rawm), lp, lperm, lpick, &rad);
  if (lane == 0) {
    a.spec[q] = pick >= 0 ? pick : -1;
    a.spec_rad[q] = rad;
  }
}

__global__ __launch_bounds__(kWave * kMassWaves) void k_exact_rows_mass(PrepassArgs a, int order_static) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double lp_w[kMassWaves][kWave];
  __shared__ int lperm_w[kMassWaves][kWave];
  __shared__ int lpick_w[kMassWaves];
  __shared__ int s_sl[kWave], s_cnt[kWave];
  __shared__ double s_l0[kWave], s_l1[kWave];
  const int K = a.K, m = a.m, E = K + m, D = a.d, dp = a.nq * 16, m1 = m + 1;
  double* ltab = (double*)smem;                                  // [K][2D]
  double* lval0 = ltab + (size_t)K * 2 * D;                       // [waves][m][D]
  uint8_t* lcode = (uint8_t*)(lval0 + (size_t)kMassWaves * m * D);  // [K][dp]
  uint8_t* lx0 = lcode + (size_t)K * dp;                          // [waves][dp]
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int q = tid; q < K * 2 * D; q += blockDim.x) {
    const int e = q / (2 * D);
    ltab[q] = a.slots.tab[(int64_t)a.slot_of_label[e] * 2 * D + (q - e * 2 * D)];
  }
  for (int q = tid; q < K * dp; q += blockDim.x) {
    const int e = q / dp;
    lcode[q] = a.slots.codes[(int64_t)a.slot_of_label[e] * dp + (q - e * dp)];
  }
  if (tid < K) {
    const int sl = a.slot_of_label[tid], c = a.counts[sl];
    s_sl[tid] = sl;
    s_cnt[tid] = c;
    s_l1[tid] = a.logn[c];
    s_l0[tid] = a.logn[c - 1];
  }
  __syncthreads();
  const int total = *a.dense_total;
  double* lval = lval0 + (size_t)wv * m * D;
  uint8_t* lx = lx0 + (size_t)wv * dp;
  const bool clu = lane < K, on = lane < E;
  const int col = clu ? s_sl[lane] : a.S + (lane - K);
  // lane's row of values: a cluster's table (stride 2, the mismatch value selected by the code
  // compare) or the wave's gathered latent values (stride 1); 32-bit offsets in doubles from
  // the start of the LDS block
  const double* lds_d = (const double*)smem;
  const int boff = clu ? lane * 2 * D : (int)(lval - lds_d) + (on ? lane - K : 0) * D;
  const int stride = clu ? 2 : 1;
  const uint8_t* cl = lcode + (size_t)(clu ? lane : 0) * dp;
  // batches of kMassBatch points claimed from a counter (k_cluster_summary clears it; a
  // workgroup that is not resident leaves its share to the others); the batch's records
  // (k_list_fill wrote them to rq) and stream draws are loaded together, one lane per word
  // (order_static: batch b = wave + k waves of the grid instead, no claims -- A/B, HDPM_MASS_STATIC)
  constexpr int kMassBatch = 4;
  for (int bi = 0;; ++bi) {
    int q0 = 0;
    if (order_static) {
      q0 = (int)(((int64_t)blockIdx.x * kMassWaves + wv + (int64_t)bi * gridDim.x * kMassWaves) * kMassBatch);
    } else {
      if (lane == 0) q0 = atomicAdd(a.wide_ctr + 1, kMassBatch);
      q0 = __shfl(q0, 0);
    }
    if (q0 >= total) break;
    const int nb = min(kMassBatch, total - q0);
    const int kq = lane >> 4, wq = lane & 15;                     // point of the batch, word
    int4 rec = make_int4(0, 0, 0, 0);
    if (kq < nb) rec = a.rq[q0 + kq];
    uint32_t rw = 0;
    if (kq < nb && wq < m1 && m1 <= 16) rw = a.raw[(int64_t)rec.y * m1 + wq];
    for (int k = 0; k < nb; ++k) {
      const int q = q0 + k;
      const int row = __shfl(rec.x, 16 * k), own = __shfl(rec.z, 16 * k);
      const int64_t i = __shfl(rec.y, 16 * k);
      const uint32_t rawm = (uint32_t)__shfl(rec.w, 16 * k);
      if (lane < a.nq) *(uint4*)(lx + lane * 16) = *(const uint4*)(a.codes_t + tiled_offset(i, lane * 16, a.nq));
      // latent values: (u, j) pairs over the lanes, a batch of 8 per lane with every load issued first
      // (the point's m latent draws come from the 16 words its lane group loaded; with m + 1 > 16
      // words each lane reads its draw from the stream itself)
      for (int b0 = 0; b0 < m * D; b0 += 8 * kWave) {
        uint8_t cc[8];
        double2 pr[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int idx = b0 + t * kWave + lane;
          const int u = idx / D;
          const uint32_t y = m1 <= 16 ? (uint32_t)__shfl((int)rw, 16 * k + min(u, m - 1))
                                      : a.raw[i * m1 + min(u, m - 1)];
          if (idx < m * D) {
            const int j = idx - u * D;
            const int64_t pe = pick_entry(y, a.P);
            cc[t] = a.pool.codes[pe * dp + j];
            pr[t] = *(const double2*)(a.pool.tab + (pe * D + j) * 2);
          }
        }
        wave_sync();                   // lx of this point is in
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int idx = b0 + t * kWave + lane;
          if (idx < m * D) {
            const int u = idx / D, j = idx - u * D;
            lval[u * D + j] = lx[j] != cc[t] ? pr[t].y : pr[t].x;
          }
        }
      }
      wave_sync();
      // lane e's entry in attribute order (n8:47-49), 16 values loaded before they are added;
      // padding past D adds +0.0, which leaves the sum unchanged
      double acc = 0.0;
      int off = boff;
      for (int j0 = 0; j0 < D; j0 += 16, off += 16 * stride) {
        const uint4 xw = *(const uint4*)(lx + j0);
        const uint4 cw = clu ? *(const uint4*)(cl + j0) : xw;
        // bit 0 of each byte: the codes differ (the mismatch value)
        uint32_t nz[4] = {xw.x ^ cw.x, xw.y ^ cw.y, xw.z ^ cw.z, xw.w ^ cw.w};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          uint32_t t = nz[w];
          t |= t >> 4;
          t |= t >> 2;
          t |= t >> 1;
          nz[w] = t & 0x01010101u;
        }
        double v[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const int sel = (int)((nz[b >> 2] >> (8 * (b & 3))) & 1u);
          v[b] = j0 + b < D ? lds_d[off + b * stride + sel] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < 16; ++b) acc += v[b];
      }
      if (on) a.L[(int64_t)row * (a.S + m) + col] = acc;
      if (a.spec) mass_decide(a, q, own, acc, rawm, s_sl, s_cnt, s_l0, s_l1, lp_w[wv], lperm_w[wv], &lpick_w[wv]);
      wave_sync();                     // lx / lval are rewritten by the next point
    }
  }
}

// Exact rows with a thread per listed point, for sweeps without snapshot draws (nearly every
// point listed: the device-wide resolver draws them all) and D <= 128.  The K clusters' codes
// and (match, mismatch) pairs are staged in LDS; every lane of a wave reads the same pair at
// the same time (a broadcast) and selects by its own point's code, four clusters' sums
// interleaved; the m latent entries are walked per lane, 16 attributes per step.  Each sum runs
// in attribute order (n8:47-49), so every row is bit-exact; ~5 VALU per (entry, attribute) for
// 64 points at once instead of a wave per point.  Dynamic LDS: K (2 D 8 + dp) bytes.
constexpr int kLanesMaxNq = 8;
__global__ __launch_bounds__(256) void k_exact_rows_lanes(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int K = a.K, m = a.m, D = a.d, nq = a.nq, dp = nq * 16;
  double* ltab = (double*)smem;                                   // [K][D][2]
  uint8_t* lcode = (uint8_t*)(ltab + (size_t)K * 2 * D);          // [K][dp]
  __shared__ int s_col[kWave];
  for (int q = threadIdx.x; q < K * 2 * D; q += blockDim.x) {
    const int e = q / (2 * D);
    ltab[q] = a.slots.tab[(int64_t)a.slot_of_label[e] * 2 * D + (q - e * 2 * D)];
  }
  for (int q = threadIdx.x; q < K * dp; q += blockDim.x) {
    const int e = q / dp;
    lcode[q] = a.slots.codes[(int64_t)a.slot_of_label[e] * dp + (q - e * dp)];
  }
  if (threadIdx.x < K) s_col[threadIdx.x] = a.slot_of_label[threadIdx.x];
  __syncthreads();
  const int total = *a.dense_total;
  const int stride = gridDim.x * blockDim.x;
  for (int q0 = blockIdx.x * blockDim.x; q0 < total; q0 += stride) {   // uniform trip count per block
    const int q = q0 + threadIdx.x;
    const bool on = q < total;
    const int4 r = on ? a.rq[q] : make_int4(0, 0, 0, 0);
    const int64_t i = r.y;
    double* Lr = a.L + (int64_t)r.x * (a.S + m);
    uint32_t xw[4 * kLanesMaxNq];
#pragma unroll
    for (int c = 0; c < kLanesMaxNq; ++c) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < nq) v = *(const uint4*)(a.codes_t + tiled_offset(i, c * 16, nq));
      xw[4 * c] = v.x; xw[4 * c + 1] = v.y; xw[4 * c + 2] = v.z; xw[4 * c + 3] = v.w;
    }
    for (int k0 = 0; k0 < K; k0 += 4) {
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      const double* tb[4];
      const uint8_t* cb[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = min(k0 + kk, K - 1);
        tb[kk] = ltab + (size_t)k * 2 * D;
        cb[kk] = lcode + (size_t)k * dp;
      }
#pragma unroll
      for (int c = 0; c < kLanesMaxNq; ++c) {
        if (c >= nq) break;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t x4 = xw[4 * c + w];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const uint32_t c4 = *(const uint32_t*)(cb[kk] + c * 16 + 4 * w);
            const uint32_t dx = x4 ^ c4;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const int j = c * 16 + 4 * w + b;
              if (j < D) {
                const double2 pr = *(const double2*)(tb[kk] + 2 * j);
                acc[kk] += ((dx >> (8 * b)) & 0xffu) ? pr.y : pr.x;
              }
            }
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        if (on && k0 + kk < K) Lr[s_col[k0 + kk]] = acc[kk];
    }
    const uint32_t* raw = a.raw + i * (m + 1);
    for (int u = 0; u < m; ++u) {
      const int64_t pe = on ? pick_entry(raw[u], a.P) : 0;
      const uint8_t* cc = a.pool.codes + pe * dp;
      const double* tl = a.pool.tab + pe * 2 * D;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < kLanesMaxNq; ++c) {
        if (c >= nq) break;
        const uint4 cq = *(const uint4*)(cc + c * 16);
        const uint32_t cw[4] = {cq.x, cq.y, cq.z, cq.w};
        double v[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const int j = c * 16 + b;
          const uint32_t dx = xw[4 * c + (b >> 2)] ^ cw[b >> 2];
          v[b] = j < D ? tl[2 * j + (((dx >> (8 * (b & 3))) & 0xffu) ? 1 : 0)] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < 16; ++b) acc += v[b];
      }
      if (on) Lr[a.S + u] = acc;
    }
  }
}

// The same with the clusters' values in a level-indexed LDS table: vt[j][l][k] = the value
// cluster k contributes at attribute j for a point of level l + 1 -- dhamming's match value if
// l + 1 is its center's level there, else its mismatch value (n8:47-49 -> cf:355-377) -- so a
// lane reads its own point's value directly (one address per level: no bank conflicts, no
// compare / select), two clusters per 16-B read.  Sums per cluster in attribute order as
// before (bit-exact).  One workgroup of 16 waves per CU (the table: K D mmax 8 bytes, 80 KB at
// C5), a thread per listed point; the latent entries as in k_exact_rows_lanes.
constexpr int kLvThreads = 1024;
constexpr int kLvGroup = 4;       // clusters summed together (accumulators per lane)
__host__ __device__ inline int exact_lv_kp(int K) { return (K + kLvGroup - 1) / kLvGroup * kLvGroup; }
// [dp][mmax][KP] doubles: clusters padded to whole groups, attributes to the 16-byte code
// chunks (zeros: the padding adds +0.0 to every sum, so no lane or attribute branches)
__host__ __device__ inline size_t exact_lv_lds_bytes(int K, int nq, int mmax) {
  return (size_t)exact_lv_kp(K) * nq * 16 * mmax * 8;
}
__global__ __launch_bounds__(kLvThreads) void k_exact_rows_lv(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) double vt[];
  __shared__ int s_col[kWave];
  const int K = a.K, m = a.m, D = a.d, nq = a.nq, dp = nq * 16, mm = a.mmax;
  const int KP = exact_lv_kp(K);
  const int per = mm * KP;                        // doubles per attribute
  for (int q = threadIdx.x; q < dp * per; q += blockDim.x) {
    const int j = q / per, r = q - j * per, l = r / KP, k = r - l * KP;
    double v = 0.0;
    if (k < K && j < D) {
      const int64_t sl = a.slot_of_label[k];
      const int c = a.slots.codes[sl * dp + j];
      v = a.slots.tab[(sl * D + j) * 2 + (c == l + 1 ? 0 : 1)];
    }
    vt[q] = v;
  }
  __shared__ double s_l0[kWave], s_l1[kWave];    // the launch's log-counts (latent bounds)
  if (threadIdx.x < K) {
    const int sl = a.slot_of_label[threadIdx.x], c = a.counts[sl];
    s_col[threadIdx.x] = sl;
    s_l1[threadIdx.x] = a.logn[c];
    s_l0[threadIdx.x] = c > 0 ? a.logn[c - 1] : -INFINITY;
  }
  __syncthreads();
  const int total = *a.dense_total;
  const int stride = gridDim.x * blockDim.x;
  const bool lb = a.lbound && a.lmask && a.pool_head && m <= 32;
  for (int q0 = blockIdx.x * blockDim.x; q0 < total; q0 += stride) {
    const int q = q0 + threadIdx.x;
    const bool on = q < total;
    const int4 r = on ? a.rq[q] : make_int4(0, 0, 0, 0);
    const int64_t i = r.y;
    const int own = r.z;
    double* Lr = a.L + (int64_t)r.x * (a.S + m);
    double mxc = -INFINITY;         // the best cluster log-weight in the launch's state (n8:40-92)
    uint32_t xw[4 * kLanesMaxNq];
#pragma unroll
    for (int c = 0; c < kLanesMaxNq; ++c) {
      uint4 v = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
      if (c < nq && on) v = *(const uint4*)(a.codes_t + tiled_offset(i, c * 16, nq));
      xw[4 * c] = v.x; xw[4 * c + 1] = v.y; xw[4 * c + 2] = v.z; xw[4 * c + 3] = v.w;
    }
    for (int k0 = 0; k0 < K; k0 += kLvGroup) {
      double acc[kLvGroup];
#pragma unroll
      for (int kk = 0; kk < kLvGroup; ++kk) acc[kk] = 0.0;
      const double* g = vt + k0;
      // (KP laundered per group: the per-attribute offsets l KP would otherwise be hoisted out
      // of the group loop, 128 live values, and spilled)
      int kpl = KP;
      asm volatile("" : "+s"(kpl));
#pragma unroll
      for (int c = 0; c < kLanesMaxNq; ++c) {
        if (c >= nq) break;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t x4 = xw[4 * c + w];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int j = c * 16 + 4 * w + b;
            // a padding attribute's byte is 0: level 1's row of zeros
            const int x = (int)((x4 >> (8 * b)) & 0xffu);
            const int l = (x > 0 ? x : 1) - 1;
            const double2* p = (const double2*)(g + j * per + l * kpl);
#pragma unroll
            for (int kk = 0; kk < kLvGroup; kk += 2) {
              const double2 v = p[kk >> 1];
              acc[kk] += v.x;
              acc[kk + 1] += v.y;
            }
          }
          // (the scheduler would issue every LDS read of the unrolled attributes first and spill)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int kk = 0; kk < kLvGroup; ++kk) {
        const int k = k0 + kk;
        if (k < K) {
          const int sl = s_col[k];
          if (on) Lr[sl] = acc[kk];
          mxc = fmax(mxc, (sl == own ? s_l0[k] : s_l1[k]) + acc[kk]);
        }
      }
    }
    const uint32_t* raw = a.raw + i * (m + 1);
    unsigned int lm = 0;
    for (int u = 0; u < m; ++u) {
      const int64_t pe = on ? pick_entry(raw[u], a.P) : 0;
      if (lb && on) {
        // far below the clusters: its head bound stands for it (latent_exact's readers)
        const double ub = latent_head_ub(a, i, pe);
        if (a.logfac + ub <= mxc - kLatMargin) {
          Lr[a.S + u] = ub;
          lm |= 1u << u;
          continue;
        }
      }
      const uint8_t* cc = a.pool.codes + pe * dp;
      const double* tl = a.pool.tab + pe * 2 * D;
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < kLanesMaxNq; ++c) {
        if (c >= nq) break;
        const uint4 cq = *(const uint4*)(cc + c * 16);
        const uint32_t cw[4] = {cq.x, cq.y, cq.z, cq.w};
        double v[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const int j = c * 16 + b;
          const uint32_t dx = xw[4 * c + (b >> 2)] ^ cw[b >> 2];
          v[b] = j < D ? tl[2 * j + (((dx >> (8 * (b & 3))) & 0xffu) ? 1 : 0)] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < 16; ++b) acc += v[b];
      }
      if (on) Lr[a.S + u] = acc;
    }
    if (lb && on) a.lmask[r.x] = lm;
  }
}

// Snapshot draws for the thread-per-point exact rows (k_exact_rows_lanes / _lv), which build
// rows only: per listed point its n8:95-102 draw in the launch's state (the counts and slots
// every row was built against) from its row, as k_exact_rows_mass's mass_decide does with
// decide_values, on the point's own lane (fp_draw: the resolver's exact draw), with the
// radius under which it holds.  A pick inside a group of equal values is left to the resolver
// (spec -1).  The device-wide resolver starts its rounds from these outcomes and keeps every
// draw whose radius the count drift stays within.
template <int EM>
__global__ __launch_bounds__(256) void k_snap_draws(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  __shared__ uint64_t etab[256];
  __shared__ int s_sl[kWave];
  __shared__ double s_l0[kWave], s_l1[kWave];
  const int K = a.K, m = a.m, E = K + m, ncol = a.S + m;
  for (int e = threadIdx.x; e < 256; e += blockDim.x) etab[e] = devtab::kGlibcExpTab[e];
  if (threadIdx.x < K) {
    const int sl = a.slot_of_label[threadIdx.x], c = a.counts[sl];
    s_sl[threadIdx.x] = sl;
    s_l1[threadIdx.x] = a.logn[c];
    s_l0[threadIdx.x] = c > 0 ? a.logn[c - 1] : -INFINITY;
  }
  __syncthreads();
  const int total = *a.dense_total;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < total; q += gridDim.x * blockDim.x) {
    const int4 r = a.rq[q];
    const int own = r.z;
    const double* row = a.L + (int64_t)r.x * ncol;
    const int own_cnt = a.counts[own];
    const bool single = own_cnt == 1;
    double v[EM];
    double vo = -INFINITY, mo = -INFINITY;
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      if (e < K) {
        const int s = s_sl[e];
        v[e] = (s == own ? s_l0[e] : s_l1[e]) + row[s];                     // n8:40-92
        if (s == own) vo = v[e];
        else mo = fmax(mo, v[e]);
      } else if (e < E) {
        const int l = e - K;
        v[e] = a.logfac + ((l == 0 && single) ? row[own] : row[a.S + l]);     // n8:65-75
        mo = fmax(mo, v[e]);
      } else {
        v[e] = -INFINITY;
      }
    }
    // the prepass's tests (prepass_finish: the own cluster ahead of every other entry by
    // thresh, or by a margin the draw's uniform certifies), here on exact values: what a
    // launch with the prepass would have listed
    const double mg = vo - mo;
    const bool unc = !(own_cnt >= 2 && (mg > a.thresh_ref || stay_by_uniform(mg - a.dmax2_ref, (uint32_t)r.w, E)));
    const unsigned long long ub = __ballot(unc);
    if ((threadIdx.x & 63) == 0 && ub && a.wide_ctr) atomicAdd(a.wide_ctr + 2, __popcll(ub));
    if (a.lmask) {
      const unsigned int lmv = a.lmask[r.x];
      if (lmv) latent_fix<EM>(a.codes_t, a.nq, a.d, a.pool, a.raw, a.P, a.logfac, v, K, E, lmv, single, r.y, m, a.lat_negl);
    }
    double rad = 0.0;
    const int pick = fp_draw<EM, true>(v, E, raw_to_unif((uint32_t)r.w), etab, &rad);
    a.spec[q] = pick >= 0 ? pick : -1;
    // (capped: a kept draw's latents stay kLatNegligible below the clusters, kernels.hip kLatMargin)
    a.spec_rad[q] = pick >= 0 ? fmin(rad, kSpecRadCap) : 0.0;
  }
}

static int lanes_grid(size_t lds) {
  const int cus = device_cus();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_exact_rows_lanes, 256, lds) != hipSuccess || per <= 0) per = 1;
  return cus * per;
}

static int lv_grid(size_t lds) {
  const int cus = device_cus();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_exact_rows_lv, kLvThreads, lds) != hipSuccess || per <= 0)
    per = 1;
  return cus * per;
}

static int mass_grid(size_t lds) {
  const int cus = device_cus();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_exact_rows_mass, kWave * kMassWaves, lds) != hipSuccess ||
      per <= 0)
    per = 1;
  // two per CU when their LDS fits the CU's 160 KB (points are claimed from a counter, so a
  // workgroup that does not become resident only finds the list done)
  const size_t tot = lds + sizeof(double) * kMassWaves * kWave + sizeof(int) * kMassWaves * (kWave + 1);
  if (per < 2 && 2 * tot <= 160 * 1024) per = 2;
  return cus * per;
}

static hipError_t launch_snap_draws(const PrepassArgs& a, hipStream_t s) {
  if (a.spec) {
    const dim3 g((unsigned)(device_cus() * 4)), b(256);
    const int E = a.K + a.m;
    if (E <= 24) HDPM_LAUNCH(k_snap_draws<24>, g, b, 0, s, a);
    else if (E <= 32) HDPM_LAUNCH(k_snap_draws<32>, g, b, 0, s, a);
    else HDPM_LAUNCH(k_snap_draws<64>, g, b, 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_exact_rows(const PrepassArgs& a0, int nblocks, hipStream_t s, int* path) {
  if (path) *path = 0;
  PrepassArgs a = a0;
  // latent bounds only from the level-table kernel (below); every other kernel writes exact
  // columns, and the snapshot draws then read no flags
  if (!a.lbound || !a.pool_head || a.m > 32) a.lbound = 0;
  PrepassArgs an = a;
  an.lmask = nullptr;
  an.lbound = 0;
  if (!a.lbound) a.lmask = nullptr;
  a.lblock = prepass_list_block(a);
  a.nlb = (a.n - a.p0 + a.lblock - 1) / a.lblock;
  const int E = a.K + a.m;
  const size_t lds = exact_wg_lds_bytes(E, a.d, a.nq * 16);
  // the workgroup kernels scan the list themselves unless it is long (exact_scan); the
  // one-wave kernel needs k_list_scan
  const bool wg = !a.exact_wave && lds <= kExactWgLdsMax && E <= 4 * kWave;
  if (a.dense_direct) {
    // every point of [p0, n) listed, in order (k_dense_list wrote the list and the records)
  } else if (a.exact_scan && a.boff) {
    HDPM_LAUNCH(k_list_offsets, dim3(1), dim3(kScanThreads), 0, s, a.cnt, a.nlb, a.boff, a.dense_total);
    const size_t mlds0 = exact_mass_lds_bytes(a.K, a.m, a.d, a.nq * 16);
    const bool mass = !a.exact_wave && ((E <= kWave && mlds0 <= 96 * 1024) || !a.spec || a.spec_lv);
    HDPM_LAUNCH(k_list_fill, dim3((unsigned)((a.nlb + 3) / 4)), dim3(256), 0, s, a, mass ? 1 : 0);
  } else if (a.exact_scan || !wg) {
    HDPM_LAUNCH(k_list_scan, dim3(1), dim3(kScanThreads), 0, s, a.cnt, a.nlb, a.lblock, a.dense,
                       a.dense_total);
  }
  if (!wg) a.exact_scan = 1;
  // grid: from the previous launch's list size (a converged chain lists ~13 points per C5
  // sweep; a random start ~1M, looped over by every resident workgroup)
  const dim3 g(a.exact_grid > 0 ? a.exact_grid : std::min(nblocks * 4, 1024)), b(kExactWgThreads);
  const size_t mlds = exact_mass_lds_bytes(a.K, a.m, a.d, a.nq * 16);
  const size_t llds = (size_t)a.K * (2 * a.d * 8 + a.nq * 16);
  // HDPM_EXACT_MASS=1: the wave-per-point kernel for these sweeps too (A/B)
  static const bool force_mass = [] {
    const char* e = std::getenv("HDPM_EXACT_MASS");
    return e && std::atoi(e) == 1;
  }();
  // HDPM_EXACT_LANES=1: the thread-per-point kernel with compare / select (A/B of the level tables)
  static const bool force_lanes = [] {
    const char* e = std::getenv("HDPM_EXACT_LANES");
    return e && std::atoi(e) == 1;
  }();
  const size_t vlds = exact_lv_lds_bytes(a.K, a.nq, a.mmax);
  const bool want_mass = force_mass || a.exact_pref == 1, want_lanes = force_lanes || a.exact_pref == 2;
  // (with snapshot draws when spec is set: k_snap_draws behind the rows)
  if (a.exact_scan && (!a.spec || a.spec_lv) && !a.exact_wave && a.nq <= kLanesMaxNq && a.K <= kWave && a.mmax >= 1 &&
      vlds <= 120 * 1024 && !want_mass && !want_lanes) {
    HDPM_LAUNCH(k_exact_rows_lv, dim3(lv_grid(vlds)), dim3(kLvThreads), vlds, s, a);
    if (path) *path = 3;
    return launch_snap_draws(a, s);
  }
  if (a.exact_scan && (!a.spec || want_lanes) && !a.exact_wave && a.nq <= kLanesMaxNq && a.K <= kWave &&
      llds <= 64 * 1024 && !want_mass) {
    HDPM_LAUNCH(k_exact_rows_lanes, dim3(lanes_grid(llds)), dim3(256), llds, s, a);
    if (path) *path = 2;
    return launch_snap_draws(an, s);
  }
  if (a.exact_scan && !a.exact_wave && E <= kWave && mlds <= 96 * 1024) {
    static const int mstatic = [] {
      const char* e = std::getenv("HDPM_MASS_STATIC");
      return e ? std::atoi(e) : 0;
    }();
    HDPM_LAUNCH(k_exact_rows_mass, dim3(mass_grid(mlds)), dim3(kWave * kMassWaves), mlds, s, a, mstatic);
    if (path) *path = 1;
    return hipGetLastError();
  }
  if (wg && E <= kWave) HDPM_LAUNCH(k_exact_rows_wg<1>, g, b, lds, s, a);
  else if (wg && E <= 4 * kWave) HDPM_LAUNCH(k_exact_rows_wg<4>, g, b, lds, s, a);
  else HDPM_LAUNCH(k_exact_rows, dim3(std::min(nblocks, 1024)), dim3(kWave * kExactWaves), 0, s, a);
  return hipGetLastError();
}

// A dense launch (every point of [p0, n) listed, engine launch_round): the list and the
// resolver's records straight from the labels and draws, instead of the prepass's bounds and
// the list scan -- row q is point p0 + q.
__global__ __launch_bounds__(256) void k_dense_list(PrepassArgs a) {
  if (!pipe_gate(a)) return;
  const int cnt = a.n - a.p0, m1 = a.m + 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.dense_total = cnt;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < cnt; q += gridDim.x * blockDim.x) {
    const int i = a.p0 + q;
    a.dense[q] = q;
    a.rowpos[i] = q;
    a.rq[q] = make_int4(q, i, a.c[i], (int)a.raw[(int64_t)i * m1 + m1 - 1]);
  }
}
hipError_t launch_dense_list(const PrepassArgs& a, hipStream_t s) {
  const int cnt = a.n - a.p0;
  HDPM_LAUNCH(k_dense_list, dim3((unsigned)std::min(4 * device_cus(), std::max(1, (cnt + 255) / 256))), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

hipError_t launch_cluster_summary(const PrepassArgs& a, hipStream_t s) {
  if (a.K > 0) {
    const int work = a.K * (a.bw + 2);
    HDPM_LAUNCH(k_cluster_summary, dim3(std::min(64, (work + 255) / 256)), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_prepass(const PrepassArgs& a, int nblocks, hipStream_t s) {
  switch (a.wb) {
    case 1: return launch_prepass_w<1>(a, nblocks, s);
    case 2: return launch_prepass_w<2>(a, nblocks, s);
    case 4: return launch_prepass_w<4>(a, nblocks, s);
    case 8: return launch_prepass_w<8>(a, nblocks, s);
    default: return hipErrorInvalidValue;
  }
}

size_t resolve_smem_bytes(int lcap, int m, int blocks) {
  // LIST mode's row tile is sized for the widest row it stages
  return resolve_lds_bytes(lcap, m, blocks, blocks ? 0 : kTileCols);
}

size_t resolve_fpg_smem_bytes(int lcap, int m) { return resolve_fpg_lds_bytes(lcap, m); }

// workgroups of k_resolve_fpg that are resident together on this device (0: none)
int resolve_fpg_max_grid(int lcap, int m) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  const size_t lds = resolve_fpg_lds_bytes(lcap, m);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_resolve_fpg<32>),
                                                   kFpThreads, lds) != hipSuccess)
    return 0;
  int per64 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per64, reinterpret_cast<const void*>(&k_resolve_fpg<64>),
                                                   kFpThreads, lds) != hipSuccess)
    return 0;
  return cus * std::min(per, per64) >= cus ? cus : 0;   // one per CU
}

// The occupancy queries of the kernels a chain reaches only later (an unconverged start:
// device-wide resolver, thread-per-point / mass exact rows) made once at the first sweep: the
// first query inside a sweep cost ~8 ms.  Returns the resolver's grid for lcap.
int warm_sweep_kernels(int lcap, int m) {
  (void)lanes_grid(0);
  (void)lv_grid(0);
  (void)mass_grid(0);
  return resolve_fpg_max_grid(lcap, m);
}

// One gated-off launch (a grid of one workgroup that returns at its gate) of every kernel a
// chain may reach only later -- the exact-rows, list, snapshot-draw and resolver variants of
// the unconverged regime -- at a context's first launch: the first launch of a kernel costs
// ~2 ms (its code object loaded), ~8 ms in the first unconverged sweep of a timed window.
// The argument blocks are the launch's own (every pointer valid); only the gate is replaced by
// `zero` (a device word that is 0; pipe_gate returns before any other access).  `scratch` is
// 16 zeroed device ints: k_list_offsets (no gate) over zero blocks writes scratch[1], and
// k_apply_moves_lds reads a zeroed control block at scratch + 4 (an unfinished sweep: it
// returns).
hipError_t warm_launch_kernels(const PrepassArgs& pa0, const ResolveArgs& ra0, const int* zero, int* scratch,
                               hipStream_t s) {
  // (raw_ptr too: a valid word, never read behind a closed gate -- pipe_gate)
  const uint32_t* const* zero_ptr = reinterpret_cast<const uint32_t* const*>(scratch + 8);
  PrepassArgs pa = pa0;
  pa.gate = zero;
  pa.raw_ptr = zero_ptr;
  ResolveArgs ra = ra0;
  ra.gate = zero;
  ra.raw_ptr = zero_ptr;
  const dim3 one(1);
  // HDPM_WARM_SYNC=1 (diagnosis): synchronise after every launch and name it on stderr
  static const bool wsync = [] {
    const char* e = std::getenv("HDPM_WARM_SYNC");
    return e && std::atoi(e) == 1;
  }();
  static const int wmask = [] {
    const char* e = std::getenv("HDPM_WARM_MASK");
    return e ? (int)std::strtol(e, nullptr, 0) : -1;
  }();
  int k = 0;
  auto step = [&](const char* name) -> hipError_t {
    hipError_t e = hipGetLastError();
    if (wsync) {
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      std::fprintf(stderr, "[warm] %2d %s: %s\n", k, name, hipGetErrorString(e));
    }
    ++k;
    return e;
  };
  auto on = [&]() { return (wmask >> k) & 1; };
  hipError_t e = hipSuccess;
#define HDPM_WARM(name, ...)                                 \
  if (e == hipSuccess) {                                     \
    if (on()) {                                              \
      hipLaunchKernelGGL(__VA_ARGS__);                       \
      e = step(name);                                        \
    } else {                                                 \
      ++k;                                                   \
    }                                                        \
  }
  HDPM_WARM("k_dense_list", k_dense_list, one, dim3(256), 0, s, pa)
  HDPM_WARM("k_list_fill", k_list_fill, one, dim3(256), 0, s, pa, 1)
  HDPM_WARM("k_list_offsets", k_list_offsets, one, dim3(kScanThreads), 0, s, (const int*)scratch, 0, scratch, scratch + 1)
  HDPM_WARM("k_exact_rows_lv", k_exact_rows_lv, one, dim3(kLvThreads), 0, s, pa)
  HDPM_WARM("k_exact_rows_lanes", k_exact_rows_lanes, one, dim3(256), 0, s, pa)
  HDPM_WARM("k_exact_rows_mass", k_exact_rows_mass, one, dim3(kWave * kMassWaves), 0, s, pa, 0)
  HDPM_WARM("k_apply_moves_lds", k_apply_moves_lds, one, dim3(256), 0, s, (const int*)scratch, (const int*)scratch,
            pa.codes_t, pa.d, pa.nq, pa.mmax, (unsigned int*)nullptr, (const ResolveCtl*)(scratch + 4), pa.n, 2)
  HDPM_WARM("k_snap_draws<24>", k_snap_draws<24>, one, dim3(256), 0, s, pa)
  HDPM_WARM("k_snap_draws<32>", k_snap_draws<32>, one, dim3(256), 0, s, pa)
  HDPM_WARM("k_snap_draws<64>", k_snap_draws<64>, one, dim3(256), 0, s, pa)
  HDPM_WARM("k_resolve_fp<24>", k_resolve_fp<24>, one, dim3(kFpThreads), 0, s, ra)
  HDPM_WARM("k_resolve_fp<32>", k_resolve_fp<32>, one, dim3(kFpThreads), 0, s, ra)
  HDPM_WARM("k_resolve_fp<64>", k_resolve_fp<64>, one, dim3(kFpThreads), 0, s, ra)
  HDPM_WARM("k_resolve_fpg<24>", k_resolve_fpg<24>, one, dim3(kFpThreads), 0, s, ra)
  HDPM_WARM("k_resolve_fpg<32>", k_resolve_fpg<32>, one, dim3(kFpThreads), 0, s, ra)
  HDPM_WARM("k_resolve_fpg<64>", k_resolve_fpg<64>, one, dim3(kFpThreads), 0, s, ra)
#undef HDPM_WARM
  return e;
}

hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s) {
  if (a.fp && a.fpg > 1) {
    const size_t lds = resolve_fpg_lds_bytes(a.lcap, a.m);
    if (a.K + a.m <= 24) HDPM_LAUNCH(k_resolve_fpg<24>, dim3(a.fpg), dim3(kFpThreads), lds, s, a);
    else if (a.K + a.m <= 32) HDPM_LAUNCH(k_resolve_fpg<32>, dim3(a.fpg), dim3(kFpThreads), lds, s, a);
    else HDPM_LAUNCH(k_resolve_fpg<64>, dim3(a.fpg), dim3(kFpThreads), lds, s, a);
  } else if (a.fp) {
    const size_t lds = resolve_fp_lds_bytes(a.lcap, a.m);
    if (a.K + a.m <= 24) HDPM_LAUNCH(k_resolve_fp<24>, dim3(1), dim3(kFpThreads), lds, s, a);
    else if (a.K + a.m <= 32) HDPM_LAUNCH(k_resolve_fp<32>, dim3(1), dim3(kFpThreads), lds, s, a);
    else HDPM_LAUNCH(k_resolve_fp<64>, dim3(1), dim3(kFpThreads), lds, s, a);
  } else if (a.blocks)
    HDPM_LAUNCH(k_resolve_blk, dim3(1), dim3(kWave), resolve_lds_bytes(a.lcap, a.m, 1), s, a);
  else
    HDPM_LAUNCH(k_resolve, dim3(1), dim3(kWave), resolve_lds_bytes(a.lcap, a.m, 0, a.S + a.m), s, a);
  return hipGetLastError();
}

hipError_t launch_relabel(int* c, const int* los, int n, const ResolveCtl* ctl, hipStream_t s) {
  HDPM_LAUNCH(k_relabel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, c, los, n, ctl);
  return hipGetLastError();
}

hipError_t launch_apply_moves(const int* mlog, const int* mcount, int grid, const uint8_t* codes_t, int d, int nq,
                              int mmax, unsigned int* freq, const ResolveCtl* ctl, int n, int nslots, hipStream_t s) {
  // LDS deltas for the slots that fit 64 KB (C5: 32 of them; the sweep's slots are < nslots)
  const int ls = std::min(nslots, (int)(64 * 1024 / ((size_t)d * mmax * 4)));
  if (ls >= 2) {
    HDPM_LAUNCH(k_apply_moves_lds, dim3(512), dim3(256), (size_t)ls * d * mmax * 4, s, mlog, mcount, codes_t, d,
                       nq, mmax, freq, ctl, n, ls);
    return hipGetLastError();
  }
  HDPM_LAUNCH(k_apply_moves, dim3(std::max(1, std::min(grid, 4096))), dim3(kWave), 0, s, mlog, mcount, codes_t,
                     d, nq, mmax, freq, ctl, n);
  return hipGetLastError();
}

hipError_t launch_freq_gather(const unsigned int* freq, const int* sol, int Kmax, int fs, unsigned int* out,
                              const ResolveCtl* ctl, int n, hipStream_t s) {
  const int64_t work = (int64_t)std::max(Kmax, 1) * fs;
  HDPM_LAUNCH(k_freq_gather, dim3((unsigned)std::min<int64_t>(1024, (work + 255) / 256)), dim3(256), 0, s, freq,
                     sol, fs, out, ctl, n);
  return hipGetLastError();
}

hipError_t launch_finish_sweep(int* counts, int* sol, int* los, int* src, int cap, const ResolveCtl* ctl, int n,
                               hipStream_t s) {
  HDPM_LAUNCH(k_finish_sweep, dim3(1), dim3(1024), (size_t)(2 * cap) * 4, s, counts, sol, los, src, ctl, n);
  return hipGetLastError();
}

// One thread: waits for the host's decision on the enqueued sweep (PipeSlot), at most
// `limit` ticks of the 100 MHz constant clock (every wave exits), then the gate of its
// kernels: go, and the previous sweep's control block (written by its resolver before this
// kernel in stream order) shows it complete without a move.
__global__ void k_pipe_wait(PipeSlot* slot, const ResolveCtl* prev, ResolveCtl* own, int n, PipeGate* g,
                            long long limit, PipeAuto au) {
  if (threadIdx.x != 0) return;
  if (au.on) {
    // the device's own go (PipeAuto): the update's chain word, the previous sweep's control block
    const volatile ResolveCtl* c = prev;
    const int cok = __hip_atomic_load(&au.chain->ok, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t end =
        (int64_t)__hip_atomic_load(reinterpret_cast<const uint64_t*>(&au.chain->end), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t r = end - au.win_start;
    const bool ok = cok == 1 && c->status == 0 && c->next >= n && c->moves == 0 && r >= 0 && r + au.sweep_len <= au.win_count;
    if (ok) {
      const uint32_t* raw = au.win_raw + r;
      g->raw = raw;
      g->status = 4;
      g->gate = 1;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(&slot->raw_dev), reinterpret_cast<uint64_t>(raw), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&slot->dev, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __hip_atomic_store(&slot->dev, 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const long long t0 = wall_clock64();
  int f = 0;
  // (relaxed polls of host memory, one acquire fence after: an acquire load invalidates the
  // XCD's L2 on every poll, under the kernels beside this one)
  for (;;) {
    f = __hip_atomic_load(&slot->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (f != 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      break;
    }
    if (wall_clock64() - t0 > limit) {
      f = 3;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  const volatile ResolveCtl* c = prev;
  const bool ok = f == 1 && c->status == 0 && c->next >= n && c->moves == 0;
  const uint64_t rw =
      __hip_atomic_load(reinterpret_cast<const uint64_t*>(&slot->raw), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  g->raw = ok ? reinterpret_cast<const uint32_t*>(rw) : nullptr;
  g->status = f;
  g->gate = ok ? 1 : 0;
  if (!ok) {              // the sweep's control block says it did not run
    volatile ResolveCtl* o = own;
    o->status = kPipeOff;
    o->next = 0;
    o->aborted = 0;
    o->uncertain = -1;
  }
}
hipError_t launch_pipe_wait(PipeSlot* slot, const ResolveCtl* prev, ResolveCtl* own, int n, PipeGate* g,
                            long long limit, hipStream_t s, const PipeAuto& au) {
  HDPM_LAUNCH(k_pipe_wait, dim3(1), dim3(64), 0, s, slot, prev, own, n, g, limit, au);
  return hipGetLastError();
}

hipError_t launch_scatter_clusters(const uint8_t* stage, int nent, int dp, int d, int bw, int full, uint8_t* codes,
                                   double* tab, uint64_t* bnd, int* counts, int* sol, int* los, int* src,
                                   hipStream_t s, const int* gate, uint64_t* csum, const double* logn, int* zero,
                                   int* wide_ctr) {
  if (csum && !full) return hipErrorInvalidValue;     // the summaries assume entry r = label r = slot r
  const int64_t work = (int64_t)nent * std::max(2 * d, std::max(dp, bw + 2));
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (work + 255) / 256));
  const ScatterSummary sum{csum, logn, zero, wide_ctr};
  HDPM_LAUNCH(k_scatter_clusters, dim3(nb), dim3(256), 0, s, stage, nent, dp, d, bw, full, codes, tab, bnd,
                     counts, sol, los, src, gate, sum);
  return hipGetLastError();
}

size_t hist_partial_words(const HistArgs& a, int* nbx_out, int* kc_out, int* tpb_out) {
  const int64_t per_label = (int64_t)a.mmax * a.d * 4;
  const int64_t budget = 96 * 1024 - (int64_t)(kHistBlock / kWave) * a.W * 64 * 8 - per_label;  // - trash row
  const int kc = budget > 0 ? (int)std::min<int64_t>(a.K, budget / per_label) : 0;
  const int64_t ntiles = ((int64_t)a.n + 63) / 64;
  const int tpb = (int)std::max<int64_t>(16, (ntiles + 255) / 256);
  const int nbx = (int)((ntiles + tpb - 1) / tpb);
  *nbx_out = nbx;
  *kc_out = kc;
  *tpb_out = tpb;
  if (kc <= 0 || a.W > 8) return 0;
  const int ny = (a.K + kc - 1) / kc;
  return (size_t)ny * nbx * kc * a.mmax * a.d;
}

hipError_t launch_hist(const HistArgs& a0, hipStream_t s) {
  HistArgs a = a0;
  int nbx, kc, tpb;
  const size_t pw = hist_partial_words(a, &nbx, &kc, &tpb);
  const hipError_t e = hipMemsetAsync(a.freq, 0, (size_t)a.K * a.d * a.mmax * 4, s);
  if (e != hipSuccess) return e;
  if (pw > 0 && a.partial && a.xpk) {
    a.KC = kc;
    a.tiles_per_block = tpb;
    const int ny = (a.K + kc - 1) / kc;
    const size_t hbytes = (((size_t)(kc + 1) * a.mmax * a.d * 4 + 15) / 16) * 16;
    const size_t lds = hbytes + (size_t)(kHistBlock / kWave) * a.W * 64 * 8;
    HDPM_LAUNCH(k_hist_packed, dim3(nbx, ny), dim3(kHistBlock), lds, s, a);
    const int hsize = kc * a.mmax * a.d;
    HDPM_LAUNCH(k_hist_reduce, dim3((hsize + 255) / 256, ny, kHistReduceSplit), dim3(256), 0, s, a, nbx);
  } else {
    const int64_t nt = (int64_t)a.n * a.nq;
    HDPM_LAUNCH(k_hist_global, dim3((nt + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_loglik(const LoglikArgs& a, hipStream_t s) {
  HDPM_LAUNCH(k_loglik, dim3((a.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_lmatrix(const uint8_t* codes_t, int n, int d, int nq, ParamTables cl, int K, double* L,
                          int* H, int64_t ldL, hipStream_t s) {
  HDPM_LAUNCH(k_lmatrix, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, codes_t, n, d, nq, cl,
                     K, L, H, ldL);
  return hipGetLastError();
}

}  // namespace hdpm

namespace hdpm {

// ------------------------------------------------------------------ split-merge
// A scan of the device chain (SmArgs::link): false when it does not run, else its draws and
// sizes into a.  Read at the kernel's start by every lane and made wave-uniform, so the
// branches on it are scalar.
__device__ __forceinline__ bool sm_link_in(SmArgs& a) {
  if (!a.link) return true;
  if (__builtin_amdgcn_readfirstlane(a.link->ok) == 0) return false;
  const uint64_t r = (uint64_t)a.link->raw;
  a.raw = (const uint32_t*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r));
  a.n1 = __builtin_amdgcn_readfirstlane(a.link->n1);
  a.n2 = __builtin_amdgcn_readfirstlane(a.link->n2);
  return true;
}

__global__ __launch_bounds__(kBlock) void k_sm_ll(SmArgs a) {
  if (!sm_link_in(a)) return;
  const int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= a.nS) return;
  const int64_t i = a.S[q];
  const int dp = a.nq * 16;
  PointCodes<0> x;
  x.load(a.codes_t, i, a.nq);
  a.ll[q] = ll_uniform<0>(x, a.d, a.two.codes, a.two.tab);
  a.ll[a.nS + q] = ll_uniform<0>(x, a.d, a.two.codes + dp, a.two.tab + 2 * a.d);
}

// k_sm_ll with both clusters' tables and codes staged in LDS; one lane per (point, cluster)
// attribute-order sum and 64-lane workgroups, so a scan of ~10^4 points spreads over the CUs.
constexpr int kSmLLBlock = 64;
__device__ __forceinline__ void sm_cert_point(const SmArgs& a, int q, double dl);
__global__ __launch_bounds__(kSmLLBlock) void k_sm_ll_lds(SmArgs a) {
  if (!sm_link_in(a)) return;
  extern __shared__ double sm_lds[];
  const int d = a.d, dp = a.nq * 16;
  double* tab = sm_lds;                                    // [2][d][2]
  uint8_t* cc = (uint8_t*)(sm_lds + 4 * d);                // [2][dp]
  {
    // staged with 8 loads in flight per lane (a load-store loop paid an L2 latency per
    // 8 bytes: 49 of them per lane at C4, most of the kernel's 36 us)
    const int nt = 2 * d, nc = 2 * dp / 16;           // uint4s of the tables, of the codes
    const uint4* st = (const uint4*)a.two.tab;
    const uint4* sc = (const uint4*)a.two.codes;
    for (int t0 = 0; t0 < nt + nc; t0 += 8 * kSmLLBlock) {
      uint4 r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = t0 + k * kSmLLBlock + (int)threadIdx.x;
        r[k] = t < nt ? st[t] : (t < nt + nc ? sc[t - nt] : make_uint4(0, 0, 0, 0));
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = t0 + k * kSmLLBlock + (int)threadIdx.x;
        if (t < nt) ((uint4*)tab)[t] = r[k];
        else if (t < nt + nc) ((uint4*)cc)[t - nt] = r[k];
      }
    }
  }
  __syncthreads();
  if (a.zero)
    for (int e = blockIdx.x * kSmLLBlock + (int)threadIdx.x; e < a.zero_n; e += gridDim.x * kSmLLBlock) a.zero[e] = 0u;
  // lane pair (2p, 2p + 1): point p of the block against cluster 0 and cluster 1, so a scan
  // of |S| points runs 2|S| lanes (the chains are sequential; more waves per SIMD is what
  // hides their issue and LDS latency)
  const int cl = threadIdx.x & 1;
  const int q = blockIdx.x * (kSmLLBlock / 2) + (threadIdx.x >> 1);
  if (q >= a.nS) return;
  const int64_t i = a.S[q];
  const double* t = tab + 2 * d * cl;
  const uint4* cz = (const uint4*)(cc + dp * cl);
  double l = 0.0;
  const int nfull = d / 16;
  // the point's 16-byte code chunks lie 1 KB apart (tiled rows): kAhead loads in flight per
  // lane (one at a time left every chunk a memory latency: 38 us per C4 scan)
  constexpr int kAhead = 8;
  const uint8_t* xp = a.codes_t + tiled_offset(i, 0, a.nq);
  uint4 buf[kAhead];
#pragma unroll
  for (int k = 0; k < kAhead; ++k) buf[k] = k < a.nq ? *(const uint4*)(xp + (size_t)k * 1024) : make_uint4(0, 0, 0, 0);
  for (int q0 = 0; q0 < a.nq; q0 += kAhead) {
#pragma unroll
    for (int k = 0; k < kAhead; ++k) {
      const int qq = q0 + k;
      if (qq >= a.nq) break;
      const uint4 xq = buf[k];
      if (qq + kAhead < a.nq) buf[k] = *(const uint4*)(xp + (size_t)(qq + kAhead) * 1024);
      const uint4 c = cz[qq];
      const uint4 dx = make_uint4(xq.x ^ c.x, xq.y ^ c.y, xq.z ^ c.z, xq.w ^ c.w);
      if (qq < nfull) {
        // all 16 terms read before their ordered adds (LDS reads in flight)
        double v[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) v[b] = t[2 * (qq * 16 + b) + (byte_differs(dx, b) ? 1 : 0)];
#pragma unroll
        for (int b = 0; b < 16; ++b) l += v[b];
      } else {
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const int j = qq * 16 + b;
          if (j < d) l += t[2 * j + (byte_differs(dx, b) ? 1 : 0)];
        }
      }
    }
  }
  a.ll[cl * a.nS + q] = l;
  if (a.cert_in_ll) {
    // the pair's other sum; lane 0 of the pair certifies the point (k_sm_cert's work)
    const double lo = __shfl_xor(l, 1);
    if (cl == 0) sm_cert_point(a, q, l - lo);
  }
}

// Exact sm:204-215 two-way draw.  probs[k] = log(n_k) + H_k; normalise; FixupProb;
// revsort of two entries (ties: second first); cumulative compare.
template <bool kOcml = false>
__device__ __forceinline__ void two_way_probs(double v0, double v1, double& p0, double& p1) {
  const double mx = fmax(v0, v1);
  p0 = dexp<kOcml>(v0 - mx);
  p1 = dexp<kOcml>(v1 - mx);
  double sum = 0.0;
  sum += p0;
  sum += p1;
  p0 = p0 / sum;
  p1 = p1 / sum;
  double s2 = 0.0;
  if (p0 > 0) s2 += p0;
  if (p1 > 0) s2 += p1;
  p0 = p0 / s2;
  p1 = p1 / s2;
}
__device__ __forceinline__ int two_way_pick(double p0, double p1, double rU) {
  // revsort(n = 2): descending, equal -> index 2 first
  const bool first0 = p0 > p1;
  const double a0 = first0 ? p0 : p1;
  return (rU <= a0) ? (first0 ? 0 : 1) : (first0 ? 1 : 0);
}
template <bool kOcml = false>
__device__ __forceinline__ int two_way_draw(double v0, double v1, double rU) {
  double p0, p1;
  two_way_probs<kOcml>(v0, v1, p0, p1);
  return two_way_pick(p0, p1, rU);
}

// One wave walks S in batches of 64 in order.  Within a batch the size n1 of c1 seen by
// lane p lies in [n1 - p, n1 + p] (n1 + n2 is fixed: points only change sides).  The draw's
// p0 is a function of D = v0 - v1 alone (one of the two exps is exp(0)), D is monotone in
// n1 (logn is increasing, rounding is monotone), and in exact arithmetic the pick is
// "0 iff (D > 0 and D >= lam) or (D <= 0 and D > -lam)" with lam = log(rU / (1 - rU)): it
// only changes where D crosses 0 (the revsort order), lam or -lam.  A lane whose D range
// stays 1e-4 away from all three (there p0 is >= 2e-15 from its threshold, far beyond the
// few-ulp rounding of the exp and divisions) has one pick for every count it can see and is
// settled in parallel without evaluating the draw; the others are drawn with their exact
// counts, all at once, by the fixed-point iteration below.
//
// The margin.  Near a threshold D0 (0, lam or -lam) the computed p0 = 1 / (1 + exp(-D)) (or
// its complement) moves by |p0'| |D - D0| >= p (1 - p) |D - D0|, and p (1 - p) >= 2e-11 for the
// thresholds a uniform in (2.3e-10, 1 - 2.3e-10) can set, so a D range kept 1e-4 from the
// threshold keeps p0 at least ~2e-15 away from the value that would flip the pick.  The
// computed D carries the error of two logn entries and two log-likelihood sums (a few ulp of
// their magnitudes, < 1e-9 for any |S| and D the engine accepts), and exp / the two
// divisions add a few ulp of p0 (< 1e-15): both far inside the margin.
constexpr double kSmScanMargin = 1e-4;

// Certified count bands of every point of S, in parallel before the walk.  For point q with
// current side s (s0 = [s == 0], s1 = [s == 1]) the scan's D at size n1 of c1 is
//   D(n1) = (log(n1 - s0) + l0) - (log(tot - n1 - s1) + l1) = log(a / (L - a)) + l0 - l1
// (a = n1 - s0, L = tot - s0 - s1) up to rounding (< 1e-9), increasing in n1.  For each
// threshold D_t in {0, lam, -lam} the real n1 where D crosses D_t -/+ margin is
// s0 + L sigmoid(D_t -/+ margin - (l0 - l1)); every integer n1 below the band
// [floor(x-) - 1, ceil(x+) + 1] has D < D_t - margin + 1e-9, every one above it D > D_t +
// margin - 1e-9.  The walk then certifies a lane by integer compares against 3 bands.
__device__ __forceinline__ void sm_cert_point(const SmArgs& a, int q, double dl) {
  const int cur = a.side[q];
  if (a.side_prev) a.side_prev[q] = cur;
  const double rU = raw_to_unif(a.raw[q]);
  const int tot = a.n1 + a.n2;
  const int s0 = cur == 0, s1 = cur == 1;
  const double L = (double)(tot - s0 - s1);
  const double lam = log(rU / (1.0 - rU));
  const double th[3] = {0.0, lam, -lam};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const double zm = (th[t] - kSmScanMargin) - dl, zp = (th[t] + kSmScanMargin) - dl;
    const double xm = (double)s0 + L / (1.0 + exp(-zm)), xp = (double)s0 + L / (1.0 + exp(-zp));
    a.cert[(2 * t) * a.nS + q] = (int)floor(xm) - 1;
    a.cert[(2 * t + 1) * a.nS + q] = (int)ceil(xp) + 1;
  }
}
__global__ __launch_bounds__(kBlock) void k_sm_cert(SmArgs a) {
  if (!sm_link_in(a)) return;
  const int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= a.nS) return;
  sm_cert_point(a, q, a.ll[q] - a.ll[a.nS + q]);
}

// The walk: wave 0 goes through S in batches of 64 in order; waves 1..15 stage the next chunk
// of S's inputs (sides, certified bands, log-likelihoods, raw draws) into an LDS double
// buffer meanwhile.  Within a batch the size n1 of c1 seen by lane p lies in [n1 - p,
// n1 + p] (n1 + n2 is fixed: points only change sides); in exact arithmetic the pick is
// "0 iff (D > 0 and D >= lam) or (D <= 0 and D > -lam)" with lam = log(rU / (1 - rU)), so it
// only changes where D crosses 0 (the revsort order), lam or -lam.  A lane whose count range
// misses all three bands keeps D 1e-4 away from every threshold (there p0 is >= 2e-15 from
// its threshold, far beyond the few-ulp rounding of the exp and divisions): it has one pick
// for every count it can see and is settled by compares; the others are drawn exactly, all
// at once, by the fixed-point iteration below.
//
// The margin.  Near a threshold D0 (0, lam or -lam) the computed p0 = 1 / (1 + exp(-D)) (or
// its complement) moves by |p0'| |D - D0| >= p (1 - p) |D - D0|, and p (1 - p) >= 2e-11 for the
// thresholds a uniform in (2.3e-10, 1 - 2.3e-10) can set, so a D kept 1e-4 from the
// threshold keeps p0 at least ~2e-15 away from the value that would flip the pick.  The
// computed D carries the error of two logn entries and two log-likelihood sums (a few ulp of
// their magnitudes, < 1e-9 for any |S| and D the engine accepts), and exp / the two
// divisions add a few ulp of p0 (< 1e-15): both far inside the margin.
constexpr int kSmScanThreads = 1024;          // wave 0 walks, 15 waves stage (one load round per chunk)
constexpr int kSmChunk = 1024;              // points per staged chunk
struct SmChunk {
  double l0[kSmChunk], l1[kSmChunk];
  uint32_t raw[kSmChunk];
  int side[kSmChunk];
  int band[6][kSmChunk];
};
__global__ __launch_bounds__(kSmScanThreads) void k_sm_scan(SmArgs a) {
  extern __shared__ unsigned char sm_scan_lds[];
  SmChunk* buf = (SmChunk*)sm_scan_lds;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (!sm_link_in(a)) return;
  if (a.wide_buf) {
    // behind k_sm_scan_wide: nothing to do when it finished; when it gave up (some of its
    // chunks may have written their sides) the walk starts from the sides before the scan
    if (__hip_atomic_load(a.wide_buf + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    for (int q = tid; q < a.nS; q += kSmScanThreads) a.side[q] = a.side_prev[q];
    __threadfence_block();
    __syncthreads();
  }
  int n1 = a.n1;
  const int tot = a.n1 + a.n2;
  const int nch = (a.nS + kSmChunk - 1) / kSmChunk;
  auto stage = [&](int c, int t0, int nt) {
    SmChunk& B = buf[c & 1];
    const int q0 = c * kSmChunk, nq = min(kSmChunk, a.nS - q0);
    for (int e = t0; e < nq; e += nt) {
      B.l0[e] = a.ll[q0 + e];
      B.l1[e] = a.ll[a.nS + q0 + e];
      B.raw[e] = a.raw[q0 + e];
      B.side[e] = a.side[q0 + e];
#pragma unroll
      for (int k = 0; k < 6; ++k) B.band[k][e] = a.cert[k * a.nS + q0 + e];
    }
  };
  if (nch > 0) stage(0, tid, kSmScanThreads);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (wv > 0) {
      if (c + 1 < nch) stage(c + 1, tid - kWave, kSmScanThreads - kWave);
    } else {
      const SmChunk& B = buf[c & 1];
      const int q0 = c * kSmChunk, nq = min(kSmChunk, a.nS - q0);
      for (int base = 0; base < nq; base += kWave) {
        const int e = base + lane;
        const bool act = e < nq;
        const int cur = act ? B.side[e] : 0;
        bool certain = false;
        int choice = cur;
        if (act) {
          // n1 as lane `lane` may see it, within the sizes the clusters can take
          const int lo = max(n1 - lane, 1 + (cur == 0)), hi = min(n1 + lane, tot - 1 - (cur == 1));
          bool above[3];
          certain = true;
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int blo = B.band[2 * t][e], bhi = B.band[2 * t + 1][e];
            certain = certain && (hi < blo || lo > bhi);
            above[t] = lo > bhi;
          }
          if (certain) choice = ((above[0] && above[1]) || (!above[0] && above[2])) ? 0 : 1;
        }
        // The uncertain lanes are drawn together by a fixed-point iteration: every lane's
        // count is the batch start plus the moves of the lanes before it (an exclusive prefix
        // sum of the current choices); each uncertain lane draws exactly at that count, and
        // the sweep repeats until no choice changes.  Lane k's count only depends on lanes
        // < k, so after round r the first r uncertain lanes hold their true draws: the fixed
        // point is the reference's sequential walk (reached in <= 64 rounds, usually 1-3).
        // Counts a lane sees before the fixed point are clamped to the sizes the clusters can
        // take.
        const bool unc = act && !certain;
        if (__ballot(unc)) {
          const double l0 = unc ? B.l0[e] : 0.0, l1 = unc ? B.l1[e] : 0.0;
          const double rU = unc ? raw_to_unif(B.raw[e]) : 0.5;
          int gprev = -1;
          const unsigned long long below = (1ull << lane) - 1ull;
          for (;;) {
            // exclusive prefix of the lanes' moves of n1 (+1: to c1, -1: to c2) by ballots
            const unsigned long long up = __ballot(act && choice == 0 && cur == 1);
            const unsigned long long dn = __ballot(act && choice == 1 && cur == 0);
            const int pre = __popcll(up & below) - __popcll(dn & below);
            bool changed = false;
            if (unc) {
              const int g = min(max(n1 + pre, 1 + (cur == 0)), tot - 1 - (cur == 1));
              if (g != gprev) {
                gprev = g;
                const int nz1 = g - (cur == 0), nz2 = tot - g - (cur == 1);
                const int pk = two_way_draw(dlog((double)nz1) + l0, dlog((double)nz2) + l1, rU);
                changed = pk != choice;
                choice = pk;
              }
            }
            if (!__ballot(changed)) break;
          }
        }
        n1 += __popcll(__ballot(act && choice == 0 && cur == 1)) - __popcll(__ballot(act && choice == 1 && cur == 0));
        if (act) a.side[q0 + e] = choice;
      }
    }
    __syncthreads();
  }
  if (tid == 0) { a.out_counts[0] = n1; a.out_counts[1] = tot - n1; }
}

// The restricted scan on many CUs (k_sm_scan_wide).  Workgroup c walks chunk c of S (256
// consecutive points) with wave 0 exactly as k_sm_scan walks its batches (certified compares,
// the fixed-point draws of the uncertain lanes), from the chunk's start count: the committed
// n1 plus the net moves of the chunks before it in the last round.  After each round (one grid
// barrier) every workgroup reads the round's chunk deltas; the scan has converged when they
// equal the previous round's (the start counts, and so every outcome, would repeat).  Chunk
// c's start depends only on chunks < c, so after round r the first r chunks are final: the
// fixed point is the sequential walk, reached in at most G + 1 rounds.  A barrier that waits
// longer than wide_limit (a workgroup not resident) sets wide_buf[1]; nothing is written then
// and the host runs k_sm_scan instead.
constexpr int kSmWideChunk = 256;
constexpr int kSmWideMaxG = 1024;
__global__ __launch_bounds__(kSmWideChunk) void k_sm_scan_wide(SmArgs a) {
  if (!sm_link_in(a)) return;     // (every workgroup alike: no barrier is left waiting)
  __shared__ double s_l0[kSmWideChunk], s_l1[kSmWideChunk];
  __shared__ uint32_t s_raw[kSmWideChunk];
  __shared__ int s_cur[kSmWideChunk], s_choice[kSmWideChunk];
  __shared__ int s_band[6][kSmWideChunk];
  __shared__ int s_prev[kSmWideMaxG];
  __shared__ int s_start, s_state;
  const int c = blockIdx.x, G = gridDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q0 = c * kSmWideChunk, nq = min(kSmWideChunk, a.nS - q0);
  if (tid < nq) {
    s_l0[tid] = a.ll[q0 + tid];
    s_l1[tid] = a.ll[a.nS + q0 + tid];
    s_raw[tid] = a.raw[q0 + tid];
    s_cur[tid] = a.side[q0 + tid];
#pragma unroll
    for (int k = 0; k < 6; ++k) s_band[k][tid] = a.cert[k * a.nS + q0 + tid];
  }
  for (int h = tid; h < G; h += kSmWideChunk) s_prev[h] = 0;
  if (tid == 0) {
    s_start = a.n1;
    s_state = 0;
  }
  __syncthreads();
  const int tot = a.n1 + a.n2;
  int* bar = a.wide_buf;
  int* gave_up = a.wide_buf + 1;
  int* dl = a.wide_buf + 4;
  int r = 0;
  for (; r <= G; ++r) {
    if (wv == 0) {
      int n1 = s_start;
      const int nstart = n1;
      for (int base = 0; base < nq; base += kWave) {
        const int e = base + lane;
        const bool act = e < nq;
        const int cur = act ? s_cur[e] : 0;
        bool certain = false;
        int choice = cur;
        if (act) {
          const int lo = max(n1 - lane, 1 + (cur == 0)), hi = min(n1 + lane, tot - 1 - (cur == 1));
          bool above[3];
          certain = true;
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int blo = s_band[2 * t][e], bhi = s_band[2 * t + 1][e];
            certain = certain && (hi < blo || lo > bhi);
            above[t] = lo > bhi;
          }
          if (certain) choice = ((above[0] && above[1]) || (!above[0] && above[2])) ? 0 : 1;
        }
        const bool unc = act && !certain;
        if (__ballot(unc)) {
          const double l0 = unc ? s_l0[e] : 0.0, l1 = unc ? s_l1[e] : 0.0;
          const double rU = unc ? raw_to_unif(s_raw[e]) : 0.5;
          int gprev = -1;
          const unsigned long long below = (1ull << lane) - 1ull;
          for (;;) {
            const unsigned long long up = __ballot(act && choice == 0 && cur == 1);
            const unsigned long long dn = __ballot(act && choice == 1 && cur == 0);
            const int pre = __popcll(up & below) - __popcll(dn & below);
            bool changed = false;
            if (unc) {
              const int g = min(max(n1 + pre, 1 + (cur == 0)), tot - 1 - (cur == 1));
              if (g != gprev) {
                gprev = g;
                const int nz1 = g - (cur == 0), nz2 = tot - g - (cur == 1);
                const int pk = two_way_draw(dlog((double)nz1) + l0, dlog((double)nz2) + l1, rU);
                changed = pk != choice;
                choice = pk;
              }
            }
            if (!__ballot(changed)) break;
          }
        }
        n1 += __popcll(__ballot(act && choice == 0 && cur == 1)) - __popcll(__ballot(act && choice == 1 && cur == 0));
        if (act) s_choice[e] = choice;
      }
      if (lane == 0) __hip_atomic_store(dl + (r & 1) * G + c, n1 - nstart, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid == 0 && a.wide_limit <= 0) {
      // a zero limit gives up at the first barrier unconditionally (deterministic: the
      // give-up test must not depend on how fast the workgroups arrive)
      __hip_atomic_store(gave_up, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_state = -1;
    } else if (tid == 0) {
      // grid barrier r: arrivals counted, agent-scope release / acquire
      __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const long long t0 = wall_clock64();
      // (relaxed polls, one acquire fence after the barrier: an agent-scope acquire load
      // invalidates the XCD's L2 on every poll)
      for (;;) {
        if (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= G * (r + 1)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          break;
        }
        if (__hip_atomic_load(gave_up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
            wall_clock64() - t0 > a.wide_limit) {
          __hip_atomic_store(gave_up, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_state = -1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (s_state < 0) break;
    // the round's deltas: this chunk's next start, and whether any delta changed
    if (wv == 0) {
      int pre = 0;
      bool diff = false;
      for (int h0 = 0; h0 < G; h0 += kWave) {
        const int h = h0 + lane;
        const int v = h < G ? __hip_atomic_load(dl + (r & 1) * G + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        diff = diff || (h < G && v != s_prev[h]);
        if (h < G) s_prev[h] = v;
        int x = h < c ? v : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        pre += x;
      }
      const bool any = __ballot(diff) != 0ull;
      if (lane == 0) {
        s_start = a.n1 + pre;
        s_state = any ? 0 : 1;
      }
    }
    __syncthreads();
    if (s_state == 1) break;
  }
  if (s_state == 1) {
    for (int e = tid; e < nq; e += kSmWideChunk) a.side[q0 + e] = s_choice[e];
    if (c == 0 && tid == 0) {
      int tot_d = 0;
      for (int h = 0; h < G; ++h) tot_d += s_prev[h];
      a.out_counts[0] = a.n1 + tot_d;
      a.out_counts[1] = tot - (a.n1 + tot_d);
      a.wide_buf[2] = r + 1;
    }
  } else if (tid == 0) {
    __hip_atomic_store(gave_up, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// G workgroups for k_sm_scan_wide, or 0 when the scan is too large for one resident grid.
int sm_scan_wide_grid(int nS) {
  const int G = (nS + kSmWideChunk - 1) / kSmWideChunk;
  return (G >= 2 && G <= kSmWideMaxG && G <= device_cus()) ? G : 0;
}
hipError_t launch_sm_scan_wide(const SmArgs& a, int G, hipStream_t s) {
  {
    const hipError_t e = hipMemsetAsync(a.wide_buf, 0, 16, s);
    if (e != hipSuccess) return e;
  }
  HDPM_LAUNCH(k_sm_scan_wide, dim3(G), dim3(kSmWideChunk), 0, s, a);
  return hipGetLastError();
}

// logprobgs_c_i terms: log(probs[current side]) with fixed launch sizes; compensated
// per-block sums (hi, lo).
__global__ __launch_bounds__(kBlock) void k_sm_lpgs(SmArgs a) {
  const int q = blockIdx.x * kBlock + threadIdx.x;
  double hi = 0.0, lo = 0.0;
  if (q < a.nS) {
    const int g = a.side_ref[q];
    const double v0 = a.logn[a.n1 - (g == 0)] + a.ll[q];
    const double v1 = a.logn[a.n2 - (g == 1)] + a.ll[a.nS + q];
    const double mx = fmax(v0, v1);
    double p0 = dexp(v0 - mx), p1 = dexp(v1 - mx);
    double sum = 0.0;
    sum += p0;
    sum += p1;
    p0 = p0 / sum;
    p1 = p1 / sum;
    hi = dlog(a.side[q] == 0 ? p0 : p1);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double oh = __shfl_xor(hi, o), ol = __shfl_xor(lo, o);
    double s, e;
    two_sum(hi, oh, s, e);
    hi = s;
    lo = lo + ol + e;
  }
  __shared__ double sh[kBlock / kWave][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { sh[wv][0] = hi; sh[wv][1] = lo; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double H = 0.0, Lo = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) {
      double s, e;
      two_sum(H, sh[w][0], s, e);
      H = s;
      Lo += sh[w][1] + e;
    }
    a.out[2 * blockIdx.x] = H;
    a.out[2 * blockIdx.x + 1] = Lo;
  }
}

// k_sm_ll_lds runs (and carries the fused cert / zeroing, which the callers set only then)
bool sm_ll_lds_fits(int d, int nq) { return (size_t)4 * d * 8 + (size_t)2 * nq * 16 <= 64 * 1024; }
hipError_t launch_sm_ll(const SmArgs& a, hipStream_t s) {
  if (a.nS == 0) return hipSuccess;
  const size_t lds = (size_t)4 * a.d * 8 + (size_t)2 * a.nq * 16;
  if (lds <= 64 * 1024) {
    const int per = kSmLLBlock / 2;     // points per workgroup (two lanes each)
    HDPM_LAUNCH(k_sm_ll_lds, dim3((a.nS + per - 1) / per), dim3(kSmLLBlock), lds, s, a);
    return hipGetLastError();
  }
  HDPM_LAUNCH(k_sm_ll, dim3((a.nS + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_sm_scan(const SmArgs& a, hipStream_t s) {
  if (a.nS > 0 && !a.cert_in_ll) HDPM_LAUNCH(k_sm_cert, dim3((a.nS + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
  HDPM_LAUNCH(k_sm_scan, dim3(1), dim3(kSmScanThreads), 2 * sizeof(SmChunk), s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ testing
// One draw from given log-weights and uniform on the device: the n8:95-102 categorical draw
// (decide_values) or the sm:204-215 two-way draw, with the engine's glibc exp or, kOcml,
// the device libm's (the behaviour before the glibc replica; the parity test shows the
// difference).
template <bool kOcml>
__global__ __launch_bounds__(kWave) void k_debug_draw(const double* logw, int E, double rU, int two_way, int* out) {
  __shared__ double lp[4 * kWave];
  __shared__ int lperm[4 * kWave];
  __shared__ int lpick;
  const int lane = threadIdx.x;
  if (two_way) {
    if (lane == 0) out[0] = two_way_draw<kOcml>(logw[0], logw[1], rU);
    return;
  }
  double pv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) pv[r] = (r * kWave + lane < E) ? logw[r * kWave + lane] : -INFINITY;
  const int pick = decide_values<4, kOcml>(pv, E, rU, lp, lperm, &lpick);
  if (lane == 0) out[0] = pick;
}
template <bool kOcml>
__global__ void k_debug_math(const double* x, int64_t n, int fn, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fn == 0 ? dexp<kOcml>(x[i]) : dlog<kOcml>(x[i]);
}
hipError_t launch_debug_draw(const double* logw, int E, double rU, int two_way, int ocml, int* out, hipStream_t s) {
  if (E < 1 || E > 4 * kWave || (two_way && E != 2)) return hipErrorInvalidValue;
  if (ocml) HDPM_LAUNCH(k_debug_draw<true>, dim3(1), dim3(kWave), 0, s, logw, E, rU, two_way, out);
  else HDPM_LAUNCH(k_debug_draw<false>, dim3(1), dim3(kWave), 0, s, logw, E, rU, two_way, out);
  return hipGetLastError();
}
hipError_t launch_debug_math(const double* x, int64_t n, int fn, int ocml, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 g((unsigned)((n + kBlock - 1) / kBlock));
  if (ocml) HDPM_LAUNCH(k_debug_math<true>, g, dim3(kBlock), 0, s, x, n, fn, out);
  else HDPM_LAUNCH(k_debug_math<false>, g, dim3(kBlock), 0, s, x, n, fn, out);
  return hipGetLastError();
}
// Frequency tables of the split-merge move on the device (split_merge.inl sm_freq_device):
// workgroup (c, part) counts attribute chunk c (16 attributes, one 16-byte load of the tiled
// codes per point) over its share of the list in LDS, then adds its nonzero counters to the
// table.  Counts are integers, so the table equals the host's membership count exactly.
constexpr int kSmFreqThreads = 256;
__global__ __launch_bounds__(kSmFreqThreads) void k_sm_freq(SmFreqArgs a, int parts) {
  if (a.link && __builtin_amdgcn_readfirstlane(a.link->ok) == 0) return;
  extern __shared__ uint32_t s_bins[];            // [16][mmax]
  const int c = blockIdx.x / parts, part = blockIdx.x - c * parts;
  const int nb = 16 * a.mmax;
  for (int e = threadIdx.x; e < nb; e += kSmFreqThreads) s_bins[e] = 0u;
  __syncthreads();
  const int per = (a.nlist + 2 + parts - 1) / parts;
  const int q0 = part * per, q1 = min(a.nlist + 2, q0 + per);
  // 4 points per lane at a time: their indices, then their code chunks, in flight together
  constexpr int kB = 4;
  for (int qb = q0; qb < q1; qb += kB * kSmFreqThreads) {
    int pi[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const int q = qb + k * kSmFreqThreads + (int)threadIdx.x;
      int i = -1;
      if (q < q1) {
        if (a.side_prev) {
          // delta mode: only the points that changed sides, +1 onto `want`, -1 off it
          if (q < a.nlist && a.side[q] != a.side_prev[q]) i = a.side[q] == a.want ? a.list[q] : ~a.list[q];
          else i = INT_MIN;
        } else if (q < a.nlist) {
          i = (a.side && a.side[q] != a.want) ? INT_MIN : a.list[q];
        } else {
          i = a.extra[q - a.nlist] >= 0 ? a.extra[q - a.nlist] : INT_MIN;
        }
      }
      pi[k] = q < q1 ? i : INT_MIN;
    }
    uint4 v[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const int i = pi[k] == INT_MIN ? -1 : (pi[k] < 0 ? ~pi[k] : pi[k]);
      v[k] = i >= 0 ? *(const uint4*)(a.codes_t + tiled_offset(i, c * 16, a.nq)) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      if (pi[k] == INT_MIN) continue;
      const uint32_t inc = pi[k] < 0 ? 0xffffffffu : 1u;
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const int x = (int)((w[b >> 2] >> (8 * (b & 3))) & 0xffu);
        if (x > 0 && c * 16 + b < a.d) atomicAdd(&s_bins[b * a.mmax + x - 1], inc);
      }
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nb; e += kSmFreqThreads) {
    const int j = c * 16 + e / a.mmax;
    if (j < a.d && s_bins[e]) atomicAdd(&a.out[(size_t)j * a.mmax + e % a.mmax], s_bins[e]);
  }
}

hipError_t launch_sm_freq(const SmFreqArgs& a, hipStream_t s) {
  if (!a.prezeroed) {
    const hipError_t e = hipMemsetAsync(a.out, 0, (size_t)a.d * a.mmax * 4, s);
    if (e != hipSuccess) return e;
  }
  const size_t lds = (size_t)16 * a.mmax * 4;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  // about 512 workgroups, every point list split into `parts` shares per attribute chunk
  const int parts = std::max(1, std::min((a.nlist + 2 + 255) / 256, 512 / std::max(a.nq, 1)));
  HDPM_LAUNCH(k_sm_freq, dim3((unsigned)(a.nq * parts)), dim3(kSmFreqThreads), lds, s, a, parts);
  return hipGetLastError();
}

// The device chain's link before scan k (SmLinkArgs): one workgroup.
__global__ __launch_bounds__(256) void k_sm_link(SmLinkArgs a) {
  __shared__ int s_ok;
  __shared__ int64_t s_r, s_end;
  if (threadIdx.x == 0) {
    int ok = __hip_atomic_load(&a.prev->ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t end = (int64_t)__hip_atomic_load((const uint64_t*)&a.prev->end, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    const int64_t r = end - a.win_start;
    if (r < 0 || r + a.nS > a.win_count) ok = 0;
    s_ok = ok;
    s_r = r;
    s_end = end;
  }
  __syncthreads();
  const int ok = s_ok;
  if (ok && a.stage[0]) {
    const UploadLayout L = upload_layout(1, a.dp, a.d, a.bw);
    for (int e = 0; e < 2; ++e) {
      const uint8_t* sb = a.stage[e ^ a.swap];
      const uint8_t* sc = sb + L.off_codes;
      const double* st = reinterpret_cast<const double*>(sb + L.off_tab);
      for (int j = threadIdx.x; j < a.dp; j += blockDim.x) a.two_codes[(size_t)e * a.dp + j] = sc[j];
      for (int j = threadIdx.x; j < 2 * a.d; j += blockDim.x) a.two_tab[(size_t)e * 2 * a.d + j] = st[j];
    }
  }
  if (threadIdx.x == 0) {
    a.link->raw = ok ? a.win_raw + s_r : nullptr;
    a.link->n1 = a.counts_in ? a.counts_in[0] : a.n1;
    a.link->n2 = a.counts_in ? a.counts_in[1] : a.n2;
    a.link->ok = ok;
    a.chain->end = s_end;
    a.chain->ok = ok;
  }
}
hipError_t launch_sm_link(const SmLinkArgs& a, hipStream_t s) {
  HDPM_LAUNCH(k_sm_link, dim3(1), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Both tables of the device chain after scan k (SmTabsArgs).
__global__ __launch_bounds__(256) void k_sm_tabs(SmTabsArgs a) {
  if (__builtin_amdgcn_readfirstlane(a.link->ok) == 0) return;
  uint32_t* f1 = a.F + (size_t)a.a1 * a.nt;
  uint32_t* f2 = a.F + (size_t)(1 - a.a1) * a.nt;
  for (int e = blockIdx.x * 256 + (int)threadIdx.x; e < a.nt; e += gridDim.x * 256) {
    const uint32_t x = f1[e] + a.delta[e];
    f1[e] = x;
    f2[e] = a.fm[e] - x;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int c0 = a.counts[0], c1 = a.counts[1];
    a.lab_cnt[0] = 0;
    a.lab_cnt[1] = 1;
    a.lab_cnt[2] = a.a1 == 0 ? c0 : c1;
    a.lab_cnt[3] = a.a1 == 0 ? c1 : c0;
  }
}
hipError_t launch_sm_tabs(const SmTabsArgs& a, hipStream_t s) {
  const int g = std::max(1, std::min(64, (a.nt + 255) / 256));
  HDPM_LAUNCH(k_sm_tabs, dim3((unsigned)g), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sm_lpgs(const SmArgs& a, hipStream_t s) {
  if (a.nS == 0) return hipSuccess;
  HDPM_LAUNCH(k_sm_lpgs, dim3((a.nS + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace hdpm

namespace hdpm {

__device__ __forceinline__ uint32_t mt_f(uint32_t a, uint32_t b, uint32_t c) {
  return c ^ (((a & 0x80000000u) | (b & 0x7fffffffu)) >> 1) ^ ((b & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// New value of element k after one in-place twist (R MT_genrand), from the old array only.
__device__ __forceinline__ uint32_t mt_twist_elem(const uint32_t* o, int k) {
  auto g1 = [&](int i) { return mt_f(o[i], o[i + 1], o[i + 397]); };            // i < 227
  auto g2 = [&](int i) { return mt_f(o[i], o[i + 1], g1(i - 227)); };           // 227 <= i < 454
  if (k < 227) return g1(k);
  if (k < 454) return g2(k);
  if (k < 623) return mt_f(o[k], o[k + 1], g2(k - 227));
  return mt_f(o[623], g1(0), g2(396));
}

__global__ __launch_bounds__(640) void k_mt_gen(MtGenArgs a) {
  __shared__ uint32_t buf[2][624];
  const int t = threadIdx.x;
  if (t < 624) buf[0][t] = a.init[t];
  __syncthreads();
  const int head = a.mti0 >= 624 ? 0 : 624 - a.mti0;
  for (int r = t; r < head && r < a.count; r += 640) a.out[r] = mt_temper(buf[0][a.mti0 + r]);
  int cur = 0;
  for (int b = 1; b <= a.nblocks; ++b) {
    uint32_t nv = 0;
    if (t < 624) {
      nv = mt_twist_elem(buf[cur], t);
      buf[cur ^ 1][t] = nv;
    }
    // LDS-only barrier: the global stores of earlier blocks stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t < 624) {
      if (b >= a.export_from) a.arrays[(int64_t)(b - 1) * 624 + t] = nv;
      const int64_t r = head + (int64_t)(b - 1) * 624 + t;
      if (r < a.count) a.out[r] = mt_temper(nv);
    }
    cur ^= 1;
  }
}

// G workgroups; workgroup g jumps 624 * bpg * g words ahead of X_0 with one GF(2)
// correlation (jpoly[g] = z^(624 bpg g - 1) mod phi, offset +1) of the next 33 blocks of
// the stream (mtjump.hpp), then twists its own
// segment of blocks [g * bpg, (g + 1) * bpg) (the last active one runs to the end).
constexpr int kJumpChunk = 4096;
__global__ __launch_bounds__(640) void k_mt_gen_multi(MtGenArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* seq = lds;                    // 33 * 624 words (jumping workgroups)
  uint32_t* buf0 = lds + 33 * 624;        // 2 * 624 words
  uint32_t* buf1 = buf0 + 624;
  uint32_t* jl = buf1 + 624;              // kJumpChunk staged bit positions
  const int t = threadIdx.x;
  const int g = blockIdx.x;
  const int64_t b_last = (a.count - 1 + a.mti0) / 624;      // last block with an output
  const int64_t b_first = (int64_t)g * a.bpg;
  if (b_first > b_last) return;
  const bool last = (g == a.G - 1) || ((int64_t)(g + 1) * a.bpg > b_last);
  const int64_t b_end = last ? b_last + 1 : (int64_t)(g + 1) * a.bpg;
  if (g == 0) {
    if (t < 624) buf0[t] = a.init[t];
  } else {
    if (t < 624) seq[t] = t == 0 ? (a.init[0] & 0x80000000u) : a.init[t];
    for (int blk = 1; blk < 33; ++blk) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (t < 624) seq[blk * 624 + t] = mt_twist_elem(seq + (blk - 1) * 624, t);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // out[t] = XOR over the set bits i of the jump polynomial of seq[i + t + 1].  The bit
    // positions are staged through LDS in chunks (coalesced loads; every lane then reads
    // the same index, an LDS broadcast), so no lane waits on a global load per index.
    uint32_t acc = 0;
    const uint32_t* L = a.jidx + ldu(a.joff + g);
    const int cnt = ldu(a.joff + g + 1) - ldu(a.joff + g);
    const uint32_t* s0 = seq + t + 1;
    for (int c0 = 0; c0 < cnt; c0 += kJumpChunk) {
      const int cn = min(kJumpChunk, cnt - c0);
      for (int q = t; q < cn; q += blockDim.x) jl[q] = L[c0 + q];
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (t < 624) {
        int q = 0;
        for (; q + 16 <= cn; q += 16) {
          uint32_t v[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v[u] = s0[jl[q + u]];
#pragma unroll
          for (int u = 0; u < 16; ++u) acc ^= v[u];
        }
        for (; q < cn; ++q) acc ^= s0[jl[q]];
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (t < 624) buf0[t] = acc;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  uint32_t* cur = buf0;
  uint32_t* nxt = buf1;
  for (int64_t b = b_first; b < b_end; ++b) {
    uint32_t nv = 0;
    if (b > b_first) {
      if (t < 624) {
        nv = mt_twist_elem(cur, t);
        nxt[t] = nv;
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      uint32_t* tmp = cur;
      cur = nxt;
      nxt = tmp;
    } else if (t < 624) {
      nv = cur[t];
    }
    if (t < 624) {
      if (b >= 1 && b >= a.export_from) a.arrays[(b - 1) * 624 + t] = nv;
      const int64_t r = b * 624 + t - a.mti0;
      if (r >= 0 && r < a.count) a.out[r] = mt_temper(nv);
    }
  }
}

hipError_t launch_mt_gen(const MtGenArgs& a, hipStream_t s) {
  if (a.G > 1 && a.jpoly) {
    const size_t lds = ((size_t)(33 + 2) * 624 + kJumpChunk) * 4;
    HDPM_LAUNCH(k_mt_gen_multi, dim3(a.G), dim3(640), lds, s, a);
  } else {
    HDPM_LAUNCH(k_mt_gen, dim3(1), dim3(640), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace hdpm
