// pool.hip -- device side of the stream-exact latent-pool generator (pool_gen.hpp).
//
//   k_pool_accept  every possible rbeta attempt of the slice, per attribute class, packed
//                  per position parity (one wave = 128 stream positions, ballots)
//   k_pool_values  one wave per pool entry: centers, the entry's accepted attempts (wave
//                  popcount scan + select over the packed words, run by run), sigma and
//                  dhamming tables, bound record (kernels.hpp layout)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"
#include "pool_gen.hpp"

namespace hdpm {

namespace {

__device__ __forceinline__ void load_tables(const uint64_t* g, uint64_t* lds) {
  for (int i = threadIdx.x; i < 512; i += blockDim.x) lds[i] = g[i];
  __syncthreads();
}

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace

__global__ __launch_bounds__(256) void k_pool_accept(PoolAcceptArgs a) {
  __shared__ uint64_t tabs[512];
  load_tables(a.gtab, tabs);
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wv >= a.nwords) return;
  const int64_t p0 = wv * 128 + 2 * lane;
  uint32_t y[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (p0 + k < a.count) y[k] = a.raw[p0 + k];
  const bool v0 = p0 + 1 < a.count, v1 = p0 + 2 < a.count;
  const double u0 = pool_unif(y[0]), u1 = pool_unif(y[1]), u2 = pool_unif(y[2]);
  const bool pe = a.par_mask & 1, po = (a.par_mask >> 1) & 1;
  for (int c = 0; c < a.nclass; ++c) {
    const PoolClass C = a.cls[c];
    const bool acc0 = pe && v0 && pool_accept(C, u0, u1, tabs, tabs + 256);
    const bool acc1 = po && v1 && pool_accept(C, u1, u2, tabs, tabs + 256);
    const uint64_t b0 = __ballot(acc0), b1 = __ballot(acc1);
    if (lane == 0) {
      if (pe) a.bm[((int64_t)c * 2 + 0) * a.nwords + wv] = b0;
      if (po) a.bm[((int64_t)c * 2 + 1) * a.nwords + wv] = b1;
    }
  }
}

// Position after the len-th accepted attempt at the parity of pos, from pos (B: that parity's
// table), by one wave 64 words at a time; -1 past the tables (pool_select_run).
__device__ __forceinline__ int64_t wave_select_run(const uint64_t* B, int64_t nwords, int64_t pos, int len) {
  const int lane = threadIdx.x & 63;
  const int par = (int)(pos & 1);
  const int64_t slot = pos >> 1;
  int64_t w = slot >> 6;
  uint64_t fmask = ~0ull << (slot & 63);
  int need = len;
  for (;;) {
    if (w >= nwords) return -1;
    const int64_t wi = w + lane;
    uint64_t word = wi < nwords ? B[wi] : 0ull;
    if (lane == 0) word &= fmask;
    const int cnt = __popcll(word);
    const int incl = wave_incl_scan(cnt);
    const int total = __shfl(incl, 63);
    if (total >= need) {
      const uint64_t reach = __ballot(incl >= need);
      const int q = __ffsll((unsigned long long)reach) - 1;
      const uint64_t wq = __shfl(word, q);
      const int before = __shfl(incl - cnt, q);
      return 2 * ((w + q) * 64 + pool_select64(wq, need - before - 1)) + par + 2;
    }
    need -= total;
    w += 64;
    fmask = ~0ull;
  }
}

// One wave per chunk (pool_gen.hpp PoolWalkArgs): C + M entry starts from a guess.
__global__ __launch_bounds__(256) void k_pool_walk(PoolWalkArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= a.chunks) return;
  const int64_t e0 = g * a.C;
  const int L = a.C + a.M;
  int64_t* out = a.walk + g * L;
  int64_t pos = 0;
  if (g > 0) {
    const int par = (int)((e0 * a.d) & 1);
    pos = (int64_t)((double)e0 * a.mu);
    if (pos > a.count - 2) pos = a.count - 2;
    if (pos < 0) pos = 0;
    pos = (pos & ~(int64_t)1) | par;
  }
  for (int k = 0; k < L; ++k) {
    if (lane == 0) out[k] = pos;
    if (k + 1 == L) break;
    pos += a.d;
    for (int r = 0; r < a.nruns && pos >= 0; ++r)
      pos = wave_select_run(a.bm + ((int64_t)a.run_cls[r] * 2 + (pos & 1)) * a.nwords, a.nwords, pos, a.run_len[r]);
    if (pos < 0) {
      if (lane == 0)
        for (int k2 = k + 1; k2 < L; ++k2) out[k2] = -1;
      return;
    }
  }
}

// One wave per chunk g >= 1: the first position of its walk found in chunk g - 1's walk (a
// binary search per lane: both walks increase), hence rel[g] = k1 - k2 - C and the index k1 in
// chunk g - 1's walk where chunk g's valid part starts.
__global__ __launch_bounds__(256) void k_pool_meet(PoolWalkArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t g = 1 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= a.chunks) return;
  const int L = a.C + a.M;
  const int64_t* prev = a.walk + (g - 1) * L;
  const int64_t* own = a.walk + g * L;
  int nprev = L;                       // prev's positions before its -1 marks (near the tables' end)
  while (nprev > 0 && prev[nprev - 1] < 0) --nprev;
  for (int k0 = 0; k0 < L; k0 += 64) {
    const int k2 = k0 + lane;
    int k1 = -1;
    if (k2 < L) {
      const int64_t x = own[k2];
      if (x >= 0) {
        int lo = 0, hi = nprev;        // first index with prev[idx] >= x
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (prev[mid] < x) lo = mid + 1;
          else hi = mid;
        }
        if (lo < nprev && prev[lo] == x) k1 = lo;
      }
    }
    const uint64_t b = __ballot(k1 >= 0);
    if (b) {
      const int q = __ffsll((unsigned long long)b) - 1;
      const int K1 = __shfl(k1, q), K2 = k0 + q;
      if (lane == 0) {
        a.rel[g] = K1 - K2 - a.C;
        a.a[g] = K1;                   // made an entry index by k_pool_scan
      }
      return;
    }
  }
  if (lane == 0) {
    a.rel[g] = 0;
    a.a[g] = -1;
    atomicOr(a.err, 4);
  }
}

// One workgroup: delta_g = sum of rel over chunks 1..g; a_g = e_{g-1} + delta_{g-1} + k1_g, then
// a running maximum (a walk that met its predecessor before that one met the true chain is
// true only from where its predecessor is); a_0 = 0, a_chunks = P + 1.
template <bool kMax>
__device__ __forceinline__ long long block_scan(long long x, long long* carry, long long* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(x, o);
    if (lane >= o) x = kMax ? (t > x ? t : x) : x + t;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  long long before = *carry;
  for (int w2 = 0; w2 < wid; ++w2) before = kMax ? (wsum[w2] > before ? wsum[w2] : before) : before + wsum[w2];
  const long long r = kMax ? (x > before ? x : before) : before + x;
  __syncthreads();
  if (threadIdx.x == blockDim.x - 1) *carry = r;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(1024) void k_pool_scan(PoolWalkArgs a) {
  __shared__ long long carry;
  __shared__ long long wsum[16];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < a.chunks; base += blockDim.x) {
    const int64_t g = base + threadIdx.x;
    const long long dl = block_scan<false>((g >= 1 && g < a.chunks) ? (long long)a.rel[g] : 0, &carry, wsum);
    if (g < a.chunks) a.delta[g] = dl;
  }
  __syncthreads();
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < a.chunks; base += blockDim.x) {
    const int64_t g = base + threadIdx.x;
    long long v = 0;
    if (g >= 1 && g < a.chunks) {
      const long long k1 = a.a[g];
      v = k1 >= 0 ? (long long)((g - 1) * a.C) + a.delta[g - 1] + k1 : 0;
    }
    const long long r = block_scan<true>(v, &carry, wsum);
    if (g >= 1 && g < a.chunks && a.a[g] >= 0) a.a[g] = r;
  }
  if (threadIdx.x == 0) {
    a.a[0] = 0;
    a.a[a.chunks] = a.P + 1;
  }
}

// One wave per chunk g: entries [a_g, a_{g+1}) from its walk (walk index e - g C - delta_g).
__global__ __launch_bounds__(256) void k_pool_place(PoolWalkArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= a.chunks || (*a.err & 4)) return;
  const int L = a.C + a.M;
  const int64_t lo = a.a[g], hi = min(a.a[g + 1], a.P + 1);
  const int64_t off = g * a.C + a.delta[g];          // the entry of walk index 0
  const int64_t* w = a.walk + g * L;
  if (lane == 0 && (lo < 0 || hi < lo)) atomicOr(a.err, 4);
  for (int64_t e = max(lo, (int64_t)0) + lane; e < hi; e += 64) {
    const int64_t k = e - off;
    int64_t v = -1;
    if (k >= 0 && k < L) v = w[k];
    if (v < 0) atomicOr(a.err, (e == a.P && k >= 0 && k < L) ? 8 : 4);
    a.starts[e] = v;
  }
}

// dynamic LDS: 512 table words, then per wave d doubles of sigma and 2d of tables
__global__ __launch_bounds__(256) void k_pool_values(PoolValueArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  load_tables(a.gtab, lds);
  const uint64_t* texp = lds;
  const uint64_t* tlog = lds + 256;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 4 + wid;
  if (e >= a.P) return;
  const int d = a.d;
  double* wsig = reinterpret_cast<double*>(lds + 512) + (size_t)wid * 3 * d;
  double* wtab = wsig + d;
  const int64_t s = a.starts[e];

  // centers (common_functions.cpp:198-199): code = (int)(m_j * u + 1)
  uint8_t* codes = a.codes + e * a.dp;
  for (int j = lane; j < a.dp; j += 64)
    codes[j] = j < d ? (uint8_t)(int)(a.att[j] * pool_unif(a.raw[s + j]) + 1) : (uint8_t)0;

  // sigmas: run by run, the run's accepted attempts in stream order
  int64_t pos = s + d;
  int j0 = 0;
  bool bad_attempt = false;
  for (int r = 0; r < a.nruns; ++r) {
    const int c = a.run_cls[r], len = a.run_len[r];
    const PoolClass C = a.cls[c];
    const int par = (int)(pos & 1);
    const uint64_t* B = a.bm + ((int64_t)c * 2 + par) * a.nwords;
    const int64_t slot = pos >> 1;
    int64_t wbase = slot >> 6;
    uint64_t fmask = ~0ull << (slot & 63);
    int done = 0;
    int64_t last = -1;
    while (done < len) {
      const int64_t wi = wbase + lane;
      uint64_t word = wi < a.nwords ? B[wi] : 0ull;
      if (lane == 0) word &= fmask;
      const int cnt = __popcll(word);
      const int incl = wave_incl_scan(cnt);
      const int total = __shfl(incl, 63);
      if (total == 0 && wbase + 64 >= a.nwords) {   // out of tables: the host parse disagrees
        if (lane == 0) atomicOr(a.err, 1);
        return;
      }
      const int nb = min(len - done, total);
      for (int t0 = 0; t0 < nb; t0 += 64) {
        const int t = t0 + lane;
        const bool act = t < nb;
        const int tt = act ? t : nb - 1;
        int q = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
          if (__shfl(incl, q + step - 1) <= tt) q += step;
        const uint64_t wq = __shfl(word, q);
        const int prev = __shfl(incl, q) - __shfl(cnt, q);
        const int bit = pool_select64(wq, tt - prev);
        const int64_t p = 2 * ((wbase + q) * 64 + bit) + par;
        if (act) {
          const int j = j0 + done + t;
          const double u1 = pool_unif(a.raw[p]), u2 = pool_unif(a.raw[p + 1]);
          double x = 0.0;
          if (!pool_attempt(C, u1, u2, texp, tlog, &x) || x > C.thr) bad_attempt = true;
          double sg, m0, m1;
          pool_sigma_tables(C, x, a.att[j], texp, tlog, &sg, &m0, &m1);
          wsig[j] = sg;
          wtab[2 * j] = m0;
          wtab[2 * j + 1] = m1;
        }
        last = __shfl(p, (nb - 1 - t0) & 63);
      }
      done += nb;
      wbase += 64;
      fmask = ~0ull;
    }
    pos = last + 2;
    j0 += len;
  }
  if (lane == 0 && pos != a.starts[e + 1]) atomicOr(a.err, 1);
  if (__ballot(bad_attempt) && lane == 0) atomicOr(a.err, 2);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  double* tab = a.tab + e * 2 * d;
  double* sig = a.sig + e * d;
  double A = 0.0, sc = 0.0, dmx = 0.0, dmn = __builtin_inf();
  for (int j = lane; j < d; j += 64) {
    const double m0 = wtab[2 * j], m1 = wtab[2 * j + 1];
    tab[2 * j] = m0;
    tab[2 * j + 1] = m1;
    sig[j] = wsig[j];
    A += m0;
    sc += fmax(fabs(m0), fabs(m1));
    const double dj = m0 - m1;
    dmx = fmax(dmx, dj);
    dmn = fmin(dmn, dj);
  }
  A = wave_sum(A);
  sc = wave_sum(sc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dmx = fmax(dmx, __shfl_xor(dmx, o));
    dmn = fmin(dmn, __shfl_xor(dmn, o));
  }
  // bound record (Ctx::bounds_for, kernels.hpp "Bound data per parameter entry")
  const double delta = dmx > 0 ? dmx / ((1 << kQ) - 1) : 0.0;
  uint64_t* rec = a.bnd + e * a.bw;
  for (int k = 0; k < a.Ws; ++k) {
    const int j = 64 * k + lane;
    const bool valid = j < d;
    const unsigned code = valid ? codes[j] - 1u : 0u;
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
  if (lane == 0) {
    double* sv = reinterpret_cast<double*>(rec + (a.wb + kQ) * a.Ws);
    sv[0] = A;
    sv[1] = delta;
    sv[2] = dmn > 0 ? dmn : 0.0;
    sv[3] = sc;
  }
}

__device__ __forceinline__ float f32_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -__builtin_inff());
  return f;
}
__device__ __forceinline__ float f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, __builtin_inff());
  return f;
}

// Order-preserving key of a double (unsigned compare of keys = numeric compare).
__device__ __forceinline__ uint64_t dkey(double x) {
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// Sum of the h smallest of the wave's values dv (NV per lane, +inf padding): bisection on
// the key for the h-th smallest value t (64 steps, each a wave-wide count of keys < mid),
// then sum(values < t) + (h - count(values < t)) t.
template <int NV>
__device__ __forceinline__ double sum_smallest(const double (&dv)[NV], const uint64_t (&key)[NV], int h) {
  if (h <= 0) return 0.0;
  uint64_t lo = 0, hi = ~0ull;        // invariant: count(key <= lo) < h <= count(key <= hi)
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    int c = 0;
#pragma unroll
    for (int k = 0; k < NV; ++k) c += __popcll(__ballot(key[k] <= mid));
    if (c >= h) hi = mid;
    else lo = mid;
  }
  // hi is the key of the h-th smallest value
  double s = 0.0, t = -__builtin_inf();
  int below = 0;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (key[k] < hi) s += dv[k];
    if (key[k] == hi) t = dv[k];
    below += __popcll(__ballot(key[k] < hi));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    t = fmax(t, __shfl_xor(t, o));     // every lane holding the key holds the same value
  }
  return s + (double)(h - below) * t;
}

// Pool-entry heads (kernels.hpp) from the dhamming tables and bound records: one wave per
// entry, nv = Ws attributes per lane (d <= 64 nv, nv <= NV).  S_a / S_b are the sums of the
// h_a / h_b smallest d_j (sum_smallest).  Host and device pools alike.
template <int NV>
__global__ __launch_bounds__(256) void k_pool_heads(const double* __restrict__ tab, const uint64_t* __restrict__ bnd,
                                                   int64_t P, int d, int wb, int nv, int bw, int ha, int hb,
                                                   uint64_t* __restrict__ head) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= P) return;
  const double* t = tab + e * 2 * d;
  double dv[NV];
  uint64_t key[NV];
  double mn = __builtin_inf();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int j = 64 * k + lane;
    dv[k] = j < d ? t[2 * j] - t[2 * j + 1] : __builtin_inf();   // d_j as in Ctx::bounds_for
    key[k] = dkey(dv[k]);
    mn = fmin(mn, dv[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o));
  const double sa = sum_smallest<NV>(dv, key, ha < d ? ha : d);
  const double sb = sum_smallest<NV>(dv, key, hb < d ? hb : d);
  const int HW = wb * nv + 2, HS = head_stride(wb, nv);
  const uint64_t* r = bnd + e * bw;
  for (int q = lane; q < HS; q += 64) {
    uint64_t v = 0;
    if (q >= HW) {
      // padding to the head stride
    } else if (q < HW - 2) {
      v = r[q];
    } else if (q == HW - 2) {
      const int SC = (wb + kQ) * nv;
      const double A_up = __longlong_as_double((long long)r[SC]) +
                          kBoundEps * (1.0 + __longlong_as_double((long long)r[SC + 3]));
      v = (uint64_t)__float_as_uint(f32_up(A_up)) | ((uint64_t)__float_as_uint(f32_down(mn > 0 ? mn : 0.0)) << 32);
    } else {
      // one float ulp below the rounded-down sums: the double sums' own rounding (<= d ulps)
      // stays on the safe side
      const float fa = nextafterf(f32_down(sa), -__builtin_inff()), fb = nextafterf(f32_down(sb), -__builtin_inff());
      v = (uint64_t)__float_as_uint(ha > 0 ? fmaxf(fa, 0.0f) : 0.0f) |
          ((uint64_t)__float_as_uint(hb > 0 ? fmaxf(fb, 0.0f) : 0.0f) << 32);
    }
    head[e * HS + q] = v;
  }
}

hipError_t launch_pool_heads(const double* tab, const uint64_t* bnd, int64_t P, int d, int wb, int Ws, int bw, int ha,
                             int hb, uint64_t* head, hipStream_t s) {
  if (P <= 0) return hipSuccess;
  if (!head_fits(wb, Ws)) return hipErrorInvalidValue;
  const dim3 g((unsigned)((P + 3) / 4)), b(256);
  if (Ws == 2) hipLaunchKernelGGL(k_pool_heads<2>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws == 4) hipLaunchKernelGGL(k_pool_heads<4>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws <= 8) hipLaunchKernelGGL(k_pool_heads<8>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws <= 16) hipLaunchKernelGGL(k_pool_heads<16>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else hipLaunchKernelGGL(k_pool_heads<32>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  return hipGetLastError();
}

hipError_t launch_pool_accept(const PoolAcceptArgs& a, hipStream_t s) {
  const int64_t blocks = (a.nwords + 3) / 4;
  hipLaunchKernelGGL(k_pool_accept, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pool_walk(const PoolWalkArgs& a, hipStream_t s) {
  if (a.C < 1 || a.M < 1 || a.chunks < 1) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)((a.chunks + 3) / 4);
  hipLaunchKernelGGL(k_pool_walk, dim3(blocks), dim3(256), 0, s, a);
  if (a.chunks > 1) hipLaunchKernelGGL(k_pool_meet, dim3((unsigned)((a.chunks - 1 + 3) / 4)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_pool_scan, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_pool_place, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pool_values(const PoolValueArgs& a, hipStream_t s) {
  const int64_t blocks = (a.P + 3) / 4;
  const size_t lds = 512 * 8 + (size_t)4 * 3 * a.d * 8;
  hipLaunchKernelGGL(k_pool_values, dim3((unsigned)blocks), dim3(256), lds, s, a);
  return hipGetLastError();
}

}  // namespace hdpm
