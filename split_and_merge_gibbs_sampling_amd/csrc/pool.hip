// pool.hip -- device side of the stream-exact latent-pool generator (pool_gen.hpp).
//
//   k_pool_accept  every possible rbeta attempt of the slice, per attribute class, packed
//                  per position parity (one wave = 128 stream positions, ballots)
//   k_pool_seg*    the entry starts: every window candidate of every chunk walked to the next
//                  chunk, the tables composed per group and chained, each chunk's entries
//                  walked from its first start on the chain (pool_gen.hpp PoolSegPlan)
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

// Entry starts by segments (pool_gen.hpp PoolSegPlan).  k_pool_seg: a workgroup per chunk, a
// thread per window candidate, walked to its first start in the next chunk (the candidates of a
// window read the same few table words: L1 / L2 hits).
__global__ __launch_bounds__(256) void k_pool_seg(PoolSegArgs a) {
  const int64_t c = blockIdx.x;
  for (int i = threadIdx.x; i < a.sp.ncand; i += blockDim.x)
    a.T[c * a.sp.ncand + i] = pool_seg_cell(a.bm, a.nwords, a.d, a.R, a.sp, c, i);
}

// The tables of a group's chunks composed, one thread per candidate of the group's first window.
__global__ __launch_bounds__(256) void k_pool_seg_group(PoolSegArgs a) {
  const int64_t g = blockIdx.x;
  const int64_t c0 = g * a.sp.G, c1 = min(a.sp.nchunks, c0 + a.sp.G);
  for (int i = threadIdx.x; i < a.sp.ncand; i += blockDim.x) {
    int idx = i, n = 0;
    bool bad = false;
    for (int64_t c = c0; c < c1; ++c) {
      const uint32_t t = a.T[c * a.sp.ncand + idx];
      if ((t & 0xFFFFu) == kSegBad) { bad = true; break; }
      idx = (int)(t & 0xFFFFu);
      n += (int)(t >> 16);
    }
    a.gj[g * a.sp.ncand + i] = bad ? -1 : idx;
    a.gn[g * a.sp.ncand + i] = n;
  }
}

// The chain over the groups (one thread, one dependent load per group), from candidate 0 of
// chunk 0; the group that holds entry P (or a broken cell) is unrolled per chunk here.
__global__ __launch_bounds__(64) void k_pool_seg_top(PoolSegArgs a) {
  if (threadIdx.x != 0) return;
  const PoolSegPlan& sp = a.sp;
  int idx = 0;
  int64_t E = 0, gfin = sp.ngroups;
  for (int64_t g = 0; g < sp.ngroups; ++g) {
    const int32_t j = a.gj[g * sp.ncand + idx], n = a.gn[g * sp.ncand + idx];
    a.cidx[g * sp.G] = idx;
    a.cE[g * sp.G] = E;
    if (j < 0 || E + n > a.P) {
      gfin = g;
      for (int64_t c = g * sp.G; c < min(sp.nchunks, (g + 1) * sp.G) && E <= a.P; ++c) {
        a.cidx[c] = idx;
        a.cE[c] = E;
        const uint32_t t = a.T[c * sp.ncand + idx];
        if ((t & 0xFFFFu) == kSegBad) break;
        idx = (int)(t & 0xFFFFu);
        E += t >> 16;
      }
      break;
    }
    idx = j;
    E += n;
  }
  a.aux[0] = gfin;
  if (gfin == sp.ngroups) atomicOr(a.err, 8);
}

// Every chunk of the groups before the unrolled one: its first start on the chain.
__global__ __launch_bounds__(256) void k_pool_seg_fill(PoolSegArgs a) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.aux[0]) return;
  int idx = a.cidx[g * a.sp.G];
  int64_t E = a.cE[g * a.sp.G];
  for (int64_t c = g * a.sp.G; c < min(a.sp.nchunks, (g + 1) * a.sp.G); ++c) {
    a.cidx[c] = idx;
    a.cE[c] = E;
    const uint32_t t = a.T[c * a.sp.ncand + idx];
    idx = (int)(t & 0xFFFFu);
    E += t >> 16;
  }
}

// A thread per chunk on the chain: its entries walked from its first start and written; the
// walk must end at the next chunk's first start (else the chain left a window: bit 2).
__global__ __launch_bounds__(256) void k_pool_seg_emit(PoolSegArgs a) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.sp.nchunks || a.cidx[c] < 0) return;
  const int64_t Xn = (c + 1) * a.sp.B;
  int64_t p = c * a.sp.B + (int64_t)a.cidx[c] * a.sp.step, e = a.cE[c];
  while (p < Xn) {
    a.starts[e] = p;
    if (e == a.P) return;
    p = pool_entry_end(a.bm, a.nwords, a.d, a.R, p);
    if (p < 0) {
      atomicOr(a.err, 8);
      return;
    }
    ++e;
  }
  if (!(c + 1 < a.sp.nchunks && a.cidx[c + 1] == (p - Xn) / a.sp.step && a.cE[c + 1] == e)) atomicOr(a.err, 4);
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

// S_a / S_b (the sums of the h_a / h_b smallest d_j), as lower bounds, by a bitonic sort of the wave's 64 NV values rounded
// down to float (32-bit keys, no payload: non-negative floats order as their bits; padding
// +inf sorts last).  The heads round both sums down to float and one ulp further, so the
// sums need only stay below the exact ones: every key is <= its d_j, and the double sums of
// at most 2048 floats round by far less than that float ulp.
template <int NV>
__device__ __forceinline__ void sum_smallest2(const double (&dv)[NV], int ha, int hb, double* sa, double* sb) {
  const int lane = threadIdx.x & 63;
  constexpr int N = 64 * NV;
  uint32_t key[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k)
    key[k] = dv[k] == __builtin_inf() ? 0x7f800000u : __float_as_uint(f32_down(dv[k] > 0.0 ? dv[k] : 0.0));
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int ks = stride >> 6;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          if (k & ks) continue;
          const bool up = ((k * 64 + lane) & size) == 0;
          const uint32_t x = key[k], y = key[k | ks];
          key[k] = up ? min(x, y) : max(x, y);
          key[k | ks] = up ? max(x, y) : min(x, y);
        }
      } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const bool up = ((k * 64 + lane) & size) == 0, lower = (lane & stride) == 0;
          const uint32_t o = (uint32_t)__shfl_xor((int)key[k], stride);
          key[k] = (lower == up) ? min(key[k], o) : max(key[k], o);
        }
      }
    }
  }
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int r = k * 64 + lane;
    const double x = (double)__uint_as_float(key[k]);
    a += r < ha ? x : 0.0;
    b += r < hb ? x : 0.0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  *sa = a;
  *sb = b;
}

// Pool-entry heads (kernels.hpp) from the dhamming tables and bound records: one wave per
// entry, nv = Ws attributes per lane (d <= 64 nv, nv <= NV).  S_a / S_b are the sums of the
// h_a / h_b smallest d_j, as lower bounds (sum_smallest2).  Host and device pools alike.
template <int NV>
__global__ __launch_bounds__(256) void k_pool_heads(const double* __restrict__ tab, const uint64_t* __restrict__ bnd,
                                                   int64_t P, int d, int wb, int nv, int bw, int ha, int hb,
                                                   uint64_t* __restrict__ head) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= P) return;
  const double* t = tab + e * 2 * d;
  double dv[NV];
  double mn = __builtin_inf();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int j = 64 * k + lane;
    dv[k] = j < d ? t[2 * j] - t[2 * j + 1] : __builtin_inf();   // d_j as in Ctx::bounds_for
    mn = fmin(mn, dv[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o));
  double sa, sb;
  sum_smallest2<NV>(dv, ha < d ? ha : d, hb < d ? hb : d, &sa, &sb);
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
  if (Ws == 2) HDPM_LAUNCH(k_pool_heads<2>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws == 4) HDPM_LAUNCH(k_pool_heads<4>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws <= 8) HDPM_LAUNCH(k_pool_heads<8>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else if (Ws <= 16) HDPM_LAUNCH(k_pool_heads<16>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  else HDPM_LAUNCH(k_pool_heads<32>, g, b, 0, s, tab, bnd, P, d, wb, Ws, bw, ha, hb, head);
  return hipGetLastError();
}

hipError_t launch_pool_accept(const PoolAcceptArgs& a, hipStream_t s) {
  const int64_t blocks = (a.nwords + 3) / 4;
  HDPM_LAUNCH(k_pool_accept, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pool_seg(const PoolSegArgs& a, hipStream_t s) {
  const PoolSegPlan& sp = a.sp;
  if (sp.nchunks < 1 || sp.ncand < 1 || sp.ncand >= 0xFFFF || sp.B < 2 || sp.G < 1 || sp.nchunks > 0x7fffffff ||
      sp.ngroups != (sp.nchunks + sp.G - 1) / sp.G)
    return hipErrorInvalidValue;
  HDPM_LAUNCH(k_pool_seg, dim3((unsigned)sp.nchunks), dim3(256), 0, s, a);
  HDPM_LAUNCH(k_pool_seg_group, dim3((unsigned)sp.ngroups), dim3(256), 0, s, a);
  HDPM_LAUNCH(k_pool_seg_top, dim3(1), dim3(64), 0, s, a);
  HDPM_LAUNCH(k_pool_seg_fill, dim3((unsigned)((sp.ngroups + 255) / 256)), dim3(256), 0, s, a);
  HDPM_LAUNCH(k_pool_seg_emit, dim3((unsigned)((sp.nchunks + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pool_values(const PoolValueArgs& a, hipStream_t s) {
  const int64_t blocks = (a.P + 3) / 4;
  const size_t lds = 512 * 8 + (size_t)4 * 3 * a.d * 8;
  HDPM_LAUNCH(k_pool_values, dim3((unsigned)blocks), dim3(256), lds, s, a);
  return hipGetLastError();
}

}  // namespace hdpm
