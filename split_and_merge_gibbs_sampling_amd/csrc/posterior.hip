// posterior.hip -- posterior similarity matrix and VI lower bounds on the device.
//
// The reference's analysis (realdata_analysis/zoo_simulator.R:193-236, 339-344) computes
// comp.psm(C) (mcclust: psm[i][j] = share of the saved iterations in which points i and j
// share a cluster), minVI(psm) (mcclust.ext: the partition minimising the lower bound of
// the posterior expected variation of information) and arandi.  At the BASELINE sizes the
// N x N matrix is the whole cost (C4: 70k^2 = 4.9e9 entries; R holds it as doubles in 39
// GB), so it is built and queried here:
//
//   k_psm_pack   the saved labels (M x N int32, the reference's results$c_i) transposed to
//                one byte per (point, iteration), rows padded to a multiple of 16 with 0xFF
//   k_psm_tile   co-clustering counts of a 128 x 128 tile of point pairs: the two rows'
//                label bytes 16 iterations at a time (LDS), XOR, and the zero bytes counted
//                ((x & 0x7f7f7f7f) + 0x7f7f7f7f | x has the top bit of every nonzero byte,
//                v_bcnt of the complement's top bits adds the equal ones); tiles with
//                j >= i only, mirrored; counts exact in uint32 (psm = count / M)
//   k_vi_terms   per point i and candidate partition c: sum_j psm[i][j] and
//                sum_{j: c_j = c_i} psm[i][j] (the two sums of mcclust.ext VI.lb)
//
// Bound: k_psm_tile is VALU-bound (compare + count of N^2 / 2 pairs x M iterations, 5
// integer ops per 4 iterations of a pair); k_vi_terms streams the N^2 counts once per
// candidate (HBM).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hdpm {

constexpr int kPsmTile = 128;
constexpr int kPsmThreads = 256;

__global__ void k_psm_pack(const int32_t* __restrict__ trace, int M, int N, int Mp, uint8_t* __restrict__ lab) {
  // one thread per (point, iteration), iterations fastest in the output row
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)N * Mp;
  if (t >= tot) return;
  const int i = (int)(t / Mp), m = (int)(t % Mp);
  lab[t] = m < M ? (uint8_t)trace[(int64_t)m * N + i] : (uint8_t)0xFF;
}

__device__ __forceinline__ uint32_t eq_bytes(uint32_t a, uint32_t b) {
  const uint32_t x = a ^ b;
  const uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;   // top bit set iff the byte != 0
  return __popc(~t & 0x80808080u);
}

// Tile (bi, bj) of kPsmTile x kPsmTile pairs, bj >= bi; thread (ty, tx) of 16 x 16 owns
// rows bi*128 + ty*8 .. +7 and columns bj*128 + tx*8 .. +7.
__global__ __launch_bounds__(kPsmThreads) void k_psm_tile(const uint8_t* __restrict__ lab, int N, int Mp, int pad,
                                                         uint32_t* __restrict__ cnt, int nt) {
  // linear tile index over the upper triangle (bj >= bi)
  int t = blockIdx.x, bi = 0;
  while (t >= nt - bi) { t -= nt - bi; ++bi; }
  const int bj = bi + t;
  __shared__ uint4 sa[kPsmTile], sb[kPsmTile];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = bi * kPsmTile, j0 = bj * kPsmTile;
  uint32_t acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = 0u;
  for (int m0 = 0; m0 < Mp; m0 += 16) {
    {
      const int r = tid & (kPsmTile - 1);
      const int row = (tid < kPsmTile ? i0 : j0) + r;
      uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      if (row < N) v = *(const uint4*)(lab + (int64_t)row * Mp + m0);
      if (tid < kPsmTile) sa[r] = v; else sb[r] = v;
    }
    __syncthreads();
    uint4 A[8], B[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) A[a] = sa[ty * 8 + a];
#pragma unroll
    for (int b = 0; b < 8; ++b) B[b] = sb[tx * 8 + b];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b)
        acc[a][b] += eq_bytes(A[a].x, B[b].x) + eq_bytes(A[a].y, B[b].y) + eq_bytes(A[a].z, B[b].z) +
                     eq_bytes(A[a].w, B[b].w);
    __syncthreads();
  }
  // padding iterations (0xFF in every row) match: subtract them
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = i0 + ty * 8 + a;
    if (i >= N) continue;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + tx * 8 + b;
      if (j >= N) continue;
      const uint32_t v = acc[a][b] - (uint32_t)pad;
      cnt[(int64_t)i * N + j] = v;
      if (bi != bj) cnt[(int64_t)j * N + i] = v;
    }
  }
}

// sums of row i of psm = cnt / M: over all j, and over j with cls[c][j] == cls[c][i]
// (one workgroup per (i, candidate); ordered per-thread partial sums, then a fixed-order
// tree: deterministic)
__global__ __launch_bounds__(256) void k_vi_terms(const uint32_t* __restrict__ cnt, int N, double dM,
                                                 const int32_t* __restrict__ cls, int ncand, double* __restrict__ all,
                                                 double* __restrict__ same) {
  const int i = blockIdx.x, c = blockIdx.y;
  const int32_t* cl = cls + (int64_t)c * N;
  const int ci = cl[i];
  const uint32_t* row = cnt + (int64_t)i * N;
  double sa = 0.0, ss = 0.0;
  for (int j = threadIdx.x; j < N; j += 256) {
    const double p = (double)row[j] / dM;     // psm = count / M
    sa += p;
    ss += cl[j] == ci ? p : 0.0;
  }
  __shared__ double ra[256], rs[256];
  ra[threadIdx.x] = sa;
  rs[threadIdx.x] = ss;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) { ra[threadIdx.x] += ra[threadIdx.x + o]; rs[threadIdx.x] += rs[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (c == 0) all[i] = ra[0];
    same[(int64_t)c * N + i] = rs[0];
  }
}

hipError_t launch_psm(const int32_t* trace, int M, int N, uint8_t* lab, uint32_t* cnt, hipStream_t s) {
  const int Mp = (M + 15) & ~15;
  const int64_t tot = (int64_t)N * Mp;
  hipLaunchKernelGGL(k_psm_pack, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, trace, M, N, Mp, lab);
  const int nt = (N + kPsmTile - 1) / kPsmTile;
  const int64_t ntiles = (int64_t)nt * (nt + 1) / 2;
  hipLaunchKernelGGL(k_psm_tile, dim3((unsigned)ntiles), dim3(kPsmThreads), 0, s, lab, N, Mp, Mp - M, cnt, nt);
  return hipGetLastError();
}

hipError_t launch_vi_terms(const uint32_t* cnt, int N, int M, const int32_t* cls, int ncand, double* all, double* same,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_vi_terms, dim3(N, ncand), dim3(256), 0, s, cnt, N, (double)M, cls, ncand, all, same);
  return hipGetLastError();
}

}  // namespace hdpm
