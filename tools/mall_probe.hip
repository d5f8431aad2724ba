// mall_probe.hip -- random-gather rate vs working-set size on one MI355X (design tool, not
// part of the library): can the prepass's pool-entry heads (3M random picks per C5 sweep)
// be served from the 256 MB Infinity Cache (MALL) if they were smaller?  Each pass has 1M
// threads gather three random records of 32, 48 or 64 B (the prepass's three latent heads per
// point) from a buffer of the given size, next to 16 B per thread of streamed data; warm-up
// passes first.  Prints the time per pass and the rate.
//   hipcc --offload-arch=gfx950 -O3 -o mall_probe tools/mall_probe.hip && ./mall_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

// thread t: G random records of W uint4 each (W = 2: 32 B, 3: 48 B, 4: 64 B), plus S uint4 of
// streamed data (the point rows) at t
template <int W>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ buf, int64_t nrec, int G,
                                                const uint4* __restrict__ stream, int64_t nstream, uint64_t seed,
                                                uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (t < nstream) {
    const uint4 v = stream[t];
    acc.x ^= v.x;
    acc.y ^= v.w;
  }
  uint4 v[3][W];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    if (r < G) {
      const int64_t e = (int64_t)(mix(seed + t * 131 + r) % (uint64_t)nrec);
#pragma unroll
      for (int k = 0; k < W; ++k) v[r][k] = buf[e * W + k];
    }
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
    if (r < G)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        acc.x ^= v[r][k].x;
        acc.y ^= v[r][k].y;
        acc.z ^= v[r][k].z;
        acc.w ^= v[r][k].w;
      }
  if ((acc.x & 0xfffff) == 0x12345) out[t & 1023] = acc;
}

template <int W>
static int run(int64_t points, int64_t nrec, const uint4* buf, const uint4* stream, uint4* out) {
  const int64_t nstream = points * 4;   // 64 B of streamed point data per point
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 g((unsigned)((nstream + 255) / 256)), blk(256);
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL(k_probe<W>, g, blk, 0, 0, buf, nrec, 0, stream, nstream, (uint64_t)w, out);
  // the gathers: points threads x 3 records
  const dim3 gp((unsigned)((points + 255) / 256));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_probe<W>, gp, blk, 0, 0, buf, nrec, 3, stream, points, 17ull + w, out);
  CK(hipEventRecord(a));
  const int reps = 10;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL(k_probe<W>, gp, blk, 0, 0, buf, nrec, 3, stream, points, 100ull + w, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / reps;
  const double bytes = (double)points * (3.0 * W * 16 + 16);
  std::printf("record %3d B  working set %7.1f MB  %8.1f us per pass  %7.1f GB/s (gathers + 16 B/point stream)\n", W * 16,
              (double)nrec * W * 16 / 1e6, us, bytes / us / 1e3);
  return 0;
}

int main() {
  const int64_t points = 1000000;
  const size_t maxb = (size_t)1 << 30;
  uint4 *buf, *stream, *out;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&stream, (size_t)points * 4 * 16));
  CK(hipMalloc(&out, 1024 * 16));
  CK(hipMemset(buf, 1, maxb));
  CK(hipMemset(stream, 2, (size_t)points * 4 * 16));
  for (double mb : {48.0, 96.0, 144.0, 192.0, 256.0, 384.0, 1024.0}) {
    if (run<2>(points, (int64_t)(mb * 1e6 / 32), buf, stream, out)) return 1;
    if (run<3>(points, (int64_t)(mb * 1e6 / 48), buf, stream, out)) return 1;
    if (run<4>(points, (int64_t)(mb * 1e6 / 64), buf, stream, out)) return 1;
  }
  return 0;
}
