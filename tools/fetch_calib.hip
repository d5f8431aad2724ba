// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE on gfx950 for the prepass's access
// shapes (design tool, not part of the library): aligned random gathers of 64-B and
// 128-B records and 16-B-per-lane streaming reads, each over a 1 GiB buffer (beyond the
// Infinity Cache), with a known byte count per dispatch.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d out -o run --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

// each thread gathers R records of W uint4 at random record indices
template <int W>
__global__ void k_gather(const uint4* __restrict__ buf, int64_t nrec, int R, uint64_t seed, uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int r = 0; r < R; ++r) {
    const int64_t e = (int64_t)(mix(seed + t * 131 + r) % (uint64_t)nrec);
    const uint4* p = buf + e * W;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const uint4 v = p[k];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  if ((acc.x & 0xfffff) == 0x12345) out[t & 1023] = acc;
}

// 16-lane groups each gather R records of W 8-B words at random record indices (a lane per
// word, as k_prepass_wide reads a wide pool-entry head: 56 words = 448 B at C4)
template <int W>
__global__ void k_gather_group(const uint64_t* __restrict__ buf, int64_t nrec, int R, uint64_t seed, uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t g = t >> 4;
  const int lane = (int)(t & 15);
  uint64_t acc = 0;
  for (int r = 0; r < R; ++r) {
    const int64_t e = (int64_t)(mix(seed + g * 131 + r) % (uint64_t)nrec);
    const uint64_t* p = buf + e * W;
#pragma unroll
    for (int k = lane; k < W; k += 16) acc ^= p[k];
  }
  if ((acc & 0xfffff) == 0x12345) out[t & 1023] = make_uint4((uint32_t)acc, 0, 0, 0);
}

__global__ void k_stream(const uint4* __restrict__ buf, int64_t n16, uint4* out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = buf[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x & 0xfffff) == 0x12345) out[threadIdx.x] = acc;
}

// The prepass's own access mix, as a practical ceiling (bench.py measured_ceiling): per point a
// streamed row of W words (tiled [N/64][W][64] as the bit-sliced rows) and 16 B of draws, and
// three 64-B records gathered at random from a pool of P records (C5: 1M points, W = 4, P = 3M:
// the pool's 192 MB sit in the Infinity Cache, which the 1 GiB gathers above do not).
__global__ void k_mix64(const uint64_t* __restrict__ rows, const uint4* __restrict__ raw, const uint4* __restrict__ pool,
                        int64_t n, int W, int64_t P, uint64_t seed, uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint64_t acc = 0;
  for (int w = 0; w < W; ++w) acc ^= rows[((t >> 6) * W + w) * 64 + (t & 63)];
  const uint4 r = raw[t];
  acc ^= r.x ^ r.y;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int64_t e = (int64_t)(mix(seed + t * 7 + k) % (uint64_t)P);
    const uint4* p = pool + e * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= p[q].x ^ p[q].w;
  }
  if ((acc & 0xfffff) == 0x12345) out[t & 1023] = make_uint4((uint32_t)acc, 0, 0, 0);
}
// C4's mix (k_prepass_wide): a 16-lane group per point streams its row of W words (lane w:
// words w, w + 16, ...) and gathers three HW-word heads (448 B) from P of them (94 MB).
__global__ void k_mix448g(const uint64_t* __restrict__ rows, const uint4* __restrict__ raw,
                          const uint64_t* __restrict__ pool, int64_t n, int W, int HW, int64_t P, uint64_t seed,
                          uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t g = t >> 4;
  const int lane = (int)(t & 15);
  if (g >= n) return;
  uint64_t acc = 0;
  for (int w = lane; w < W; w += 16) acc ^= rows[((g >> 6) * W + w) * 64 + (g & 63)];
  if (lane == 0) {
    const uint4 r = raw[g];
    acc ^= r.x ^ r.y;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int64_t e = (int64_t)(mix(seed + g * 7 + k) % (uint64_t)P);
    for (int w = lane; w < HW; w += 16) acc ^= pool[e * HW + w];
  }
  if ((acc & 0xfffff) == 0x12345) out[t & 1023] = make_uint4((uint32_t)acc, 0, 0, 0);
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  uint4 *buf, *out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1024 * sizeof(uint4)) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  const int threads = 256, blocks = 4096, R = 3;
  const double nthr = (double)threads * blocks;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(threads), 0, 0, buf, (int64_t)(bytes / 64), R, 77 + rep, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("gather64  %.0f records, %.1f MB, %.1f us\n", nthr * R, nthr * R * 64 / 1e6, ms * 1e3);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_gather<8>, dim3(blocks), dim3(threads), 0, 0, buf, (int64_t)(bytes / 128), R, 91 + rep, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("gather128 %.0f records, %.1f MB, %.1f us\n", nthr * R, nthr * R * 128 / 1e6, ms * 1e3);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, buf, (int64_t)(bytes / 16 / 4), out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("stream16  %.1f MB, %.1f us\n", bytes / 4 / 1e6, ms * 1e3);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_gather_group<56>, dim3(blocks * 4), dim3(threads), 0, 0, (const uint64_t*)buf,
                       (int64_t)(bytes / 448), R, 55 + rep, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("gather448g %.0f records, %.1f MB, %.1f us\n", nthr * 4 / 16 * R, nthr * 4 / 16 * R * 448 / 1e6,
                ms * 1e3);
  }
  // the prepass mixes (bytes per point: C5 32 + 16 + 3 x 64 = 240, C4 416 + 16 + 3 x 448 = 1,776)
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    const int64_t n5 = 1 << 20, P5 = 3 * n5;
    const uint64_t* rows5 = (const uint64_t*)buf;                       // 32 MB
    const uint4* raw5 = (const uint4*)((const char*)buf + (64 << 20));  // 16 MB
    const uint4* pool5 = (const uint4*)((const char*)buf + (128 << 20)); // 192 MB
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_mix64, dim3((unsigned)(n5 / 256)), dim3(256), 0, 0, rows5, raw5, pool5, n5, 4, P5, 13 + rep, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("mix64 (C5) %lld points, %.1f MB, %.1f us, %.1f GB/s\n", (long long)n5, n5 * 240 / 1e6, ms * 1e3,
                n5 * 240 / 1e6 / ms);
    const int64_t n4 = 70000, P4 = 3 * n4;
    const int W4 = 52, HW4 = 56;
    const uint64_t* rows4 = (const uint64_t*)buf;                                      // 29 MB
    const uint4* raw4 = (const uint4*)((const char*)buf + (64 << 20));
    const uint64_t* pool4 = (const uint64_t*)((const char*)buf + (128 << 20));         // 94 MB
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_mix448g, dim3((unsigned)((n4 * 16 + 255) / 256)), dim3(256), 0, 0, rows4, raw4, pool4, n4, W4,
                       HW4, P4, 29 + rep, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("mix448g (C4) %lld points, %.1f MB, %.1f us, %.1f GB/s\n", (long long)n4, n4 * 1776 / 1e6, ms * 1e3,
                n4 * 1776 / 1e6 / ms);
  }
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
