// The stream-exact pool pipeline (csrc/pool_gen.hpp + pool_host.hpp: packed attempt
// tables, host walk, values) modelled on the host against the sequential generator
// (code/launcher.cpp:74-77: per entry D centers, then D rhig sigmas), bit for bit, and
// the position after the pool.  Built and run by tests/test_host_logic.py.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../split_and_merge_gibbs_sampling_amd/csrc/pool_host.hpp"

using namespace hdpm;

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                          \
    }                                                                   \
  } while (0)

// the segment parse (pool_parse_segments, the device's k_pool_seg* step for step) against the
// sequential walk, on the packed tables of the slice
static void check_segments(const char* name, const PoolPlan& pl, int d, const std::vector<uint32_t>& raw, int64_t P) {
  const int64_t count = (int64_t)raw.size();
  const int nc = (int)pl.cls.size();
  const int64_t nwords = (count + 127) / 128;
  std::vector<uint64_t> bm((size_t)nc * 2 * nwords, 0);
  for (int64_t p = 0; p + 1 < count; ++p)
    for (int c = 0; c < nc; ++c)
      if (pool_accept(pl.cls[c], pool_unif(raw[p]), pool_unif(raw[p + 1]), glibc::kGlibcExpTab, glibc::kGlibcLogTab))
        bm[((size_t)c * 2 + (p & 1)) * nwords + ((p >> 1) >> 6)] |= 1ull << ((p >> 1) & 63);
  PoolRuns R{(int)pl.run_cls.size(), pl.run_cls.data(), pl.run_len.data()};
  std::vector<int64_t> s0(P + 1), s1(P + 1, -7);
  const int64_t e0 = pool_parse(bm.data(), nwords, d, R, 0, 0, P, s0.data());
  s0[P] = e0;
  const PoolSegPlan sp = pool_seg_plan(pl, d, count);
  const int64_t e1 = pool_parse_segments(bm.data(), nwords, d, R, sp, P, s1.data());
  CHECK(e0 >= 0 && e1 == e0);
  CHECK(s0 == s1);
  std::printf("%s: segments B=%lld step=%d ncand=%d chunks=%lld groups=%lld %s\n", name, (long long)sp.B, sp.step,
              sp.ncand, (long long)sp.nchunks, (long long)sp.ngroups, (e1 == e0 && s0 == s1) ? "ok" : "MISMATCH");
}

static void run_case(const char* name, const std::vector<int32_t>& att, const std::vector<double>& v,
                     const std::vector<double>& w, int64_t P, int pre, uint32_t seed) {
  const int d = (int)att.size();
  PoolPlan pl = pool_plan(d, att.data(), v.data(), w.data());
  CHECK(pl.ok);
  if (!pl.ok) return;
  Rng r;
  r.set_seed(seed);
  for (int k = 0; k < pre; ++k) (void)r.unif();
  const Rng start = r;
  // sequential reference
  std::vector<uint8_t> c0((size_t)P * d);
  std::vector<double> s0((size_t)P * d);
  for (int64_t e = 0; e < P; ++e) {
    for (int j = 0; j < d; ++j) c0[e * d + j] = (uint8_t)(int)(att[j] * r.unif() + 1);
    for (int j = 0; j < d; ++j) {
      int err = 0;
      s0[e * d + j] = rhig1(r, v[j], w[j], (double)att[j], &err);
      CHECK(err == 0);
    }
  }
  const uint64_t used = r.pos - start.pos;
  // pipeline on the slice
  const int64_t count = pool_slice_len(pl, P) + 624;
  std::vector<uint32_t> raw(count);
  Rng g = start;
  for (int64_t k = 0; k < count; ++k) raw[k] = g.raw();
  std::vector<uint8_t> c1((size_t)P * d);
  std::vector<double> s1((size_t)P * d);
  const int64_t end = pool_model(pl, d, att.data(), raw.data(), count, P, c1.data(), s1.data());
  CHECK(end == (int64_t)used);
  CHECK(std::memcmp(c0.data(), c1.data(), c0.size()) == 0);
  CHECK(std::memcmp(s0.data(), s1.data(), s0.size() * 8) == 0);
  check_segments(name, pl, d, raw, P);
  std::printf("%s: P=%lld d=%d classes=%zu runs=%zu draws=%llu (%.1f per entry, estimate %.1f) %s\n", name,
              (long long)P, d, pl.cls.size(), pl.run_cls.size(), (unsigned long long)used, (double)used / P,
              pl.mean_len, end == (int64_t)used ? "ok" : "MISMATCH");
}

int main() {
  // untempering inverts R's tempering
  Rng r;
  r.set_seed(99u);
  for (int k = 0; k < 2000; ++k) {
    const uint32_t y = r.mt[k % 624] ^ (uint32_t)(k * 2654435761u);
    uint32_t t = y;
    t ^= (t >> 11);
    t ^= (t << 7) & 0x9d2c5680u;
    t ^= (t << 15) & 0xefc60000u;
    t ^= (t >> 18);
    CHECK(mt_untemper(t) == y);
  }
  // Zoo hyperparameters (zoo:36-38): two classes, three runs
  {
    std::vector<int32_t> att(16, 2);
    att[12] = 6;
    std::vector<double> v(16, 6.0), w(16, 0.25);
    v[12] = 3.0;
    w[12] = 0.5;
    for (int pre : {0, 1, 623, 624, 1000}) run_case("zoo", att, v, w, 303, pre, 42u + pre);
  }
  // odd D with an rbeta BC class (v - 1 < 1) next to BB ones
  {
    std::vector<int32_t> att{3, 3, 5, 2, 4, 4, 7};
    std::vector<double> v{1.8, 1.8, 6.0, 6.0, 3.0, 1.5, 6.0}, w{0.25, 0.25, 0.25, 0.4, 0.5, 0.3, 0.25};
    run_case("odd-bc", att, v, w, 4000, 17, 7u);
  }
  // C3-like: m_j in 2..6 per attribute, one (v, w)
  {
    std::vector<int32_t> att(64);
    for (int j = 0; j < 64; ++j) att[j] = 2 + (j * 7 + 3) % 5;
    std::vector<double> v(64, 6.0), w(64, 0.25);
    run_case("c3-like", att, v, w, 3000, 5, 11u);
  }
  // C4-like: one class, long run
  {
    std::vector<int32_t> att(784, 6);
    std::vector<double> v(784, 3.0), w(784, 0.5);
    run_case("c4-like", att, v, w, 200, 300, 13u);
  }
  // C5-like: one class, D = 128 (the bench pool's shape), enough entries for several groups
  {
    std::vector<int32_t> att(128, 4);
    std::vector<double> v(128, 6.0), w(128, 0.25);
    run_case("c5-like", att, v, w, 20000, 77, 9u);
  }
  if (fails) return 1;
  std::printf("pool pipeline ok\n");
  return 0;
}
