// Host-side checks of csrc/rmath.hpp pieces used by the engine's update_phi pipeline:
// StreamAhead (stream generated ahead + exact state restore) and rbeta_setup/draw split.
// Built and run by tests/test_host_logic.py (no GPU needed).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../split_and_merge_gibbs_sampling_amd/csrc/rmath.hpp"

using namespace hdpm;

static int fails = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                       \
    }                                                                \
  } while (0)

static bool same(const Rng& a, const Rng& b) {
  return a.mti == b.mti && a.pos == b.pos && std::memcmp(a.mt, b.mt, sizeof(a.mt)) == 0;
}

int main() {
  // StreamAhead: values and restored states equal sequential draws, from any start
  for (int pre : {0, 1, 311, 623, 624, 625, 1300}) {
    Rng r;
    r.set_seed(20240601u);
    for (int k = 0; k < pre; ++k) (void)r.unif();
    StreamAhead sa;
    CHECK(sa.fill(r, 3000));
    sa.logits(0, sa.n);
    Rng ref = r;
    for (int c = 0; c <= 3000; c += (c < 1300 ? 1 : 97)) {
      Rng got = r;
      sa.restore(got, c);
      Rng seq = r;
      for (int k = 0; k < c; ++k) (void)seq.unif();
      CHECK(same(got, seq));
      if (c < 3000) {
        Rng one = seq;
        CHECK(sa.u[c] == one.unif());
        const double u = sa.u[c];
        CHECK(sa.lg[c] == std::log(u / (1.0 - u)));
        if (c + 1 < 3000) CHECK(sa.lz[c] == std::log(u * u * sa.u[c + 1]));
      }
    }
    // spilling past the prefix continues the live stream
    Rng live = r;
    sa.live = &live;
    sa.used = 0;
    sa.spilled = false;
    Rng seq = r;
    for (int k = 0; k < 3500; ++k) CHECK(sa.next(nullptr) == seq.unif());
    sa.finish();
    CHECK(same(live, seq));
    (void)ref;
  }
  // fill_raw: the same prefix from the tempered words of the state's block onwards (as
  // copied from a device window); states come back by untempering
  for (int pre : {1, 311, 623, 624, 1300}) {
    Rng r;
    r.set_seed(20240602u);
    for (int k = 0; k < pre; ++k) (void)r.unif();
    // the words of r's block from its start, then the next blocks (a replay from the block start)
    Rng g;
    g.set_seed(20240602u);
    const int blk_start = pre - r.mti;
    for (int k = 0; k < blk_start; ++k) (void)g.unif();
    std::vector<uint32_t> words(624 * 8);
    for (auto& w : words) w = g.raw();
    for (int i = 0; i < 624; ++i) CHECK(mt_untemper(words[i]) == r.mt[i]);
    StreamAhead sa;
    sa.fill_raw(r, words.data(), 3000);
    sa.logits(0, 1500);
    sa.logits(1500, sa.n);
    for (int c = 0; c <= 3000; c += (c < 1300 ? 1 : 97)) {
      Rng got = r;
      sa.restore(got, c);
      Rng seq = r;
      for (int k = 0; k < c; ++k) (void)seq.unif();
      CHECK(same(got, seq));
      if (c < 3000) {
        Rng one = seq;
        CHECK(sa.u[c] == one.unif());
        if (c + 1 < 3000) CHECK(sa.lz[c] == std::log(sa.u[c] * sa.u[c] * sa.u[c + 1]));
      }
    }
  }
  // the split rbeta equals the one-call form, draw for draw
  const double ps[][2] = {{0.3, 0.7}, {0.5, 5.0}, {2.0, 3.0}, {14501.0, 35501.0}, {1.0, 1.0}, {0.0, 0.0}, {3.0, 0.0}};
  for (auto& p : ps) {
    Rng a, b;
    a.set_seed(9);
    b.set_seed(9);
    StreamAhead sa;
    sa.fill(b, 5000);
    sa.logits(0, sa.n);
    sa.live = &b;
    for (int k = 0; k < 500; ++k) {
      const double x = rbeta(a, p[0], p[1]);
      const double y = rbeta_draw_s(sa, rbeta_setup(p[0], p[1]));
      CHECK(x == y || (x != x && y != y));
    }
    sa.finish();
    CHECK(same(a, b));
  }
  if (fails) {
    std::fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  std::printf("host rng ok\n");
  return 0;
}
