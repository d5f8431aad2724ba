// Bitwise comparison of glibc_math.hpp's exp/log replicas with the host libm
// (tests/test_host_logic.py builds and runs this with g++).
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../split_and_merge_gibbs_sampling_amd/csrc/glibc_math.hpp"

using hdpm::glibc::asd;
using hdpm::glibc::asu;

static bool same(double a, double b) { return asu(a) == asu(b) || (a != a && b != b); }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(12345);
  long bad_exp = 0, bad_log = 0, cnt = 0;
  auto check = [&](double x) {
    ++cnt;
    const double e0 = std::exp(x), e1 = hdpm::glibc::exp_h(x);
    if (!same(e0, e1)) {
      if (bad_exp++ < 5) printf("exp(%a): libm %a replica %a\n", x, e0, e1);
    }
    const double e2 = hdpm::glibc::exp_bf(x, hdpm::glibc::kGlibcExpTab);   // the branch-free variant
    if (!same(e0, e2)) {
      if (bad_exp++ < 5) printf("exp(%a): libm %a branch-free %a\n", x, e0, e2);
    }
    const double l0 = std::log(x), l1 = hdpm::glibc::log_h(x);
    if (!same(l0, l1)) {
      if (bad_log++ < 5) printf("log(%a): libm %a replica %a\n", x, l0, l1);
    }
  };
  // special values
  const double sp[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, 0x1p-1074, 0x1p-1022, 0x1.fffffffffffffp1023,
                       709.78, 709.79, -745.1, -745.2, -708.5, 512.0, -512.0, 1023.9, -1023.9, 0x1p-55, -0x1p-60,
                       0.9375, 1.03515625, 0x1.09p0, 0x1.ep-1};
  for (double x : sp) check(x);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (long i = 0; i < n; ++i) {
    // uniforms and the argument shapes of the pool generator
    const double u = U(g);
    check(u);
    check(u / (1.0 - u));
    check(-40.0 + 80.0 * U(g));
    check(0.9 + 0.2 * U(g));           // log's near-1 path
    check(1.0 + (U(g) - 0.5) * 1e-6);
    // random bit patterns over all finite exponents
    const uint64_t b = g();
    check(asd(b & 0x7fffffffffffffffull) < INFINITY ? asd(b & 0x7fffffffffffffffull) : 1.5);
    check(asd((b & 0x800fffffffffffffull) | ((uint64_t)(0x3c0 + (b >> 60) * 6) << 52)));   // |x| in 2^-63..2^26
    check(-700.0 + 1400.0 * U(g));     // exp's special-case band
    check(-1100.0 + 1100.0 * U(g));    // fp_draw's arguments v - max <= 0, subnormal results
    check(-(512.0 + 512.0 * U(g)));
  }
  printf("checked %ld inputs: %ld exp mismatches, %ld log mismatches\n", cnt, bad_exp, bad_log);
  return (bad_exp || bad_log) ? 1 : 0;
}
