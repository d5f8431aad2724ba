// glibc_math.hpp -- the host libm's exp and log, operation for operation, on host and device.
//
// Every draw of the latent pool (code/launcher.cpp:74-77, 124-128) and every rbeta attempt
// behind it goes through exp/log (nmath rbeta, code/hyperg.cpp:346-378, dhamming
// code/common_functions.cpp:355-377).  The reference gets them from glibc; for the device
// pool generator to produce the same bits it runs the same algorithms with the same
// tables: glibc 2.35 sysdeps/ieee754/dbl-64/e_exp.c and e_log.c as built for x86-64 hosts
// with AVX2 + FMA (the ifunc variants __exp_fma / __log_fma).  The operation order, and
// which products are fused, follow that machine code exactly; the tables come from the
// system libm (tools/gen_glibc_tables.py -> glibc_tables.inc).  Special inputs (zero,
// negative, subnormal, infinite, NaN; |x| >= 512 for exp) take glibc's special paths too;
// only NaN payloads may differ.
//
// Correctness is checked against libm itself (tests/cpp/glibc_math_test.cpp, and at
// context creation by Ctx::glibc_selfcheck, which disables the device generator on a
// host whose libm differs).
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define HDPM_HD __host__ __device__
#else
#define HDPM_HD
#endif

namespace hdpm {
namespace glibc {

#define HDPM_GLIBC_TABLE static const
#include "glibc_tables.inc"
#undef HDPM_GLIBC_TABLE

HDPM_HD inline double asd(uint64_t u) { return __builtin_bit_cast(double, u); }
HDPM_HD inline uint64_t asu(double d) { return __builtin_bit_cast(uint64_t, d); }

// e_exp.c specialcase(): |x| in [512, 1024), where 2^k may leave the normal range.
HDPM_HD inline double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000u) == 0) {
    const double scale = asd(sbits - (1009ull << 52));
    return __builtin_fma(scale, tmp, scale) * 0x1p1009;
  }
  const double scale = asd(sbits + (1022ull << 52));
  const double st = tmp * scale;
  double y = scale + st;
  if (1.0 > y) {
    const double hi = y + 1.0;
    double lo = scale - y;
    lo = lo + st;
    double y2 = (1.0 - hi) + y;
    y2 = y2 + lo;
    y2 = y2 + hi;
    y2 = y2 - 1.0;
    if (y2 == 0.0) y2 = 0.0;
    y = y2;
  }
  return y * 0x1p-1022;
}

// exp(x); T = kGlibcExpTab or a copy of it (LDS on the device)
HDPM_HD inline double exp_r(double x, const uint64_t* T) {
  const uint64_t ix = asu(x);
  const uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
  bool special = false;
  if (abstop - 0x3c9u > 0x3eu) {
    if ((int)(abstop - 0x3c9u) < 0) return x + 1.0;          // |x| < 2^-54
    if (abstop >= 0x409u) {                                   // |x| >= 1024, inf, nan
      if (ix == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ffu) return x + 1.0;
      return (ix >> 63) ? 0.0 : __builtin_inf();
    }
    special = true;
  }
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
  if (special) return exp_special(tmp, sbits, ki);
  const double scale = asd(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// exp_r without branches: every path of exp_r evaluated (the main path's table index is
// masked, so any input is safe) and the result selected, with the same operations on the
// selected path -- straight-line code, so unrolled callers issue their table loads together
// (k_resolve_fp's per-lane draws).  Same bits as exp_r for every input.
HDPM_HD inline double exp_bf(double x, const uint64_t* T) {
  const uint64_t ix = asu(x);
  const uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
  const bool out = abstop - 0x3c9u > 0x3eu;
  const bool tiny = out && (int)(abstop - 0x3c9u) < 0;
  const bool huge = out && !tiny && abstop >= 0x409u;
  const bool special = out && !tiny && !huge;
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
  const double r_main = __builtin_fma(scale, tmp, scale);
  // exp_special, both branches
  const double sc1 = asd(sbits - (1009ull << 52));
  const double r_hi = __builtin_fma(sc1, tmp, sc1) * 0x1p1009;
  const double sc2 = asd(sbits + (1022ull << 52));
  const double st = tmp * sc2;
  const double y = sc2 + st;
  const double hi = y + 1.0;
  double lo = sc2 - y;
  lo = lo + st;
  double y2 = (1.0 - hi) + y;
  y2 = y2 + lo;
  y2 = y2 + hi;
  y2 = y2 - 1.0;
  y2 = y2 == 0.0 ? 0.0 : y2;
  const double r_lo = (1.0 > y ? y2 : y) * 0x1p-1022;
  const double r_sp = (ki & 0x80000000u) == 0 ? r_hi : r_lo;
  const double r_huge = ix == 0xfff0000000000000ull ? 0.0
                        : (abstop >= 0x7ffu ? x + 1.0 : ((ix >> 63) ? 0.0 : __builtin_inf()));
  return tiny ? x + 1.0 : (huge ? r_huge : (special ? r_sp : r_main));
}

// log(x); T = kGlibcLogTab ({invc, logc} x 128) or a copy of it
HDPM_HD inline double log_r(double x, const uint64_t* T) {
  uint64_t ix = asu(x);
  if (ix - 0x3fee000000000000ull <= 0x308ffffffffffull) {    // x in [0x1.ep-1, 0x1.09p0)
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
    double t2 = __builtin_fma(r, kLogB2, kLogB1);
    double t3 = __builtin_fma(r, kLogB5, kLogB4);
    const double r2 = r * r;
    const double t5 = __builtin_fma(r, kLogB8, kLogB7);
    t2 = __builtin_fma(r2, kLogB3, t2);
    t3 = __builtin_fma(r2, kLogB6, t3);
    const double r3 = r * r2;
    double t1 = __builtin_fma(r2, kLogB9, t5);
    t1 = __builtin_fma(r3, kLogB10, t1);
    t1 = __builtin_fma(t1, r3, t3);
    t1 = __builtin_fma(t1, r3, t2);
    const double w = __builtin_fma(r, 0x1p27, r);
    const double rhi = __builtin_fma(-0x1p27, r, w);        // -(2^27 r) + w, one rounding
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = __builtin_fma(rhi2, kLogB0, r);
    const double tt = r - hi;
    const double rp = r + rhi;
    double lo = __builtin_fma(rhi2, kLogB0, tt);
    const double b = kLogB0 * rlo;
    lo = __builtin_fma(b, rp, lo);
    t1 = __builtin_fma(t1, r3, lo);
    return hi + t1;
  }
  const uint32_t top = (uint32_t)(ix >> 48);
  if (top - 0x0010u > 0x7fdfu) {
    if ((ix << 1) == 0) return -__builtin_inf();               // +-0
    if (ix == 0x7ff0000000000000ull) return x;                 // +inf
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
    ix = asu(x * 0x1p52) - (52ull << 52);                       // subnormal
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const uint32_t i = (uint32_t)(tmp >> 45) & 127u;
  const int k = (int)((int64_t)tmp >> 52);
  const double z = asd(ix - (tmp & 0xfff0000000000000ull));
  const double kd = (double)k;
  const double invc = asd(T[2 * i]);
  const double logc = asd(T[2 * i + 1]);
  const double r = __builtin_fma(z, invc, -1.0);
  const double t1 = __builtin_fma(kd, kLogLn2hi, logc);
  const double p5 = __builtin_fma(r, kLogA2, kLogA1);
  const double hi = r + t1;
  const double r2 = r * r;
  double lo = t1 - hi;
  lo = lo + r;
  lo = __builtin_fma(kd, kLogLn2lo, lo);
  const double ar3 = r * r2;
  double q = __builtin_fma(r, kLogA4, kLogA3);
  lo = __builtin_fma(r2, kLogA0, lo);
  q = __builtin_fma(q, r2, p5);
  const double y = __builtin_fma(ar3, q, lo);
  return y + hi;
}

inline double exp_h(double x) { return exp_r(x, kGlibcExpTab); }
inline double log_h(double x) { return log_r(x, kGlibcLogTab); }

}  // namespace glibc
}  // namespace hdpm
