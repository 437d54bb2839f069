// glibc_pow.hpp -- pow(x, 2.0) and pow(2.0, y) exactly as glibc 2.35's libm computes them on
// x86_64: the tie-break variance (reference tiebreak.py:110: `(c - mean_conf) ** 2` is
// CPython float_pow -> libm pow) and the decay factor (decay.py:58: `2.0 ** exponent`).  Third-party algorithm: glibc 2.35 sysdeps/ieee754/dbl-64/e_pow.c
// (ARM optimized-routines pow: table-driven log_inline with a ~2^-68 tail, then exp_inline),
// which is NOT correctly rounded -- pow(d, 2.0) differs from d*d for ~0.08% of random d and
// ~18% of exact-midpoint squares -- so d*d cannot stand in for it.
//
// Restated here, not linked: the constants come from the system libm
// (tools/gen_pow_tables.py -> glibc_pow_tables.inc), and every a*b+c the FMA build of the
// library fuses (x86_64 multiarch __pow_fma: __FP_FAST_FMA, GCC contraction, which never
// fuses a product used in two basic blocks) is an explicit fma here; everything else is
// unfused (the library builds with -ffp-contract=off).  Checked bit for bit against libm on
// 8e7 inputs incl. subnormal, tiny, huge and exact-midpoint squares (tools/pow2_check.c via
// tests/test_host_logic.py::test_glibc_pow2_restatement_matches_libm).
#pragma once
#include <stdint.h>

#ifndef BCE_POW_HOST_TEST
#include <hip/hip_runtime.h>
#define BCE_POW_FN __device__ __forceinline__
#else
#define BCE_POW_FN static inline
#define __device__
#define __constant__
#endif

#include "glibc_pow_tables.inc"

namespace bce_pow {
#pragma clang fp contract(off)

BCE_POW_FN uint64_t asu(double x) { return __builtin_bit_cast(uint64_t, x); }
BCE_POW_FN double asd(uint64_t u) { return __builtin_bit_cast(double, u); }
BCE_POW_FN uint32_t top12(double x) { return (uint32_t)(asu(x) >> 52); }

// log(x) = y + tail for the bit pattern ix (subnormals pre-normalised), e_pow.c log_inline
BCE_POW_FN double log_inline(uint64_t ix, double* tail) {
  const uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> (52 - 7)) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = asd(iz), kd = (double)k;
  const double invc = kPowLogTab[i][0], logc = kPowLogTab[i][1], logctail = kPowLogTab[i][2];
  const double r = __builtin_fma(z, invc, -1.0);
  const double t1 = __builtin_fma(kd, BCE_POW_LN2HI, logc);
  const double t2 = t1 + r;
  const double lo1 = __builtin_fma(kd, BCE_POW_LN2LO, logctail);
  const double lo2 = t1 - t2 + r;
  const double ar = kPowPoly[0] * r, ar2 = r * ar, ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = __builtin_fma(ar, r, -ar2);
  const double lo4 = t2 - hi + ar2;
  const double q3 = __builtin_fma(r, kPowPoly[6], kPowPoly[5]);
  const double q2 = __builtin_fma(ar2, q3, __builtin_fma(r, kPowPoly[4], kPowPoly[3]));
  const double q1 = __builtin_fma(ar2, q2, __builtin_fma(r, kPowPoly[2], kPowPoly[1]));
  const double lo = __builtin_fma(ar3, q1, lo1 + lo2 + lo3 + lo4);
  const double y = hi + lo;
  *tail = hi - y + lo;
  return y;
}

// e_pow.c specialcase: results near overflow / underflow (|x| of exp >= 512)
BCE_POW_FN double specialcase(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {
    sbits -= 1009ull << 52;
    const double scale = asd(sbits);
    return 0x1p1009 * __builtin_fma(scale, tmp, scale);
  }
  sbits += 1022ull << 52;
  const double scale = asd(sbits);
  const double st = scale * tmp;  // used in two blocks: the library does not fuse it
  double y = scale + st;
  if (__builtin_fabs(y) < 1.0) {
    const double one = (y < 0.0) ? -1.0 : 1.0;
    double lo = scale - y + st;
    const double hi = one + y;
    lo = one - hi + y + lo;
    y = (hi + lo) - one;
    if (y == 0) y = asd(sbits & 0x8000000000000000ull);
  }
  return 0x1p-1022 * y;
}

// exp(x + xtail), e_pow.c exp_inline with sign_bias 0 (the square is never negative)
BCE_POW_FN double exp_inline(double x, double xtail, const unsigned long long* tab = kExpTab) {
  uint32_t abstop = top12(x) & 0x7ff;
  if (abstop - top12(0x1p-54) >= top12(512.0) - top12(0x1p-54)) {
    if (abstop - top12(0x1p-54) >= 0x80000000u) return 1.0 + x;
    if (abstop >= top12(1024.0)) return (asu(x) >> 63) ? 0.0 : __builtin_inf();
    abstop = 0;
  }
  double kd = __builtin_fma(BCE_EXP_INVLN2N, x, BCE_EXP_SHIFT);
  const uint64_t ki = asu(kd);
  kd -= BCE_EXP_SHIFT;
  double r = __builtin_fma(kd, BCE_EXP_NEGLN2LON, __builtin_fma(kd, BCE_EXP_NEGLN2HIN, x));
  r += xtail;
  const uint64_t idx = 2 * (ki & 127);
  const uint64_t top = ki << (52 - 7);
  const double tail = asd(tab[idx]);
  const uint64_t sbits = tab[idx + 1] + top;
  const double r2 = r * r;
  const double tmp = __builtin_fma(r2 * r2, __builtin_fma(r, BCE_EXP_C5, BCE_EXP_C4),
                                   __builtin_fma(r2, __builtin_fma(r, BCE_EXP_C3, BCE_EXP_C2), tail + r));
  if (abstop == 0) return specialcase(tmp, sbits, ki);
  const double scale = asd(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// pow(x, 2.0) as glibc 2.35 (x86_64, FMA build) returns it, for every double x.
// Fast path: the library's result is within 0.52 ulp of the exact square (its documented
// bound; the approximation error is ~2^-64 relative), so when the exact square's rounding
// error lo = fma(x, x, -hi) is below 0.4 ulp of hi = x*x -- and hi is a normal number that is
// not a power of two (uniform spacing on both sides) -- hi is the only double within reach
// and pow returns it.  Only ~0.1% of inputs (near-midpoint squares, tiny or huge results)
// take the restated algorithm below; tools/pow2_check.cpp checks both paths against libm.
BCE_POW_FN double pow2_full(double x);
// x*x and ok = true when it is libm's pow(x, 2.0) (the case above); ok = false otherwise.
BCE_POW_FN double pow2_fast(double x, bool& ok) {
  const double hi = x * x;
  const double lo = __builtin_fma(x, x, -hi);
  const uint64_t b = asu(hi);
  ok = false;
  if (hi >= 0x1p-1000 && hi < 0x1p1000 && (b & 0xFFFFFFFFFFFFFull) != 0) {
    const double ulp = asd(b + 1) - hi;
    ok = __builtin_fabs(lo) < 0.4 * ulp;
  }
  return hi;
}
BCE_POW_FN double pow2(double x) {
  bool ok;
  const double hi = pow2_fast(x, ok);
  return ok ? hi : pow2_full(x);
}

BCE_POW_FN double pow2_full(double x) {
  uint64_t ix = asu(x);
  uint32_t topx = top12(x);
  if (topx - 0x001 >= 0x7ff - 0x001) {  // x <= 0, subnormal, inf or nan
    if (2 * ix - 1 >= 2 * asu(__builtin_inf()) - 1) return x * x;  // +-0, +-inf, nan
    if (ix >> 63) {  // y = 2 is an even integer: pow(-x, 2) = pow(x, 2)
      ix &= 0x7fffffffffffffffull;
      topx &= 0x7ff;
    }
    if (topx == 0) {  // subnormal: normalise with the exponent going negative
      ix = asu(x * 0x1p52);
      ix &= 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  double lo;
  const double hi = log_inline(ix, &lo);
  const double ehi = 2.0 * hi;
  const double elo = __builtin_fma(2.0, lo, __builtin_fma(2.0, hi, -ehi));
  return exp_inline(ehi, elo);
}

// pow(2.0, y) as glibc 2.35 returns it (decay.py:58 `2.0 ** exponent`): log_inline(2.0) is
// a constant pair (glibc_pow_tables.inc), so only the exp half runs.  CPython's float_pow
// answers y == 0 (1.0) and NaN y (NaN) itself; the rest follows e_pow.c's special cases for
// x = 2 (|y| < 2^-65: 1 + y; |y| >= 2^63: inf / 0; y = +-inf: inf / 0).
// tab: kExpTab or a copy of it (a kernel may stage the 2 KB in LDS: one ds_read per lookup
// instead of a per-lane gather from the constant table)
BCE_POW_FN double pow_base2(double y, const unsigned long long* tab = kExpTab) {
  const uint64_t iy = asu(y);
  const uint32_t topy = top12(y) & 0x7ff;
  if (topy - 0x3be >= 0x43e - 0x3be) {
    if (2 * iy - 1 >= 2 * asu(__builtin_inf()) - 1) {  // +-0, +-inf, nan
      if (2 * iy == 0) return 1.0;
      if (2 * iy > 2 * asu(__builtin_inf())) return 2.0 + y;  // nan
      return (iy >> 63) ? 0.0 : y * y;
    }
    if (topy < 0x3be) return 1.0 + y;
    return (iy >> 63) ? 0.0 : __builtin_inf();
  }
  const double ehi = y * BCE_POW_LOG2_HI;
  const double elo = __builtin_fma(y, BCE_POW_LOG2_LO, __builtin_fma(y, BCE_POW_LOG2_HI, -ehi));
  return exp_inline(ehi, elo, tab);
}

}  // namespace bce_pow
