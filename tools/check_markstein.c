// check_markstein.c -- the FULL tie-break kernel divides an integer k (|k| < 2^53) by
// 10^nd (nd in 0..22) as q = RN(k * rinv), r = fma(-q, 10^nd, k), RN(q + r * rinv) with
// rinv = RN(10^-nd) (bce_device.hpp py_round_nd_sel).  This compares that against the IEEE
// quotient k / 10^nd for every nd: all k below 2^20, and 2e7 random k per nd drawn with
// a log-uniform magnitude up to 2^53 (plus k near 2^53 and near multiples of 10^nd); and the
// group means a / c, c in 1..32, the same way with rinv = RN(1 / c).
//   gcc -O2 -ffp-contract=off -o /tmp/check_markstein tools/check_markstein.c -lm && /tmp/check_markstein
// An optional argument scales the random sample counts down (tests/test_host_logic.py runs
// it with 100: ~31M quotients in a few seconds).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

static long bad = 0, tried = 0;
static void one(double k, double s, double rinv) {
  const double q0 = k * rinv;
  const double q = fma(fma(-q0, s, k), rinv, q0);
  const double ref = k / s;
  ++tried;
  if (q != ref) {
    if (bad < 10) printf("MISMATCH k=%.17g s=%.17g q=%.17g ref=%.17g\n", k, s, q, ref);
    ++bad;
  }
}

int main(int argc, char** argv) {
  const long scale = argc > 1 ? atol(argv[1]) : 1;
  for (int nd = 0; nd <= 22; ++nd) {
    double s = 1.0;
    for (int i = 0; i < nd; ++i) s *= 10.0;
    const double rinv = 1.0 / s;
    for (int64_t k = 0; k < (1 << 20); ++k) {
      one((double)k, s, rinv);
      one(-(double)k, s, rinv);
    }
    for (long i = 0; i < 20000000 / scale; ++i) {
      const int bits = 1 + (int)(next() % 53);
      const uint64_t k = next() >> (64 - bits);
      one((double)k, s, rinv);
    }
    for (int64_t j = 0; j < 100000 / scale; ++j) {
      one(9007199254740991.0 - (double)j, s, rinv);
      const double m = floor((double)(next() >> 11) / s) * s;  // a multiple of 10^nd below 2^53
      if (m + 1 < 9007199254740992.0) {
        one(m, s, rinv);
        one(m + 1, s, rinv);
        if (m >= 1) one(m - 1, s, rinv);
      }
    }
  }
  // the FULL kernel's group means: a / c for c in 1..32 with a in [2^-1000, 2^1000] (the
  // kernel divides outside that range), rinv = RN(1 / c)
  for (int c = 1; c <= 32; ++c) {
    const double b = (double)c, rinv = 1.0 / b;
    for (long i = 0; i < 20000000 / scale; ++i) {
      const uint64_t r = next();
      const int e = (int)(r % 2000) - 1000;                              // exponent in [-1000, 1000)
      const double m = 1.0 + (double)(next() >> 12) * 0x1p-52;          // random significand
      one(ldexp(m, e), b, rinv);
      const double q = ldexp(1.0 + (double)(next() >> 12) * 0x1p-52, (int)(r % 40) - 20);
      const double a0 = q * b;                                           // near-exact multiples
      one(a0, b, rinv);
      one(nextafter(a0, 0.0), b, rinv);
      one(nextafter(a0, 1e300), b, rinv);
    }
    for (int k = 1; k < (1 << 16); ++k) one((double)k, b, rinv);         // small integer sums
  }
  printf("%ld of %ld quotients differ from IEEE division\n", bad, tried);
  return bad != 0;
}
