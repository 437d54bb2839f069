// pow2_check.cpp -- host check of csrc/glibc_pow.hpp against the system libm (test tooling).
//   g++ -O2 -ffp-contract=off -DBCE_POW_HOST_TEST -I<csrc> tools/pow2_check.cpp -o pow2_check -lm
//   ./pow2_check N      -> "tested=T mismatches=K d_mul_differs=D pow2_tested=.. pow2_mismatches=.. exp2_differs=.."
// Inputs per round: a difference of two U[0,1) (the tie-break's c - mean), an odd 27-28-bit
// significand scaled down (exact-midpoint squares), an arbitrary positive bit pattern
// (subnormal .. huge) and a negative tiny value (underflowing squares).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "glibc_pow.hpp"

static uint64_t s = 88172645463325252ull;
static uint64_t xr() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double U() { return (double)(xr() >> 11) * 0x1p-53; }
static uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  volatile double two = 2.0;  // keep the compiler from turning pow(x, 2) into x*x
  long tot = 0, bad = 0, dmul = 0;
  for (long i = 0; i < n; ++i) {
    double xs[4];
    xs[0] = U() - U();
    uint64_t o = (xr() & ((1ull << 27) - 1)) | (1ull << 26) | 1ull;
    if (xr() & 1) o = (((o << 1) | 1) & ((1ull << 28) - 1)) | (1ull << 27);
    xs[1] = ldexp((double)o, -(int)(xr() % 40) - 27);
    uint64_t u = xr() & 0x7fffffffffffffffull;
    memcpy(&xs[2], &u, 8);
    xs[3] = -ldexp(U(), -(int)(xr() % 1100));
    for (double x : xs) {
      if (isnan(x)) continue;
      ++tot;
      const double a = pow(x, two), b = bce_pow::pow2(x), c = bce_pow::pow2_full(x);
      if (bits(a) != bits(b) || bits(a) != bits(c)) {
        if (bad < 5) printf("x=%a libm=%a restated=%a\n", x, a, b);
        ++bad;
      }
      if (bits(a) != bits(x * x)) ++dmul;
    }
  }
  // pow(2.0, y): decay exponents -elapsed/half_life (decay.py:52-58) and arbitrary y
  long tot2 = 0, bad2 = 0, ex2 = 0;
  for (long i = 0; i < n; ++i) {
    double ys[4];
    const double hl[4] = {30.0, 7.0, 365.25, 1.0 + 100.0 * U()};
    ys[0] = -(U() * 400.0) / hl[xr() & 3];                    // elapsed days up to 400
    ys[1] = -(double)(xr() % 100000000000ull) / 1e6 / 86400.0 / 30.0;  // int-microsecond elapsed
    ys[2] = (U() - 0.5) * 2200.0;                              // over/underflow, subnormal results
    uint64_t u = xr();
    memcpy(&ys[3], &u, 8);                                     // any bit pattern
    for (double y : ys) {
      if (isnan(y)) continue;
      ++tot2;
      const double a = pow(2.0, y), b = bce_pow::pow_base2(y);
      if (bits(a) != bits(b)) {
        if (bad2 < 5) printf("y=%a libm=%a restated=%a\n", y, a, b);
        ++bad2;
      }
      if (bits(a) != bits(exp2(y))) ++ex2;
    }
  }
  printf("tested=%ld mismatches=%ld d_mul_differs=%ld pow2_tested=%ld pow2_mismatches=%ld exp2_differs=%ld\n", tot, bad,
         dmul, tot2, bad2, ex2);
  return (bad | bad2) != 0;
}
