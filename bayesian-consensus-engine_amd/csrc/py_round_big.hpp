// py_round_big.hpp -- CPython round(x, ndigits) for the precisions whose 10^|ndigits| is not
// an exact double: 23 <= ndigits <= 323 and -308 <= ndigits <= -16 (tiebreak.py:54 calls
// round(prediction, self.precision) with any int precision, tiebreak.py:46-47).
//
// CPython's float.__round__ (Objects/floatobject.c, double_round) formats x with
// _Py_dg_dtoa(x, mode 3, ndigits): the decimal k * 10^-ndigits nearest to the EXACT binary
// value of x, ties to even k, and converts that string back with _Py_dg_strtod (correctly
// rounded; ERANGE with a result >= 1 raises OverflowError).  Restated here with exact integer
// arithmetic on x = m * 2^e:
//   ndigits = n > 0:  k = round_half_even(m * 5^n / 2^-(e+n))  (x itself when e + n >= 0 or
//                     when the spacing of doubles around x exceeds 10^-n), then
//                     RN(k / (5^n * 2^n)) by a long division carrying a sticky bit;
//   ndigits = -p < 0: k = round_half_even(m * 2^e / (5^p * 2^p)) (zero when |x| < 0.4*10^p,
//                     x itself when the spacing around x exceeds 10^p), then
//                     RN(k * 5^p * 2^p), overflow reported.
// Big integers are 28 little-endian 32-bit limbs (896 bits >= m * 5^323, 804 bits), so the
// same code runs on the host and the device.  This is the rare path (predictions below
// ~1e-7 at ndigits >= 23, any prediction >= 4e15 at ndigits <= -16): the tie-break kernels
// are instantiated separately for it (tiebreak.hip), keeping the ndigits = 6 path unchanged.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define BCE_HD __host__ __device__
#else
#define BCE_HD
#endif

namespace bce_round {

constexpr int kLimbs = 28;

struct Big {
  uint32_t w[kLimbs];
};

BCE_HD inline void bset(Big& a, uint64_t v) {
  for (int i = 0; i < kLimbs; ++i) a.w[i] = 0;
  a.w[0] = (uint32_t)v;
  a.w[1] = (uint32_t)(v >> 32);
}

BCE_HD inline void bmul(Big& a, uint32_t x) {
  uint64_t c = 0;
  for (int i = 0; i < kLimbs; ++i) {
    const uint64_t t = (uint64_t)a.w[i] * x + c;
    a.w[i] = (uint32_t)t;
    c = t >> 32;
  }
}

BCE_HD inline int clz32(uint32_t v) { return v ? __builtin_clz(v) : 32; }

BCE_HD inline int bbitlen(const Big& a) {
  for (int i = kLimbs - 1; i >= 0; --i)
    if (a.w[i]) return 32 * i + 32 - clz32(a.w[i]);
  return 0;
}

BCE_HD inline bool bzero(const Big& a) { return bbitlen(a) == 0; }

BCE_HD inline void bshl(Big& a, int s) {
  if (s <= 0) return;
  const int q = s >> 5, r = s & 31;
  for (int i = kLimbs - 1; i >= 0; --i) {
    const int j = i - q;
    uint32_t v = 0;
    if (j >= 0) {
      v = a.w[j] << r;
      if (r && j > 0) v |= a.w[j - 1] >> (32 - r);
    }
    a.w[i] = v;
  }
}

BCE_HD inline void bshr(Big& a, int s) {
  if (s <= 0) return;
  const int q = s >> 5, r = s & 31;
  for (int i = 0; i < kLimbs; ++i) {
    const int j = i + q;
    uint32_t v = 0;
    if (j < kLimbs) {
      v = a.w[j] >> r;
      if (r && j + 1 < kLimbs) v |= a.w[j + 1] << (32 - r);
    }
    a.w[i] = v;
  }
}

BCE_HD inline int bcmp(const Big& a, const Big& b) {
  for (int i = kLimbs - 1; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}

BCE_HD inline void bsub(Big& a, const Big& b) {  // a -= b, a >= b
  int64_t br = 0;
  for (int i = 0; i < kLimbs; ++i) {
    const int64_t t = (int64_t)a.w[i] - (int64_t)b.w[i] - br;
    br = t < 0 ? 1 : 0;
    a.w[i] = (uint32_t)(t + (br << 32));
  }
}

BCE_HD inline void badd1(Big& a) {
  for (int i = 0; i < kLimbs; ++i)
    if (++a.w[i] != 0) return;
}

BCE_HD inline bool bbit(const Big& a, int i) { return i >= 0 && i < 32 * kLimbs && ((a.w[i >> 5] >> (i & 31)) & 1u); }

// any bit below position i set
BCE_HD inline bool bany_below(const Big& a, int i) {
  if (i <= 0) return false;
  const int q = (i < 32 * kLimbs ? i : 32 * kLimbs) >> 5, r = i & 31;
  for (int k = 0; k < q; ++k)
    if (a.w[k]) return true;
  return (q < kLimbs && r) ? (a.w[q] & ((1u << r) - 1u)) != 0 : false;
}

// 64 bits of a starting at bit lo
BCE_HD inline uint64_t bbits64(const Big& a, int lo) {
  uint64_t v = 0;
  for (int k = 0; k < 64; ++k)
    if (bbit(a, lo + k)) v |= 1ull << k;
  return v;
}

BCE_HD inline void bpow5(Big& a, int n) {  // a = 5^n
  bset(a, 1);
  for (; n >= 13; n -= 13) bmul(a, 1220703125u);  // 5^13
  uint32_t r = 1;
  for (; n > 0; --n) r *= 5u;
  bmul(a, r);
}

BCE_HD inline void bmul64(Big& a, uint64_t v) {  // a *= v (v < 2^64)
  Big hi = a;
  bmul(a, (uint32_t)v);
  bmul(hi, (uint32_t)(v >> 32));
  bshl(hi, 32);
  uint64_t c = 0;
  for (int i = 0; i < kLimbs; ++i) {
    const uint64_t t = (uint64_t)a.w[i] + hi.w[i] + c;
    a.w[i] = (uint32_t)t;
    c = t >> 32;
  }
}

// q = floor(N / D) (q < 2^64 by the caller's sizing), N := N mod D.  Restoring division.
BCE_HD inline uint64_t bdiv(Big& N, Big D) {
  const int sh = bbitlen(N) - bbitlen(D);
  if (sh < 0) return 0;
  bshl(D, sh);
  uint64_t q = 0;
  for (int i = sh; i >= 0; --i) {
    q <<= 1;
    if (bcmp(N, D) >= 0) {
      bsub(N, D);
      q |= 1;
    }
    bshr(D, 1);
  }
  return q;
}

// RN(B * 2^E2 + (a positive amount below B's last bit if sticky)) as a double, subnormals and
// overflow included (*ovf set when the result is infinite).  Requires that a sticky amount
// only ever lies below a dropped bit (callers keep >= 2 guard bits when sticky).
BCE_HD inline double bround(const Big& B, int E2, bool sticky, bool* ovf) {
  const int L = bbitlen(B);
  if (L == 0) return 0.0;
  const int top = L - 1 + E2;
  int lsb = top - 52;
  if (lsb < -1074) lsb = -1074;
  const int sh = lsb - E2;  // bits of B below the kept ones
  uint64_t mant;
  bool half = false, below = sticky;
  if (sh <= 0) {
    mant = bbits64(B, 0) << (-sh);  // B has <= 53 bits here
  } else {
    mant = (sh >= L) ? 0 : bbits64(B, sh);
    half = bbit(B, sh - 1);
    below = below || bany_below(B, sh - 1);
  }
  if (half && (below || (mant & 1ull))) ++mant;
  if (lsb + (mant ? 63 - __builtin_clzll(mant) : 0) > 1023) {
    if (ovf) *ovf = true;
    return __builtin_huge_val();
  }
  return ldexp((double)mant, lsb);
}

// |x| = m * 2^e with m < 2^53 an integer; ex = frexp exponent (|x| in [2^(ex-1), 2^ex))
BCE_HD inline void decompose(double ax, uint64_t* m, int* e, int* ex) {
  int k = 0;
  const double f = frexp(ax, &k);
  *m = (uint64_t)ldexp(f, 53);
  *e = k - 53;
  *ex = k;
}

// round(x, n) for n >= 1 (used for 23..323)
BCE_HD inline double round_pos(double x, int n) {
  if (!(x == x) || x == 0.0 || fabs(x) == __builtin_huge_val()) return x;
  const double ax = fabs(x);
  uint64_t m;
  int e, ex;
  decompose(ax, &m, &e, &ex);
  if (e + n >= 0) return x;  // x * 10^n is an integer: the decimal is x itself
  // spacing of doubles around |x| (>= 2^(ex - 54)) above 10^-n: the decimal, within
  // 0.5 * 10^-n of x, rounds back to x (margin 1 on the log2 comparison)
  if ((double)(ex - 54) + (double)n * 3.321928094887362 > 1.0) return x;
  Big B;
  bset(B, m);
  for (int r = n; r > 0;) {  // B = m * 5^n
    const int c = r >= 13 ? 13 : r;
    uint32_t f = 1;
    for (int i = 0; i < c; ++i) f *= 5u;
    bmul(B, f);
    r -= c;
  }
  const int s = -(e + n);  // > 0
  const bool half = bbit(B, s - 1);
  const bool below = bany_below(B, s - 1);
  const bool odd = bbit(B, s);
  Big K = B;
  bshr(K, s);
  if (half && (below || odd)) badd1(K);  // ties to even (dtoa mode 3)
  if (bzero(K)) return copysign(0.0, x);
  // RN(K / (5^n * 2^n)): Q = floor(K * 2^t / 5^n) with 56..57 bits, remainder as sticky
  Big D;
  bpow5(D, n);
  const int t = 56 + bbitlen(D) - bbitlen(K);
  if (t >= 0) bshl(K, t);
  else bshl(D, -t);
  const uint64_t q = bdiv(K, D);
  const bool sticky = !bzero(K);
  Big Q;
  bset(Q, q);
  const double r = bround(Q, -(t + n), sticky, nullptr);
  return copysign(r, x);
}

// round(x, -p) for p >= 1 (used for 16..308); *ovf set when CPython raises OverflowError
// ("rounded value too large to represent")
BCE_HD inline double round_neg(double x, int p, bool* ovf) {
  if (!(x == x) || x == 0.0 || fabs(x) == __builtin_huge_val()) return x;
  const double ax = fabs(x);
  uint64_t m;
  int e, ex;
  decompose(ax, &m, &e, &ex);
  // x itself when the spacing around |x| exceeds 10^p (the multiple of 10^p nearest to x is
  // within half of it)
  if ((double)(ex - 54) - (double)p * 3.321928094887362 > 1.0) return x;
  // zero when |x| < 0.4 * 10^p (nearest multiple 0; 10^p as a double is within an ulp)
  if (ax < 0.4 * pow(10.0, (double)p)) return copysign(0.0, x);
  // k = round_half_even(m * 2^e / (5^p * 2^p)) from V * 4 = m * 2^(e - p + 2) / 5^p
  const int g = 2;
  const int f = e - p + g;
  Big N, D;
  bset(N, m);
  bpow5(D, p);
  if (f >= 0) bshl(N, f);
  else bshl(D, -f);
  const uint64_t w = bdiv(N, D);  // floor(4V), N := remainder
  uint64_t k = w >> g;
  const bool half = (w >> (g - 1)) & 1ull;
  const bool below = (w & ((1ull << (g - 1)) - 1ull)) != 0 || !bzero(N);
  if (half && (below || (k & 1ull))) ++k;
  if (k == 0) return copysign(0.0, x);
  Big B;
  bpow5(B, p);
  bmul64(B, k);
  bool o = false;
  const double r = bround(B, p, false, &o);
  if (o && ovf) *ovf = true;
  return copysign(r, x);
}

}  // namespace bce_round
