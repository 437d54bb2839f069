// bce_device.hpp -- gfx950 device helpers shared by the engine's kernels.
//
// Wave64 cross-lane primitives (DPP, ds_swizzle, ds_bpermute), ballots and the
// CPython-compatible scalar helpers (min/max argument order, exact decimal rounding).
// Everything on the parity path is compiled with FP contraction OFF so that a*b+c rounds
// twice, exactly like CPython (SURVEY.md §7 hard part 2).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bce {

constexpr int kWave = 64;
constexpr unsigned kSent32 = 0xFFFFFFFFu;
constexpr unsigned long long kSent64 = 0xFFFFFFFFFFFFFFFFull;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ unsigned long long ballot(bool p) {
  return __ballot(p);
}

// Exchange with lane ^ MASK inside 32-lane halves (MASK < 32) or across halves (32).
template <int MASK>
__device__ __forceinline__ unsigned xor_shfl(unsigned v) {
  if constexpr (MASK == 1) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (MASK == 2) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (MASK < 32) {
    return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (MASK << 10));  // bitmask mode
  } else {
    return (unsigned)__shfl_xor((int)v, 32);
  }
}

__device__ __forceinline__ unsigned xor_shfl_rt(unsigned v, int m) {
  switch (m) {
    case 1: return xor_shfl<1>(v);
    case 2: return xor_shfl<2>(v);
    case 4: return xor_shfl<4>(v);
    case 8: return xor_shfl<8>(v);
    case 16: return xor_shfl<16>(v);
    default: return xor_shfl<32>(v);
  }
}

// lane-1 across the whole wave (DPP wave_shr:1); lane 0 reads `fill`.
__device__ __forceinline__ int wave_shr1(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xF, 0xF, false);
}

// Pull from an arbitrary lane (ds_bpermute).
__device__ __forceinline__ int pull_i32(int v, int src_lane) {
  return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}
__device__ __forceinline__ double pull_f64(double v, int src_lane) {
  int2 x = *reinterpret_cast<int2*>(&v);
  int2 y;
  y.x = __builtin_amdgcn_ds_bpermute(src_lane << 2, x.x);
  y.y = __builtin_amdgcn_ds_bpermute(src_lane << 2, x.y);
  return *reinterpret_cast<double*>(&y);
}
// Push to an arbitrary lane (ds_permute): lane `dst` receives v.
__device__ __forceinline__ int push_i32(int v, int dst_lane) {
  return __builtin_amdgcn_ds_permute(dst_lane << 2, v);
}

// Bitonic sort (ascending) of one 32-bit key per lane inside aligned G-lane segments.
template <int G>
__device__ __forceinline__ unsigned bitonic_sort_seg(unsigned key, int l) {
#pragma unroll
  for (int k = 2; k <= G; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const unsigned other = xor_shfl_rt(key, j);
      const bool up = (l & k) == 0;
      const bool lower = (l & j) == 0;
      const unsigned mn = key < other ? key : other;
      const unsigned mx = key < other ? other : key;
      key = (lower == up) ? mn : mx;
    }
  }
  return key;
}

// CPython builtin min(a, b) / max(a, b): the second argument wins only on strict < / >.
__device__ __forceinline__ double py_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double py_max(double a, double b) { return (b > a) ? b : a; }

// k integer-valued: k * 0.5 is exact, and an integer exactly when k is even (every double
// >= 2^53 is an even integer) -- fmod(k, 2.0) == 0.0 without ocml's fmod loop
__device__ __forceinline__ bool is_even(double k) { return rint(k * 0.5) == k * 0.5; }

// CPython round(x, nd) for 0 <= nd <= 22 (10^nd exact): the correctly rounded decimal (half-even on
// the exact binary value) converted back to the nearest double.  x*10^nd is split
// exactly (hi + lo via the fma error term), the nearest integer k of hi+lo is found with
// ties-to-even, and k/10^nd is one IEEE division (k < 2^53 is exact) == strtod of the
// nd-digit decimal string.  For |x| >= thresh (= 2^E with ulp(x) > 10^-nd) rounding
// moves x by less than half an ulp, so the answer is x itself (also NaN / inf).
__device__ __forceinline__ double py_round_nd(double x, double scale, double thresh) {
  if (!(fabs(x) < thresh)) return x;
  const double hi = x * scale;
  const double lo = __builtin_fma(x, scale, -hi);  // exact error of the product
  const double k0 = rint(hi);
  const double d = hi - k0;  // exact
  double k = k0;
  if (d == 0.5 || d == -0.5) {
    if (lo != 0.0) k = ((d > 0.0) == (lo > 0.0)) ? k0 + (d > 0.0 ? 1.0 : -1.0) : k0;
  } else if (d == 0.0 && (lo == 0.5 || lo == -0.5)) {
    const double k1 = k0 + (lo > 0.0 ? 1.0 : -1.0);
    k = is_even(k0) ? k0 : k1;
  }
  double r = k / scale;
  if (r == 0.0) r = copysign(0.0, x);
  return r;
}

// py_round_nd as selects (no divergent branches in an unrolled loop), and the division by
// 10^nd as q = RN(k * rinv) with one FMA correction, rinv = RN(10^-nd): k is an integer
// below 2^53 and 10^nd <= 10^22, so the residual k - q*10^nd is exact and RN(q + r*rinv) is
// the correctly rounded k / 10^nd (Markstein's theorem; checked against IEEE division by
// tools/check_markstein.c over every nd in 0..22).
__device__ __forceinline__ double py_round_nd_sel(double x, double scale, double rinv, double thresh) {
  const double hi = x * scale;
  const double lo = __builtin_fma(x, scale, -hi);
  const double k0 = rint(hi);
  const double d = hi - k0;
  const bool dhalf = (d == 0.5) | (d == -0.5);
  const bool up1 = dhalf & (lo != 0.0) & ((d > 0.0) == (lo > 0.0));
  const bool up2 = (d == 0.0) & ((lo == 0.5) | (lo == -0.5)) & !is_even(k0);
  const double step = (up1 ? (d > 0.0) : (lo > 0.0)) ? 1.0 : -1.0;
  const double k = (up1 | up2) ? k0 + step : k0;
  const double q = k * rinv;
  double r = __builtin_fma(__builtin_fma(-q, scale, k), rinv, q);
  r = (r == 0.0) ? copysign(0.0, x) : r;
  return (fabs(x) < thresh) ? r : x;
}

// py_round_nd_sel without its tie analysis: k = rint(x * 10^nd) is the answer unless the
// product sits exactly on a half (|d| == 0.5) or is an integer with |lo| == 0.5 -- then
// `slow` is set and the caller reruns py_round_nd_sel for that lane.
__device__ __forceinline__ double py_round_nd_fast(double x, double scale, double rinv, double thresh, bool& slow) {
  const double hi = x * scale;
  const double lo = __builtin_fma(x, scale, -hi);
  const double k = rint(hi);
  const double d = hi - k;
  const bool in = fabs(x) < thresh;
  // int operands: branch-free, and no -Wbitwise-instead-of-logical on bools
  slow = ((int)in & ((int)(fabs(d) == 0.5) | ((int)(d == 0.0) & (int)(fabs(lo) == 0.5)))) != 0;
  const double q = k * rinv;
  double r = __builtin_fma(__builtin_fma(-q, scale, k), rinv, q);
  r = (r == 0.0) ? copysign(0.0, x) : r;
  return in ? r : x;
}

// CPython round(x, nd) for -15 <= nd < 0 (P = 10^-nd, exact): the correctly rounded
// (half-even) multiple of P, converted back with one rounding.  k0 = rint(x / P) is at most
// one off; the remainder r = x - k0 * P is exact under the FMA (|r| <= |x| with x's
// granularity, or an integer < 2^53 for integer-valued x), so |r| against P / 2 decides k
// exactly.  For |x| >= 2^53 * P the nearest multiple is within ulp(x) / 4: the answer is x.
__device__ __forceinline__ double py_round_neg(double x, double P) {
  if (!(fabs(x) < 9007199254740992.0 * P)) return x;  // also NaN / inf
  const double k0 = rint(x / P);
  const double r = __builtin_fma(-k0, P, x);  // exact
  const double h = 0.5 * P;
  double k = k0;
  if (fabs(r) > h) {
    k = k0 + (r > 0.0 ? 1.0 : -1.0);
  } else if (fabs(r) == h) {
    const double k1 = k0 + (r > 0.0 ? 1.0 : -1.0);
    k = is_even(k0) ? k0 : k1;
  }
  double out = k * P;
  if (out == 0.0) out = copysign(0.0, x);
  return out;
}

__device__ __forceinline__ double py_round6(double x) {
  return py_round_nd(x, 1e6, 8589934592.0 /* 2^33 */);
}

}  // namespace bce
