// consensus_wide.hip -- core.compute_consensus (core.py:63-179) for markets with
// 64 < n <= 4096 signals: one workgroup of NW waves per market, P = 64*NW*R keys.
//
// Per market (core.py:103 sorted source ids, core.py:115-116 duplicates averaged in input
// order, core.py:111-112 table lookups, core.py:119-151 weights and ordered sums):
//   1. keys (sid << IB | input index, 32 bits; needs n_sources <= 2^(32-IB)) from the sid
//      registers loaded one market ahead; the next market's sids are issued right away.
//   2. register bitonic network (flip form): stages inside a thread are min/max pairs, lane
//      exchanges are VALU only (DPP in rows, v_permlane16/32_swap across rows and halves),
//      the few stages that cross waves go through LDS rows (region B, two alternating
//      buffers: one barrier per stage).
//   3. input-order probabilities (loaded during the previous market) land in region A, are
//      range-checked (core.py:59-60), read back in sorted order into registers and written
//      over region A in place; run leaders get their unique index from a workgroup prefix
//      count and land in region B (sid << IB | first sorted position).
//   4. per unique j (thread t owns j = t + NT*i): the run's probabilities summed in input
//      order (builtin sum, core.py:116; FAST: runs longer than kWaveRun by the whole wave
//      in a fixed order), one {rel, conf} row + present bit gathered,
//      products w, avg*w, conf*w (core.py:119,136,142); usid / weight written.
//        FAST  (BCE_MODE_FAST): per-thread partial sums in round order, then a fixed
//              butterfly over the wave and a wave-ordered sum over the workgroup --
//              deterministic, within the north-star 1e-9 of the reference order.
//        EXACT: rounds of products staged through a two-slot LDS ring; wave 0 carries the
//              three left-to-right chains (core.py:120,136,142) on lanes 0..2 -- with
//              several waves it does only that, fed by the others through LDS counters
//              (no barriers), so the serial chains overlap the next rounds' gathers.
//      normalizedWeight reads w[j] back from the weight output (or, without one, from the
//      dead sorted-probability slot j where it was parked).
//   5. the next market's probabilities are issued, then per-market outputs and
//      normalizedWeight = w / total (core.py:151).
// LDS: region A = P doubles (+ read-ahead pad), region B = max(sort exchange rows,
// leaders [+ the exact chain buffers]).  FAST at P = 4096 fits three workgroups per CU.
#include <stdio.h>
#include <stdlib.h>

#include "consensus_common.hpp"

#pragma clang fp contract(off)

constexpr int kWideHR = 1;       // rounds of NT uniques whose gathers are in flight together (2: C3 fast +6%)
constexpr int kWideWPE = 4;      // min waves per SIMD (register budget; 4 vs 2: exact -1.3%, fast unchanged)
constexpr int kWideNWBF = 4;     // FAST nweight read-backs per batch (1: 1.645, 2: 1.634, 4: 1.587 ms C3)
constexpr bool kWideChainDeep = true;  // EXACT piped chain wave: chain_add_deep (16-term steps)
constexpr bool kWideChain3 = true;     // EXACT chains run on lanes 0..2 only (exec = 3 lanes)

namespace bce {
namespace {

constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
constexpr int kWaveRun = 48;  // FAST: duplicate runs longer than this are summed wave-wide

// NW waves (threads = 64*NW) hold P = 64*NW*R keys; the sort network spans NN >= NW waves
// (PN = 64*NN*R, a power of two): NN > NW is a non-power-of-two bin -- the network's
// missing waves hold +inf keys, so every exchange with them leaves the key in place and
// they are never materialised (6 waves for 2049..3072 signals, 3 for 1025..1536).
// KT: the sort key, (sid << IB) | input index -- 32 bits while n_sources <= 2^(32 - IB), else
// 64 bits (large tables, DESIGN.md §4.2 "Large source tables").
template <int NW, int R, bool FAST, int NN = NW, class KT = unsigned>
struct WideCfg {
  static constexpr int NT = 64 * NW;
  static constexpr int P = NT * R;
  static constexpr int PN = 64 * NN * R;
  static constexpr int IB = ilog2c(PN);
  static constexpr int LW = (int)(sizeof(KT) / 4);  // u32 words per key
  static constexpr int HR = (R < kWideHR) ? R : kWideHR;
  // register budget: workgroups of >= 4 waves get 4 waves per SIMD (<= 128 VGPRs), so two
  // LDS-sized workgroups share a CU
  // (the 6-wave FAST kernel at 5 waves per SIMD, <= 102 VGPRs, so three workgroups share a
  // CU: C3 fast 1.55 -> 1.72 ms from its spills, profiles/r03g/wide_ab.txt)
  static constexpr int WPE = kWideWPE;
  static constexpr int A_DBL = P + 64;  // + the run sums' read-ahead
  // region B (u32): sort exchange rows (32-bit keys: two alternating buffers of P words;
  // 64-bit keys: one buffer of P keys), then leaders [P] keys (+ exact: chain buffers
  // [2][3][NT] doubles + the chain's read-ahead)
  static constexpr int X_U32 = 2 * P;
  static constexpr int LEAD_U32 = LW * P + (FAST ? 0 : 2 * (6 * NT + 32));
  static constexpr int B_U32 = (X_U32 > LEAD_U32) ? X_U32 : LEAD_U32;
};

// 64-bit key halves through the 32-bit lane primitives
__device__ __forceinline__ unsigned k_lo(uint64_t v) { return (unsigned)v; }
__device__ __forceinline__ unsigned k_hi(uint64_t v) { return (unsigned)(v >> 32); }
__device__ __forceinline__ uint64_t k_make(unsigned hi, unsigned lo) { return ((uint64_t)hi << 32) | lo; }

// v from lane ^ M (whole wave) for the masks the flip-form sort uses -- all VALU, no LDS
// round trip: DPP for the in-row patterns, the CDNA4 half-exchanges v_permlane16_swap /
// v_permlane32_swap (plus a lane select) across rows and halves.
template <int M>
__device__ __forceinline__ unsigned lane_xor(unsigned v) {
  const int lane = lane_id();
  if constexpr (M == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  else if constexpr (M == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // 2,3,0,1
  else if constexpr (M == 3) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);  // 3,2,1,0
  else if constexpr (M == 4) {  // row_ror:N reads lane (l - N) mod 16: bit 2 set -> ror 4, clear -> ror 12
    const unsigned a = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
    const unsigned b = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);
    return (lane & 4) ? a : b;
  } else if constexpr (M == 7) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  else if constexpr (M == 8) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);    // row_ror:8
  else if constexpr (M == 15) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);   // row_mirror
  else if constexpr (M == 16) {  // odd rows <-> even rows
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else if constexpr (M == 32) {  // upper half <-> lower half
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? r[0] : r[1];
  } else if constexpr (M == 31) {  // l ^ 31 = (l ^ 16) ^ 15
    return (unsigned)__builtin_amdgcn_mov_dpp((int)lane_xor<16>(v), 0x140, 0xF, 0xF, false);
  } else if constexpr (M == 63) {  // l ^ 63 = (l ^ 32) ^ 31
    return lane_xor<31>(lane_xor<32>(v));
  } else {
    static_assert(M == 1, "unsupported lane distance");
    return v;
  }
}

template <int M>
__device__ __forceinline__ uint64_t lane_xor(uint64_t v) {
  return k_make(lane_xor<M>(k_hi(v)), lane_xor<M>(k_lo(v)));
}

// Inclusive prefix sum over the wave with DPP (GFX9 row shifts + row broadcasts).
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Index of wave-crossing stage (K, J) among the network's wave-crossing stages (they
// alternate between two exchange buffers, so each needs one barrier, not two).
constexpr int xw_index(int K, int J, int R) {
  int idx = 0;
  for (int k = 2; k < K; k <<= 1)
    for (int j = k / 2; j >= 1; j >>= 1)
      if ((j == k / 2) ? (k > 64 * R) : (j >= 64 * R)) ++idx;
  for (int j = K / 2; j > J; j >>= 1)
    if ((j == K / 2) ? (K > 64 * R) : (j >= 64 * R)) ++idx;
  return idx;
}

// One lane stage over 8 keys with the partner's key read through DPP inside the
// instructions that use it: per key v_sub_co_u32_dpp (borrow = partner < key, into VCC),
// s_xor_b64 with the stage's lower-lane mask, v_cndmask_b32_dpp (keep the key or take the
// partner's) -- two VALU per key instead of a v_mov_b32_dpp, a v_cmp and a v_cndmask (the
// compiler neither folds DPP into a compare nor into a select whose DPP operand is src1,
// and gfx950 has no VOPC DPP).  FLIP: key r's partner is key R-1-r of the partner lane.
// The outputs are early-clobber, so no instruction in the block reads a register written
// in it; `s_nop 1` covers the VALU-write -> DPP-read hazard on the inputs; the s_xor writes
// SCC, so the block clobbers it (a scalar branch condition computed before it is dead).
#define BCE_DPP_CAS(O, A, B, C)                                                  \
  "v_sub_co_u32_dpp %[j], vcc, %[" B "], %[" A "] " C " row_mask:0xf bank_mask:0xf\n" \
  "s_xor_b64 vcc, vcc, %[lm]\n"                                                  \
  "v_cndmask_b32_dpp %[" O "], %[" B "], %[" A "], vcc " C " row_mask:0xf bank_mask:0xf\n"
#define BCE_DPP_STAGE8(C, B0, B1, B2, B3, B4, B5, B6, B7)                                                       \
  asm("s_nop 1\n" BCE_DPP_CAS("o0", "k0", B0, C) BCE_DPP_CAS("o1", "k1", B1, C) BCE_DPP_CAS("o2", "k2", B2, C)    \
          BCE_DPP_CAS("o3", "k3", B3, C) BCE_DPP_CAS("o4", "k4", B4, C) BCE_DPP_CAS("o5", "k5", B5, C)           \
              BCE_DPP_CAS("o6", "k6", B6, C) BCE_DPP_CAS("o7", "k7", B7, C)                                      \
      : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]), [o4] "=&v"(o[4]),              \
        [o5] "=&v"(o[5]), [o6] "=&v"(o[6]), [o7] "=&v"(o[7]), [j] "=&v"(junk)                                  \
      : [k0] "v"(s[0]), [k1] "v"(s[1]), [k2] "v"(s[2]), [k3] "v"(s[3]), [k4] "v"(s[4]), [k5] "v"(s[5]),        \
        [k6] "v"(s[6]), [k7] "v"(s[7]), [lm] "s"(lower)                                                        \
      : "vcc", "scc")
#define BCE_DPP_STAGE8_ANY(C, FLIP)                                                   \
  do {                                                                                \
    if (FLIP)                                                                         \
      BCE_DPP_STAGE8(C, "k7", "k6", "k5", "k4", "k3", "k2", "k1", "k0");              \
    else                                                                              \
      BCE_DPP_STAGE8(C, "k0", "k1", "k2", "k3", "k4", "k5", "k6", "k7");              \
  } while (0)

// Lane bits 2 and 3 separate the two lanes of a pair by DPP bank (bank = lane bits 3..2
// of the row), so the stage needs no select at all: v_min_u32_dpp writes the lower lanes'
// banks, v_max_u32_dpp the upper lanes' (bank_mask), each reading the partner through its
// own row pattern -- two VALU per key, no compare in VCC.  CLO/BLO: the lower lanes' DPP
// pattern and banks, CHI/BHI the upper lanes'.
#define BCE_BANK_CAS(O, A, B, CLO, BLO, CHI, BHI)                                            \
  "v_min_u32_dpp %[" O "], %[" B "], %[" A "] " CLO " row_mask:0xf bank_mask:" BLO "\n"     \
  "v_max_u32_dpp %[" O "], %[" B "], %[" A "] " CHI " row_mask:0xf bank_mask:" BHI "\n"
#define BCE_BANK_STAGE8(CLO, BLO, CHI, BHI, B0, B1, B2, B3, B4, B5, B6, B7)                                   \
  asm("s_nop 1\n" BCE_BANK_CAS("o0", "k0", B0, CLO, BLO, CHI, BHI) BCE_BANK_CAS("o1", "k1", B1, CLO, BLO, CHI, BHI) \
          BCE_BANK_CAS("o2", "k2", B2, CLO, BLO, CHI, BHI) BCE_BANK_CAS("o3", "k3", B3, CLO, BLO, CHI, BHI)          \
              BCE_BANK_CAS("o4", "k4", B4, CLO, BLO, CHI, BHI) BCE_BANK_CAS("o5", "k5", B5, CLO, BLO, CHI, BHI)      \
                  BCE_BANK_CAS("o6", "k6", B6, CLO, BLO, CHI, BHI) BCE_BANK_CAS("o7", "k7", B7, CLO, BLO, CHI, BHI)  \
      : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]), [o4] "=&v"(o[4]),               \
        [o5] "=&v"(o[5]), [o6] "=&v"(o[6]), [o7] "=&v"(o[7])                                                    \
      : [k0] "v"(s[0]), [k1] "v"(s[1]), [k2] "v"(s[2]), [k3] "v"(s[3]), [k4] "v"(s[4]), [k5] "v"(s[5]),         \
        [k6] "v"(s[6]), [k7] "v"(s[7]))
#define BCE_BANK_STAGE8_ANY(CLO, BLO, CHI, BHI, FLIP)                                          \
  do {                                                                                         \
    if (FLIP)                                                                                  \
      BCE_BANK_STAGE8(CLO, BLO, CHI, BHI, "k7", "k6", "k5", "k4", "k3", "k2", "k1", "k0");     \
    else                                                                                       \
      BCE_BANK_STAGE8(CLO, BLO, CHI, BHI, "k0", "k1", "k2", "k3", "k4", "k5", "k6", "k7");     \
  } while (0)

// Lane distances the fused 8-key stage serves: lane bits 0..1 through one DPP pattern
// (quad_perm) with the compare in VCC, lane bits 2..3 (row_ror:4/12, row_ror:8,
// row_half_mirror, row_mirror) by bank.
constexpr bool dpp_fusable(int M) { return M == 1 || M == 2 || M == 3 || M == 4 || M == 7 || M == 8 || M == 15; }

template <int M, bool FLIP>
__device__ __forceinline__ void dpp_stage8(unsigned (&key)[8], uint64_t lower) {
  unsigned o[8], junk;
  const unsigned (&s)[8] = key;
  // row_ror:N reads lane (l - N) mod 16: the l ^ 4 partner is ror 12 for bit 2 clear
  // (banks 0, 2), ror 4 for bit 2 set (banks 1, 3)
  if constexpr (M == 4) BCE_BANK_STAGE8_ANY("row_ror:12", "0x5", "row_ror:4", "0xa", FLIP);
  else if constexpr (M == 8) BCE_BANK_STAGE8_ANY("row_ror:8", "0x3", "row_ror:8", "0xc", FLIP);
  else if constexpr (M == 7) BCE_BANK_STAGE8_ANY("row_half_mirror", "0x5", "row_half_mirror", "0xa", FLIP);
  else if constexpr (M == 15) BCE_BANK_STAGE8_ANY("row_mirror", "0x3", "row_mirror", "0xc", FLIP);
  else if constexpr (M == 1) BCE_DPP_STAGE8_ANY("quad_perm:[1,0,3,2]", FLIP);
  else if constexpr (M == 2) BCE_DPP_STAGE8_ANY("quad_perm:[2,3,0,1]", FLIP);
  else if constexpr (M == 3) BCE_DPP_STAGE8_ANY("quad_perm:[3,2,1,0]", FLIP);
  (void)junk;
  (void)lower;
#pragma unroll
  for (int r = 0; r < 8; ++r) key[r] = o[r];
}

// Half-cleaner across lane bit 4 or 5 (l ^ 16, l ^ 32) on pairs of keys: v_permlane16/32_swap
// of keys (a, b) leaves each lane holding both members of one pair -- a[l] and a[l ^ M] in
// the lanes with the bit clear, b[l ^ M] and b[l] in the others, the lower position always
// in the first register -- so one min/max pair does the stage for both keys, and a second
// swap puts them back.  Four VALU per two keys, no lane masks.
template <int M, int R>
__device__ __forceinline__ void swap_stage(uint64_t (&key)[R]) {  // 64-bit keys: both halves swapped
#pragma unroll
  for (int r = 0; r < R; r += 2) {
    uint64_t a, b;
    if constexpr (M == 32) {
      const auto h = __builtin_amdgcn_permlane32_swap(k_hi(key[r]), k_hi(key[r + 1]), false, false);
      const auto l = __builtin_amdgcn_permlane32_swap(k_lo(key[r]), k_lo(key[r + 1]), false, false);
      a = k_make(h[0], l[0]);
      b = k_make(h[1], l[1]);
    } else {
      const auto h = __builtin_amdgcn_permlane16_swap(k_hi(key[r]), k_hi(key[r + 1]), false, false);
      const auto l = __builtin_amdgcn_permlane16_swap(k_lo(key[r]), k_lo(key[r + 1]), false, false);
      a = k_make(h[0], l[0]);
      b = k_make(h[1], l[1]);
    }
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    if constexpr (M == 32) {
      const auto h = __builtin_amdgcn_permlane32_swap(k_hi(lo), k_hi(hi), false, false);
      const auto l = __builtin_amdgcn_permlane32_swap(k_lo(lo), k_lo(hi), false, false);
      key[r] = k_make(h[0], l[0]);
      key[r + 1] = k_make(h[1], l[1]);
    } else {
      const auto h = __builtin_amdgcn_permlane16_swap(k_hi(lo), k_hi(hi), false, false);
      const auto l = __builtin_amdgcn_permlane16_swap(k_lo(lo), k_lo(hi), false, false);
      key[r] = k_make(h[0], l[0]);
      key[r + 1] = k_make(h[1], l[1]);
    }
  }
}

template <int M, int R>
__device__ __forceinline__ void swap_stage(unsigned (&key)[R]) {
#pragma unroll
  for (int r = 0; r < R; r += 2) {
    unsigned lo, hi;
    if constexpr (M == 32) {
      const auto s1 = __builtin_amdgcn_permlane32_swap(key[r], key[r + 1], false, false);
      lo = min(s1[0], s1[1]);
      hi = max(s1[0], s1[1]);
      const auto s2 = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
      key[r] = s2[0];
      key[r + 1] = s2[1];
    } else {
      const auto s1 = __builtin_amdgcn_permlane16_swap(key[r], key[r + 1], false, false);
      lo = min(s1[0], s1[1]);
      hi = max(s1[0], s1[1]);
      const auto s2 = __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
      key[r] = s2[0];
      key[r + 1] = s2[1];
    }
  }
}

// One stage of the flip-form bitonic network over PN = 64*NN*R keys, position q = t*R + r:
// the first stage of merge K pairs q with q ^ (K-1), the others pair q with q ^ J, and the
// lower position always keeps the minimum -- no direction bits anywhere.  Threads t >= 64*NW
// (a non-power-of-two bin's missing waves) hold +inf: their partners keep their own keys.
template <int NN, int NW, int R, int K, int J, class KT>
__device__ __forceinline__ void wide_stage(KT (&key)[R], unsigned* sX, int t, int lane) {
  constexpr bool flip = (J == K / 2);
  constexpr bool K64 = sizeof(KT) == 8;
  if constexpr (flip ? (K <= R) : (J < R)) {  // inside a thread: min/max pairs
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int r2 = flip ? (r ^ (K - 1)) : (r | J);
      if (flip ? (r < r2) : ((r & J) == 0)) {
        const KT x = key[r], y = key[r2];
        key[r] = x < y ? x : y;
        key[r2] = x < y ? y : x;
      }
    }
  } else if constexpr (flip ? (K <= 64 * R) : (J < 64 * R)) {  // across lanes (never crosses a wave)
    constexpr int MK = flip ? (K / R - 1) : (J / R);
    const bool lower = (lane & (flip ? (K / R / 2) : MK)) == 0;
    if constexpr (!K64 && R == 8 && dpp_fusable(MK)) {
      dpp_stage8<MK, flip>(key, (uint64_t)ballot(lower));
      if constexpr (J > 1) wide_stage<NN, NW, R, K, J / 2>(key, sX, t, lane);
      return;
    }
    if constexpr (!flip && (MK == 16 || MK == 32)) {
      swap_stage<MK, R>(key);
      if constexpr (J > 1) wide_stage<NN, NW, R, K, J / 2>(key, sX, t, lane);
      return;
    }
    if constexpr (flip && MK == 31) {
      // the flip of merge K = 32R as a reversal of each K-block's upper half (q ^ (K/2 - 1):
      // row_mirror of key R-1-r, written in rows 1 and 3 only) and a half-cleaner on lane
      // bit 4 -- the pairs are the same; the upper half then holds its bitonic sequence
      // reversed, which the following half-cleaners sort as well (a reversed bitonic
      // sequence is bitonic), so the merge's output is the same sorted sequence
      KT nk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (K64) {
          nk[r] = k_make((unsigned)__builtin_amdgcn_update_dpp((int)k_hi(key[r]), (int)k_hi(key[R - 1 - r]), 0x140, 0xA,
                                                               0xF, false),
                         (unsigned)__builtin_amdgcn_update_dpp((int)k_lo(key[r]), (int)k_lo(key[R - 1 - r]), 0x140, 0xA,
                                                               0xF, false));
        } else {
          nk[r] = (unsigned)__builtin_amdgcn_update_dpp((int)key[r], (int)key[R - 1 - r], 0x140, 0xA, 0xF, false);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = nk[r];
      swap_stage<16, R>(key);
      if constexpr (J > 1) wide_stage<NN, NW, R, K, J / 2>(key, sX, t, lane);
      return;
    }
    KT y[R];
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = lane_xor<MK>(key[flip ? R - 1 - r : r]);
#pragma unroll
    for (int r = 0; r < R; ++r) key[r] = ((key[r] < y[r]) == lower) ? key[r] : y[r];
  } else if constexpr (K64) {  // across waves, 64-bit keys: one LDS buffer, two barriers
    constexpr int MT = flip ? (K / R - 1) : (J / R);
    const bool lower = (t & (flip ? (K / R / 2) : MT)) == 0;
    // planes of 2 keys: key r of thread t at (r/2)*NT*2 + t*2 + r%2 (16-B accesses, a wave's
    // 64 accesses consecutive)
    uint64_t* const buf = reinterpret_cast<uint64_t*>(sX);
    constexpr int PL = 2 * 64 * NW;  // keys per plane
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      uint4 v;
      v.x = k_lo(key[r]); v.y = k_hi(key[r]); v.z = k_lo(key[r + 1]); v.w = k_hi(key[r + 1]);
      *reinterpret_cast<uint4*>(buf + (r >> 1) * PL + t * 2) = v;
    }
    __syncthreads();
    uint64_t y[R];
    const bool real = NN == NW || (t ^ MT) < 64 * NW;  // partner in a missing wave: +inf
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      const uint4 v = real ? *reinterpret_cast<const uint4*>(buf + (r >> 1) * PL + (t ^ MT) * 2)
                           : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      y[r] = k_make(v.y, v.x);
      y[r + 1] = k_make(v.w, v.z);
    }
    __syncthreads();  // every read done before the next stage rewrites the buffer
    if (__builtin_amdgcn_readfirstlane((int)lower)) {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = key[r] < y[flip ? R - 1 - r : r] ? key[r] : y[flip ? R - 1 - r : r];
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = key[r] < y[flip ? R - 1 - r : r] ? y[flip ? R - 1 - r : r] : key[r];
    }
  } else {  // across waves, through LDS rows; buffers alternate, so the previous reads
            // of this buffer finished before the last stage's barrier
    constexpr int MT = flip ? (K / R - 1) : (J / R);
    unsigned* const buf = sX + (xw_index(K, J, R) & 1) * (64 * NW * R);
    const bool lower = (t & (flip ? (K / R / 2) : MT)) == 0;
    // planes of 4 keys: key r of thread t at (r/4)*NT*4 + t*4 + r%4, so every 16-B access
    // of a wave covers 1 KB of consecutive words (a thread-major row of R keys put lanes 32 B
    // apart: two lanes per bank group, a 2-way conflict on every exchange)
    constexpr int PL = 4 * 64 * NW;  // words per plane
#pragma unroll
    for (int r = 0; r < R; r += 4)
      *reinterpret_cast<uint4*>(buf + (r >> 2) * PL + t * 4) = make_uint4(key[r], key[r + 1], key[r + 2], key[r + 3]);
    __syncthreads();
    unsigned y[R];
    const bool real = NN == NW || (t ^ MT) < 64 * NW;  // partner in a missing wave: +inf
#pragma unroll
    for (int r = 0; r < R; r += 4) {
      const uint4 y4 = real ? *reinterpret_cast<const uint4*>(buf + (r >> 2) * PL + (t ^ MT) * 4)
                            : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      y[r] = y4.x;
      y[r + 1] = y4.y;
      y[r + 2] = y4.z;
      y[r + 3] = y4.w;
    }
    // `lower` is uniform over the wave here (the partner is a whole wave away): one min or
    // one max per key under a scalar branch, no compare in VCC
    if (__builtin_amdgcn_readfirstlane((int)lower)) {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = min(key[r], y[flip ? R - 1 - r : r]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) key[r] = max(key[r], y[flip ? R - 1 - r : r]);
    }
  }
  if constexpr (J > 1) wide_stage<NN, NW, R, K, J / 2>(key, sX, t, lane);
}

template <int NN, int NW, int R, int K = 2, class KT>
__device__ __forceinline__ void wide_sort(KT (&key)[R], unsigned* sX, int t, int lane) {
  wide_stage<NN, NW, R, K, K / 2>(key, sX, t, lane);
  if constexpr (K < 64 * NN * R) wide_sort<NN, NW, R, 2 * K>(key, sX, t, lane);
}

// One fixed-order sum over the wave, returned in every lane: DPP rotations inside each
// 16-lane row and quad swaps (no LDS round trips), then the four row sums in row order.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)__double_as_longlong(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)__double_as_longlong(v) >> 32), CTRL, 0xF, 0xF,
                                          false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)__double_as_longlong(v), l);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)__double_as_longlong(v) >> 32), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_fixed(double v) {
  v = v + dpp_f64<0x128>(v);  // row_ror:8
  v = v + dpp_f64<0x124>(v);  // row_ror:4
  v = v + dpp_f64<0x4E>(v);   // quad_perm 2,3,0,1
  v = v + dpp_f64<0xB1>(v);   // quad_perm 1,0,3,2
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// FAST: run averages and normalizedWeight by reciprocal products instead of IEEE divisions
// (a few ulps; FAST's contract is 1e-9 relative)
constexpr bool kWideFastRecip = true;

// builtin sum() from 0 over a run of len sorted probabilities in input order (core.py:116);
// terms past the run add +0.0, exact since the sum starts at +0.0 and is never -0.0.
// APPROX (FAST): the average as sum * (1/len) -- v_rcp_f64 refined by one Newton step.
template <int R, bool APPROX = false>
__device__ __forceinline__ double run_sum(const double* sA, int q0, int len) {
  double x[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] = sA[q0 + e];
  double sum = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) sum += (e < len) ? x[e] : 0.0;
  if (len > 4) {  // long (hot-source) run: 8 terms per step, the next 8 in flight
    int e0 = 4;
    double xa[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xa[e] = sA[q0 + e0 + e];
    for (; e0 + 8 <= len; e0 += 8) {
      double xb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) xb[e] = sA[q0 + e0 + 8 + e];
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += xa[e];
#pragma unroll
      for (int e = 0; e < 8; ++e) xa[e] = xb[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += (e0 + e < len) ? xa[e] : 0.0;
  }
  if constexpr (APPROX) {
    const double c = (double)len;
    double y = __builtin_amdgcn_rcp(c);
    y = __builtin_fma(__builtin_fma(-c, y, 1.0), y, y);
    return (len > 1) ? sum * y : sum;
  } else {
    return (len > 1) ? sum / (double)len : sum;
  }
}

// acc += src[0] + src[1] + ... + src[ce-1], left to right (the reference's chains,
// core.py:120,136,142).  Full 8-term steps run in asm: two 4-term batches in fixed
// registers, each reloaded right after its adds, so one batch's LDS latency hides under the
// other's dependent adds (the compiler would copy loop-carried batch registers behind an
// lgkmcnt(0)).  The < 8-term tail is added in C++ with masked terms adding +0.0 -- exact,
// because these chains never hold -0.0.  src is 16-B aligned; reads may run 8 past ce.
// chain_add_deep: the piped EXACT path's dedicated chain wave reads further ahead (16-term
// steps over four 4-term batches, 12 terms ahead of the adds instead of 4; 32 fixed VGPRs);
// reads may run 16 past ce (the chain ring holds 6 (NT - NP) = 384 doubles of slack past its
// last chain).
__device__ __forceinline__ void chain_tail(double& acc, const double* src, int from, int ce) {
  double xt[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) xt[e] = src[from + e];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc += (from + e < ce) ? xt[e] : 0.0;
}
__device__ __forceinline__ void chain_add(double& acc, const double* src, int ce) {
  const int nfull = ce & ~7;
  if (nfull) {
    unsigned addr = (unsigned)(uintptr_t)src;
    int steps = nfull >> 3;
    asm volatile(
        "ds_read_b128 v[112:115], %[ad] offset:0\n"
        "ds_read_b128 v[116:119], %[ad] offset:16\n"
        "ds_read_b128 v[120:123], %[ad] offset:32\n"
        "ds_read_b128 v[124:127], %[ad] offset:48\n"
        "1:\n"
        "s_waitcnt lgkmcnt(3)\n"
        "v_add_f64 %[acc], %[acc], v[112:113]\n"
        "v_add_f64 %[acc], %[acc], v[114:115]\n"
        "s_waitcnt lgkmcnt(2)\n"
        "v_add_f64 %[acc], %[acc], v[116:117]\n"
        "v_add_f64 %[acc], %[acc], v[118:119]\n"
        "ds_read_b128 v[112:115], %[ad] offset:64\n"
        "ds_read_b128 v[116:119], %[ad] offset:80\n"
        "s_waitcnt lgkmcnt(3)\n"
        "v_add_f64 %[acc], %[acc], v[120:121]\n"
        "v_add_f64 %[acc], %[acc], v[122:123]\n"
        "s_waitcnt lgkmcnt(2)\n"
        "v_add_f64 %[acc], %[acc], v[124:125]\n"
        "v_add_f64 %[acc], %[acc], v[126:127]\n"
        "ds_read_b128 v[120:123], %[ad] offset:96\n"
        "ds_read_b128 v[124:127], %[ad] offset:112\n"
        "v_add_u32 %[ad], 64, %[ad]\n"
        "s_sub_u32 %[st], %[st], 1\n"
        "s_cmp_lg_u32 %[st], 0\n"
        "s_cbranch_scc1 1b\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [ad] "+v"(addr), [st] "+s"(steps)
        :
        : "memory", "scc", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
          "v122", "v123", "v124", "v125", "v126", "v127");
  }
  if (nfull < ce) chain_tail(acc, src, nfull, ce);
}
// (four 4-term batches in fixed registers v[96, 127], each reloaded 16 terms ahead right after
// its adds; six batches -- 24-term steps, 48 fixed VGPRs -- spilled 22 VGPRs in the 8-wave
// kernel and ran C3 exact 2.00 vs 1.90 ms, profiles/archive/r05r/)
__device__ __forceinline__ void chain_add_deep(double& acc, const double* src, int ce) {
  const int steps = ce / 16;
  const int nfull = steps * 16;
  if (steps) {
    unsigned addr = (unsigned)(uintptr_t)src;
    int st = steps;
    asm volatile(
        "ds_read_b128 v[96:99], %[ad] offset:0\n"
        "ds_read_b128 v[100:103], %[ad] offset:16\n"
        "ds_read_b128 v[104:107], %[ad] offset:32\n"
        "ds_read_b128 v[108:111], %[ad] offset:48\n"
        "ds_read_b128 v[112:115], %[ad] offset:64\n"
        "ds_read_b128 v[116:119], %[ad] offset:80\n"
        "ds_read_b128 v[120:123], %[ad] offset:96\n"
        "ds_read_b128 v[124:127], %[ad] offset:112\n"
        "1:\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[96:97]\n"
        "v_add_f64 %[acc], %[acc], v[98:99]\n"
        "v_add_f64 %[acc], %[acc], v[100:101]\n"
        "v_add_f64 %[acc], %[acc], v[102:103]\n"
        "ds_read_b128 v[96:99], %[ad] offset:128\n"
        "ds_read_b128 v[100:103], %[ad] offset:144\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[104:105]\n"
        "v_add_f64 %[acc], %[acc], v[106:107]\n"
        "v_add_f64 %[acc], %[acc], v[108:109]\n"
        "v_add_f64 %[acc], %[acc], v[110:111]\n"
        "ds_read_b128 v[104:107], %[ad] offset:160\n"
        "ds_read_b128 v[108:111], %[ad] offset:176\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[112:113]\n"
        "v_add_f64 %[acc], %[acc], v[114:115]\n"
        "v_add_f64 %[acc], %[acc], v[116:117]\n"
        "v_add_f64 %[acc], %[acc], v[118:119]\n"
        "ds_read_b128 v[112:115], %[ad] offset:192\n"
        "ds_read_b128 v[116:119], %[ad] offset:208\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[120:121]\n"
        "v_add_f64 %[acc], %[acc], v[122:123]\n"
        "v_add_f64 %[acc], %[acc], v[124:125]\n"
        "v_add_f64 %[acc], %[acc], v[126:127]\n"
        "ds_read_b128 v[120:123], %[ad] offset:224\n"
        "ds_read_b128 v[124:127], %[ad] offset:240\n"
        "v_add_u32 %[ad], 128, %[ad]\n"
        "s_sub_u32 %[st], %[st], 1\n"
        "s_cmp_lg_u32 %[st], 0\n"
        "s_cbranch_scc1 1b\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [ad] "+v"(addr), [st] "+s"(st)
        :
        : "memory", "scc", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127");
  }
  for (int from = nfull; from < ce; from += 8) chain_tail(acc, src, from, ce);
}

// LDS of one market's workgroup of NW waves, carved from a byte buffer.
//   region A  P doubles (+ read-ahead pad): input-order probs, then sorted probs in place
//   region B  sort exchange rows, then leaders [P] (+ exact: chain buffers [2][3][NT])
//   small     per-wave last keys / counts, totals, error index, exact hand-off counters
template <int NW, int R, bool FAST, int NN, class KT = unsigned>
struct WideLds {
  using Cfg = WideCfg<NW, R, FAST, NN, KT>;
  static constexpr int A_BYTES = Cfg::A_DBL * 8;
  static constexpr int B_BYTES = ((Cfg::B_U32 * 4 + 15) / 16) * 16;
  static constexpr int TOT_OFF = A_BYTES + B_BYTES;          // sTot [3*NW] doubles
  static constexpr int LAST_OFF = TOT_OFF + 24 * NW;          // sLast [NW] keys
  static constexpr int CNT_OFF = LAST_OFF + (int)sizeof(KT) * NW;  // sCnt [NW]
  static constexpr int MISC_OFF = CNT_OFF + 4 * NW;           // sErr, sRdy[2], sDone
  static constexpr int BYTES = ((MISC_OFF + 16 + 15) / 16) * 16;
  double* sA;
  unsigned* sB;
  double* sTot;
  KT* sLast;
  int* sCnt;
  int* sErr;
  int* sRdy;
  int* sDone;
  __device__ __forceinline__ explicit WideLds(unsigned char* base)
      : sA(reinterpret_cast<double*>(base)),
        sB(reinterpret_cast<unsigned*>(base + A_BYTES)),
        sTot(reinterpret_cast<double*>(base + TOT_OFF)),
        sLast(reinterpret_cast<KT*>(base + LAST_OFF)),
        sCnt(reinterpret_cast<int*>(base + CNT_OFF)),
        sErr(reinterpret_cast<int*>(base + MISC_OFF)),
        sRdy(reinterpret_cast<int*>(base + MISC_OFF + 4)),
        sDone(reinterpret_cast<int*>(base + MISC_OFF + 12)) {}
};

// The buffer loads of a market's sids
// and probabilities into registers (records = n signals, so i >= n reads 0).
template <int NW, int R>
__device__ __forceinline__ void wide_load(const ConsArgs& a, int64_t off, int n, int t, unsigned (&ps)[R],
                                          double (&pp)[R]) {
  constexpr int NT = 64 * NW, P = NT * R;
  const int cnt = n < P ? n : P;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a.sid + off), 0, cnt * 4, 0x00020000);
#pragma unroll
  for (int c = 0; c < R; ++c) ps[c] = __builtin_amdgcn_raw_buffer_load_b32(rs, t * 4, c * NT * 4, 0);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)(a.prob + off), 0, cnt * 8, 0x00020000);
#pragma unroll
  for (int c = 0; c < R; ++c)
    pp[c] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rp, t * 8, c * NT * 8, 0));
}

// One market (m, off, n) on a workgroup of NW waves; t = thread.  ps / pp hold
// its sids and probabilities (loaded by the caller); issue_next() is called once the keys are
// built, to start the workgroup's next market's loads into ps / pp.
template <int NW, int R, bool FAST, int NN, class KT, class NextFn>
__device__ __forceinline__ void wide_market(const ConsArgs& a, const WideLds<NW, R, FAST, NN, KT>& L, const int t,
                                            const int32_t m, const int64_t off, int n, unsigned (&ps)[R],
                                            double (&pp)[R], NextFn&& issue_next) {
  using Cfg = WideCfg<NW, R, FAST, NN, KT>;
  constexpr int NT = Cfg::NT, P = Cfg::P, IB = Cfg::IB, HR = Cfg::HR, LW = Cfg::LW;
  constexpr KT QMASK = (KT)Cfg::PN - 1u;  // the input-index bits of a key
  constexpr int kNoErr = 0x7fffffff;
  double* const sA = L.sA;
  unsigned* const sB = L.sB;
  unsigned* const sX = sB;                                            // sort exchange rows
  KT* const sLead = reinterpret_cast<KT*>(sB);                        // [u] sid<<IB | q0
  double* const sWAC = reinterpret_cast<double*>(sB + LW * P);        // exact: [2][3][NT]
  // FAST: the region past the leaders (the dead exchange rows) parks w[j] for normalizedWeight
  // when the market's uniques fit -- C3's Zipf markets have u <= 0.55 n, which fits in ~all
  // of them -- instead of reading the weight output back (each load there waits for this
  // thread's earlier stores to retire: vmcnt is in order)
  // (race-free: the next market's first wave-crossing stage writes exchange buffer 0 =
  // sB[0, P); buffer 1 = sB[P, 2P) is written only after that stage's barrier, which every
  // thread reaches after its own tail)
  // (64-bit keys: the leaders fill region B, nothing is parked)
  constexpr int WFREE = FAST ? (Cfg::B_U32 - LW * P) / 2 : 0;
  double* const sW = reinterpret_cast<double*>(sB + LW * P);

  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // wave within the workgroup (uniform)
  const unsigned smax = (unsigned)(a.n_sources > 0 ? a.n_sources - 1 : 0);
  // normalizedWeight reads w[j] back from the weight output (this thread's own stores)
  // in workgroups of several waves (it saves their barriers); a single wave parks w[j] in
  // region A (dead sorted-prob slot j), which is faster than the global round trip.
  const bool wback = (NW > 1) && a.weight != nullptr;

  // ---- 1. keys; next market's metadata + sids --------------------------------------
  KT key[R];
  bool badsid = false;
#pragma unroll
  for (int c = 0; c < R; ++c) {
    const int i = c * NT + t;
    const unsigned s = ps[c];
    badsid |= (i < n) && (s > smax);
    key[c] = (i < n) ? ((KT)(s < smax ? s : smax) << IB) | (KT)i : ~(KT)0;
  }
  if (ballot(badsid)) raise_fault(a.fault, kFaultSid);
  int myerr = kNoErr;
  // input-order probs into region A before the next loads; region A's last readers are
  // the previous market's run sums (before its final barrier) unless normalizedWeight
  // reads w[j] from it
  if (NW > 1 && !wback) __syncthreads();
#pragma unroll
  for (int c = 0; c < R; ++c) {
    const int i = c * NT + t;
    const double p = pp[c];
    sA[i] = p;
    if ((i < n) && (p < 0.0 || p > 1.0) && myerr == kNoErr) myerr = i;  // core.py:59-60
  }
  issue_next();
  if (n > P) {  // longer than this launch's max_len: left unprocessed, reported
    raise_fault(a.fault, kFaultTooLong);
    return;  // uniform over the workgroup
  }
  if (t == 0) *L.sErr = kNoErr;

  // ---- 2. sort (core.py:103 order; ties in input order by the index bits) ----------
  wide_sort<NN, NW, R>(key, sX, t, lane);

  // ---- 3. input-order probs + range check, sorted probs in place, leaders ----------
  if (lane == 63) L.sLast[wv] = key[R - 1];
  __syncthreads();  // (a) input-order probs + sLast visible; exchange rows dead
  if (myerr != kNoErr) atomicMin(L.sErr, myerr);
  double x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = t * R + r;
    x[r] = (q < n) ? sA[key[r] & QMASK] : 0.0;
  }
  KT prev_in_wave;  // wave_shr:1
  if constexpr (LW == 2)
    prev_in_wave = k_make((unsigned)__builtin_amdgcn_update_dpp(0, (int)k_hi(key[R - 1]), 0x138, 0xF, 0xF, false),
                          (unsigned)__builtin_amdgcn_update_dpp(0, (int)k_lo(key[R - 1]), 0x138, 0xF, 0xF, false));
  else
    prev_in_wave = (unsigned)__builtin_amdgcn_update_dpp(0, (int)key[R - 1], 0x138, 0xF, 0xF, false);
  const KT prev_key = (lane > 0) ? prev_in_wave : (wv > 0 ? L.sLast[wv - 1] : (KT)0);
  unsigned lead = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = t * R + r;
    const KT ps0 = ((r == 0) ? prev_key : key[r - 1]) >> IB;
    const bool is = (q < n) && (q == 0 || (key[r] >> IB) != ps0);
    lead |= is ? (1u << r) : 0u;
  }
  const int cnt = __popc(lead);
  const int incl = wave_incl_scan(cnt);
  if (lane == 63) L.sCnt[wv] = incl;
  __syncthreads();  // (b) every read of the input-order probs done; counts visible
#pragma unroll
  for (int r = 0; r < R; r += 2) *reinterpret_cast<double2*>(sA + t * R + r) = make_double2(x[r], x[r + 1]);
  int base = incl - cnt, u = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int cw = L.sCnt[w];
    if (w < wv) base += cw;
    u += cw;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (lead & (1u << r)) {
      const int jj = base + __popc(lead & ((1u << r) - 1u));
      sLead[jj] = (key[r] & ~QMASK) | (KT)(t * R + r);
    }
  }
  if (t == 0) {
    L.sRdy[0] = L.sRdy[1] = 0;
    *L.sDone = 0;
  }
  __syncthreads();  // (c) sorted probs + leaders visible

  // ---- 4. per-unique products --------------------------------------------------------
  double acc = 0.0;                     // exact: wave 0 lanes 0..2 carry the chains
  double pw = 0.0, pa = 0.0, pc = 0.0;  // fast: this thread's partial sums
  // EXACT with several waves (and the weight output, so region A is not needed for w):
  // wave 0 only carries the chains while waves 1.. produce rounds of NP = NT - 64
  // uniques into a two-slot LDS ring, handed over with LDS counters instead of barriers,
  // so the serial chains overlap the gathers and run sums of the next rounds.
  const bool piped = !FAST && NW > 1 && wback;
  if (piped) {
    constexpr int NP = (NW > 1) ? NT - 64 : NT;
    const int nrp = (u + NP - 1) / NP;
    if (wv == 0) {
      __builtin_amdgcn_s_setprio(2);  // the chain is the critical path
      for (int r = 0; r < nrp; ++r) {
        const int slot = r & 1;
        const int need = (NW - 1) * ((r >> 1) + 1);
        int spins = 0;
        while (ldsflag(&L.sRdy[slot]) < need) {
          if (++spins > a.spin_cap) {
            raise_fault(a.fault, kFaultSpinChain);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        const int ce = (u - r * NP < NP) ? u - r * NP : NP;
        if (!kWideChain3 || lane < 3) {  // kWideChain3: only the three chain lanes read LDS
          if constexpr (kWideChainDeep) chain_add_deep(acc, sWAC + slot * 3 * NP + (lane % 3) * NP, ce);
          else chain_add(acc, sWAC + slot * 3 * NP + (lane % 3) * NP, ce);
        }
        if (lane == 0) __hip_atomic_store(L.sDone, r + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __builtin_amdgcn_s_setprio(0);
    } else {
      const int pt = t - 64;
      for (int h = 0; h < nrp; h += HR) {
        double2 rc[HR];
        int q0s[HR], q1s[HR];
        unsigned sids[HR], pwd[HR];
#pragma unroll
        for (int i = 0; i < HR; ++i) {  // every gather of the group in flight together
          const int jj = (h + i) * NP + pt;
          q0s[i] = q1s[i] = 0;
          sids[i] = pwd[i] = 0;
          rc[i] = make_double2(0.5, 0.25);  // DEFAULT_RELIABILITY / _CONFIDENCE (empty table)
          if (jj < u) {
            const KT lv = sLead[jj];
            q0s[i] = (int)(lv & QMASK);
            sids[i] = (unsigned)min(lv >> IB, (KT)smax);
            q1s[i] = (jj + 1 < u) ? (int)(sLead[jj + 1] & QMASK) : n;
            if (a.n_sources > 0) {
              rc[i] = a.relconf[sids[i]];
              pwd[i] = a.pbits[sids[i] >> 5];
            }
          }
        }
        double vw[HR], va[HR], vc[HR];
#pragma unroll
        for (int i = 0; i < HR; ++i) {
          const int jj = (h + i) * NP + pt;
          vw[i] = va[i] = vc[i] = 0.0;
          if (jj < u) {
            const double avg = run_sum<R>(sA, q0s[i], q1s[i] - q0s[i]);  // core.py:116
            const double w = rc[i].x;  // core.py:111,119
            vw[i] = w;
            va[i] = avg * w;        // core.py:136
            vc[i] = rc[i].y * w;    // core.py:142
          }
        }
#pragma unroll
        for (int i = 0; i < HR; ++i) {
          const int r = h + i;
          if (r < nrp) {
            const int slot = r & 1;
            if (r >= 2) {  // the slot's previous round is consumed
              int spins = 0;
              while (ldsflag(L.sDone) < r - 1) {
                if (++spins > a.spin_cap) {
                  raise_fault(a.fault, kFaultSpinChain);
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
            }
            double* const buf = sWAC + slot * 3 * NP;
            buf[pt] = vw[i];
            buf[NP + pt] = va[i];
            buf[2 * NP + pt] = vc[i];
            wave_sync_lds();  // this wave's part of the round is in LDS
            if (lane == 0)
              __hip_atomic_fetch_add(&L.sRdy[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
#pragma unroll
        for (int i = 0; i < HR; ++i) {
          const int jj = (h + i) * NP + pt;
          if (jj < u) {
            const int64_t p = off + jj;
            if (a.usid)
              a.usid[p] = (int32_t)sids[i] | (((pwd[i] >> (sids[i] & 31)) & 1u) ? 0 : (int32_t)0x80000000);
            a.weight[p] = vw[i];
          }
        }
      }
    }
  }
  const int nr = piped ? 0 : (u + NT - 1) / NT;
  const bool park = FAST && wback && u <= WFREE;
  for (int h = 0; h < nr; h += HR) {
    double2 rc[HR];
    int q0s[HR], q1s[HR];
    unsigned sids[HR], pwd[HR];
#pragma unroll
    for (int i = 0; i < HR; ++i) {  // every gather of the group in flight together
      const int jj = (h + i) * NT + t;
      q0s[i] = q1s[i] = 0;
      sids[i] = pwd[i] = 0;
      rc[i] = make_double2(0.5, 0.25);  // DEFAULT_RELIABILITY / _CONFIDENCE (empty table)
      if (jj < u) {
        const KT lv = sLead[jj];
        q0s[i] = (int)(lv & QMASK);
        sids[i] = (unsigned)min(lv >> IB, (KT)smax);  // <= smax by construction of the key; clamped anyway
        q1s[i] = (jj + 1 < u) ? (int)(sLead[jj + 1] & QMASK) : n;
        if (a.n_sources > 0) {
          rc[i] = a.relconf[sids[i]];
          pwd[i] = a.pbits[sids[i] >> 5];
        }
      }
    }
    double vw[HR], va[HR], vc[HR];
#pragma unroll
    for (int i = 0; i < HR; ++i) {
      const int jj = (h + i) * NT + t;
      const int len = q1s[i] - q0s[i];
      double avg = 0.0;
      if constexpr (FAST) {
        // runs longer than kWaveRun (hot sources) are summed by the whole wave in a fixed
        // order instead of by their own lane, so one hot source does not hold the wave
        avg = (jj < u && len <= kWaveRun) ? run_sum<R, kWideFastRecip>(sA, q0s[i], len) : 0.0;
        unsigned long long lm = ballot(jj < u && len > kWaveRun);
        while (lm) {
          const int LL = __builtin_ctzll(lm);
          lm &= lm - 1;
          const int lq0 = __builtin_amdgcn_readlane(q0s[i], LL), llen = __builtin_amdgcn_readlane(len, LL);
          double part = 0.0;
          for (int e = lane; e < llen; e += 64) part += sA[lq0 + e];
          part = wave_sum_fixed(part);
          if (lane == LL) avg = part / (double)llen;
        }
      } else if (jj < u) {
        avg = run_sum<R>(sA, q0s[i], len);
      }
      vw[i] = va[i] = vc[i] = 0.0;
      if (jj < u) {
        const double w = rc[i].x;  // core.py:111,119
        vw[i] = w;
        va[i] = avg * w;        // core.py:136
        vc[i] = rc[i].y * w;    // core.py:142
      }
    }
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < HR; ++i) {  // round order: fixed per thread
        pw += vw[i];
        pa += va[i];
        pc += vc[i];
      }
      if (!wback) {
        __syncthreads();  // every sorted-prob read of this group done
#pragma unroll
        for (int i = 0; i < HR; ++i) {
          const int jj = (h + i) * NT + t;
          if (jj < u) sA[jj] = vw[i];  // later groups read only positions > jj
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < HR; ++i) {
        if (h + i < nr) {
          double* const buf = sWAC + ((h + i) & 1) * 3 * NT;
          buf[t] = vw[i];
          buf[NT + t] = va[i];
          buf[2 * NT + t] = vc[i];
          __syncthreads();  // round staged; every sorted-prob read of this group is done
          const int jj = (h + i) * NT + t;
          if (jj < u && !wback) sA[jj] = vw[i];  // position jj is only read by uniques <= jj
          if (wv == 0) {
            __builtin_amdgcn_s_setprio(2);  // the chain is the critical path
            const int ce = (u - (h + i) * NT < NT) ? u - (h + i) * NT : NT;
            if (!kWideChain3 || lane < 3) chain_add(acc, buf + (lane % 3) * NT, ce);
            __builtin_amdgcn_s_setprio(0);
          }
        }
      }
    }
    // per-unique outputs after the group's LDS work, so no store is pending under it;
    // nontemporal (FAST -0.5..1%, profiles/r03k/wide_r03u_ab.txt)
#pragma unroll
    for (int i = 0; i < HR; ++i) {
      const int jj = (h + i) * NT + t;
      if (jj < u) {
        const int64_t p = off + jj;
        if (a.usid)
          __builtin_nontemporal_store((int32_t)sids[i] | (((pwd[i] >> (sids[i] & 31)) & 1u) ? 0 : (int32_t)0x80000000), &a.usid[p]);
        if (a.weight) __builtin_nontemporal_store(vw[i], &a.weight[p]);
        if (park) sW[jj] = vw[i];
      }
    }
  }

  // ---- 5. totals, per-market outputs, nweight ------------------------------------------
  if constexpr (FAST) {
    pw = wave_sum_fixed(pw);
    pa = wave_sum_fixed(pa);
    pc = wave_sum_fixed(pc);
    if (lane == 0) {
      L.sTot[3 * wv] = pw;
      L.sTot[3 * wv + 1] = pa;
      L.sTot[3 * wv + 2] = pc;
    }
  } else {
    if (wv == 0 && lane < 3) L.sTot[lane] = acc;
  }
  __syncthreads();  // totals + w[j] visible
  double tw = L.sTot[0], ta = L.sTot[1], tc = L.sTot[2];
  if constexpr (FAST) {
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      tw += L.sTot[3 * w];
      ta += L.sTot[3 * w + 1];
      tc += L.sTot[3 * w + 2];
    }
  }
  if (t == 0 && m >= 0) {
    const bool null_ = (n == 0) || (tw == 0.0);
    a.consensus[m] = null_ ? 0.0 : ta / tw;
    a.confidence[m] = null_ ? 0.0 : tc / tw;
    a.total_weight[m] = tw;
    a.n_unique[m] = u;
    if (a.err_idx) a.err_idx[m] = (*L.sErr == kNoErr) ? -1 : *L.sErr;
  }
  if (a.nweight) {  // core.py:151
    if constexpr (!FAST) {
      // every read-back issued before any nweight store: loads retire behind earlier
      // stores (vmcnt is in order), so a load/store per iteration waits out each store
      // (C3 exact -2.6%; FAST: batches of kWideNWBF, a full batch costs it spills)
      double wj[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int jj = t + NT * k;
        wj[k] = (jj < u) ? (wback ? a.weight[off + jj] : sA[jj]) : 0.0;
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int jj = t + NT * k;
        if (jj < u) a.nweight[off + jj] = (tw > 0.0) ? wj[k] / tw : 0.0;
      }
    } else {
      constexpr int NB = (kWideNWBF < R) ? kWideNWBF : R;  // read-backs per batch
      const double rtw = (tw > 0.0) ? 1.0 / tw : 0.0;
      for (int j0 = t; j0 < u; j0 += NB * NT) {
        double wj[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int jj = j0 + NT * k;
          wj[k] = (jj < u) ? (park ? sW[jj] : wback ? a.weight[off + jj] : sA[jj]) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int jj = j0 + NT * k;
          const double nw = kWideFastRecip ? ((tw > 0.0) ? wj[k] * rtw : 0.0) : ((tw > 0.0) ? wj[k] / tw : 0.0);
          if (jj < u) __builtin_nontemporal_store(nw, &a.nweight[off + jj]);
        }
      }
    }
  }
}

// One bin per launch: a persistent grid of NW-wave workgroups strides over the bin's market
// list (one market per workgroup at a time, the next one's loads issued during this one).
template <int NW, int R, bool FAST, int NN = NW, class KT = unsigned>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WideCfg<NW, R, FAST, NN, KT>::WPE, 8))) void consensus_wide_kernel(ConsArgs a) {
  dev_range(a);
  using LD = WideLds<NW, R, FAST, NN, KT>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LD::BYTES];
  const LD L(smem);
  const int t = threadIdx.x;
  const int lane = lane_id();

  // Market metadata for this workgroup's next 64 markets (li = base + G*k on lane k) is
  // loaded in one vector batch, so picking a market is a readlane, never a scalar-load
  // stall.  A market's sids are loaded one market ahead, its probabilities while the
  // previous market finishes (buffer loads: records = n signals, so i >= n reads 0).
  const int64_t G = gridDim.x;
  int32_t vm = 0;
  int64_t voff = 0;
  int vn = 0;
  auto refill = [&](int64_t base) {
    const int64_t li = base + G * lane;
    vm = (li < a.n_list) ? (a.list ? (li < a.n_hi ? a.list_hi[li] : a.list[li - a.n_hi]) : (int32_t)li) : 0;
    voff = (li < a.n_list) ? a.offsets[vm] : 0;
    vn = (li < a.n_list) ? (int)(a.offsets[vm + 1] - voff) : 0;
  };
  int32_t nm = 0;
  int64_t noff = 0;
  int nn = 0;
  auto meta = [&](int64_t li) {
    const int k = (int)(((li - blockIdx.x) / G) & 63);
    if (k == 0) refill(li);
    nm = __builtin_amdgcn_readlane(vm, k);
    noff = ((int64_t)__builtin_amdgcn_readlane((int)(voff >> 32), k) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)voff, k);
    nn = __builtin_amdgcn_readlane(vn, k);
  };
  unsigned ps[R];
  double pp[R];
  if (blockIdx.x < a.n_list) {
    meta(blockIdx.x);
    wide_load<NW, R>(a, noff, nn, t, ps, pp);
  }
  for (int64_t li = blockIdx.x; li < a.n_list; li += G) {
    const int32_t m = nm;
    const int64_t off = noff;
    const int n = nn;
    wide_market<NW, R, FAST, NN, KT>(a, L, t, m, off, n, ps, pp, [&]() {
      if (li + G < a.n_list) {
        meta(li + G);
        wide_load<NW, R>(a, noff, nn, t, ps, pp);
      }
    });
  }
}

template <int NW, int R, bool FAST, int NN, class KT>
int64_t resident_kt() {
  const void* fn = reinterpret_cast<const void*>(&consensus_wide_kernel<NW, R, FAST, NN, KT>);
  return (int64_t)cu_count() * blocks_per_cu(fn, 64 * NW, 0, 1, "consensus_wide_kernel");
}

template <int NW, int R, bool FAST, int NN = NW>
int64_t resident_wide(int32_t n_sources) {
  constexpr int IB = WideCfg<NW, R, FAST, NN>::IB;
  return ((int64_t)n_sources <= (1ll << (32 - IB))) ? resident_kt<NW, R, FAST, NN, unsigned>()
                                                     : resident_kt<NW, R, FAST, NN, uint64_t>();
}

template <bool FAST>
int64_t resident_mode(int64_t max_len, int32_t n_sources) {
  if (max_len <= 128) return resident_wide<1, 2, FAST>(n_sources);
  if (max_len <= 256) return resident_wide<1, 4, FAST>(n_sources);
  if (max_len <= 512) return resident_wide<1, 8, FAST>(n_sources);
  if (max_len <= 1024) return resident_wide<2, 8, FAST>(n_sources);
  if (max_len <= 1536) return resident_wide<3, 8, FAST, 4>(n_sources);
  if (max_len <= 2048) return resident_wide<4, 8, FAST>(n_sources);
  if (max_len <= 3072) return resident_wide<6, 8, FAST, 8>(n_sources);
  return resident_wide<8, 8, FAST>(n_sources);
}

template <int NW, int R, bool FAST, int NN, class KT>
int launch_wide_kt(const ConsArgs& a, hipStream_t st) {
  const void* fn = reinterpret_cast<const void*>(&consensus_wide_kernel<NW, R, FAST, NN, KT>);
  const int per_cu = blocks_per_cu(fn, 64 * NW, 0, 1, "consensus_wide_kernel");
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(a.n_list < cap ? a.n_list : cap);
  hipLaunchKernelGGL((consensus_wide_kernel<NW, R, FAST, NN, KT>), dim3(grid), dim3(64 * NW), 0, st, a);
  return check_launch("consensus_wide_kernel");
}

// 32-bit keys while the sid fits beside the IB index bits, 64-bit keys for larger tables
template <int NW, int R, bool FAST, int NN = NW>
int launch_wide(const ConsArgs& a, hipStream_t st) {
  if (a.n_list == 0) return BCE_OK;
  constexpr int IB = WideCfg<NW, R, FAST, NN>::IB;
  if ((int64_t)a.n_sources <= (1ll << (32 - IB))) return launch_wide_kt<NW, R, FAST, NN, unsigned>(a, st);
  return launch_wide_kt<NW, R, FAST, NN, uint64_t>(a, st);
}

// (NW, R[, NN]) per length bin: P = 64*NW*R >= max_len; the 1536 and 3072 bins run the
// 2048 / 4096-key network on 3 / 6 waves
// (Round 5: a market shard's 513..1024 / 1025..2048 bins on 4 / 8 waves with R = 4 -- half the
// latency per market, more rounds -- made one 8th of C3 slower, 0.2069-0.2072 -> 0.2274-0.2300
// ms, profiles/archive/r05g/; removed.)
template <bool FAST>
int launch_wide_mode(int64_t max_len, const ConsArgs& a, hipStream_t st) {
  if (max_len <= 128) return launch_wide<1, 2, FAST>(a, st);
  if (max_len <= 256) return launch_wide<1, 4, FAST>(a, st);
  if (max_len <= 512) return launch_wide<1, 8, FAST>(a, st);
  if (max_len <= 1024) return launch_wide<2, 8, FAST>(a, st);
  if (max_len <= 1536) return launch_wide<3, 8, FAST, 4>(a, st);
  if (max_len <= 2048) return launch_wide<4, 8, FAST>(a, st);
  if (max_len <= 3072) return launch_wide<6, 8, FAST, 8>(a, st);
  return launch_wide<8, 8, FAST>(a, st);
}

}  // namespace


namespace {
__global__ void lane_xor_selftest_kernel(unsigned* out) {
  const unsigned l = (unsigned)lane_id();
  out[0 * 64 + l] = lane_xor<1>(l);
  out[1 * 64 + l] = lane_xor<2>(l);
  out[2 * 64 + l] = lane_xor<3>(l);
  out[3 * 64 + l] = lane_xor<4>(l);
  out[4 * 64 + l] = lane_xor<7>(l);
  out[5 * 64 + l] = lane_xor<8>(l);
  out[6 * 64 + l] = lane_xor<15>(l);
  out[7 * 64 + l] = lane_xor<16>(l);
  out[8 * 64 + l] = lane_xor<31>(l);
  out[9 * 64 + l] = lane_xor<32>(l);
  out[10 * 64 + l] = lane_xor<63>(l);
  out[11 * 64 + l] = (unsigned)wave_incl_scan((int)l + 1);
  out[12 * 64 + l] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)l + 100, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
}  // namespace

// Self-test of the sort's lane exchanges and the wave scan (one wave, touches only `out`):
// out[q*64 + l] must equal l ^ {1,2,3,4,7,8,15,16,31,32,63}[q], out[11*64 + l] = (l+1)(l+2)/2,
// out[12*64 + l] = l + 99 (lane l-1's l+100; 0 in lane 0).  `out` holds 13*64 words.
extern "C" int bce_debug_lane_selftest(unsigned* out, void* stream) {
  BCE_REQUIRE(out, "lane_selftest: NULL");
  hipLaunchKernelGGL(lane_xor_selftest_kernel, dim3(1), dim3(64), 0, as_stream(stream), out);
  return check_launch("lane_xor_selftest_kernel");
}


int64_t wide_resident(int64_t max_len, int32_t mode, int32_t n_sources) {
  return (mode == BCE_MODE_FAST) ? resident_mode<true>(max_len, n_sources) : resident_mode<false>(max_len, n_sources);
}

int launch_wide_len(int64_t max_len, const ConsArgs& a, hipStream_t st) {
  return (a.mode == BCE_MODE_FAST) ? launch_wide_mode<true>(max_len, a, st) : launch_wide_mode<false>(max_len, a, st);
}

}  // namespace bce
