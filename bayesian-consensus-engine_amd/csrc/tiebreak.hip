// tiebreak.hip -- DeterministicTieBreaker.resolve (tiebreak.py:73-152) per CSR market.
//
// One lane per market (n <= 32 agents, tiebreak_lpm_kernel), one wave per market
// (n <= 64; lane = agent), or one 256-thread workgroup per market with the agents staged
// in LDS (64 < n <= 4096) or in a global scratch slice (any length).  Grouping key = CPython
// round(prediction, 6) (tiebreak.py:54) restated exactly (bce::py_round_nd).  A group's
// leader is its first-seen member, so groups come out in dict insertion order for free.
// Group sums (weight, confidence) run in input order, max reliability keeps the first
// maximum (builtin max), and the winner is the lexicographic max of
// (density, max_rel, -key) -- distinct groups never tie on the full tuple, so any
// reduction order selects the same winner.
#include <atomic>

#include "bce_device.hpp"
#include "bce_internal.hpp"
#include "consensus_common.hpp"
#include "glibc_pow.hpp"
#include "py_round_big.hpp"

#pragma clang fp contract(off)

namespace bce {

struct TbArgs {
  const int64_t* offsets;
  int64_t n_markets;
  const double* pred;
  const double* conf;
  const double* weight;
  const double* rel;
  double* winner;
  int32_t* label;
  int32_t* n_groups;
  double* variance;
  double* g_key;
  int32_t* g_count;
  double* g_density;
  double* g_avgconf;
  double* g_maxrel;
  int32_t* g_of;   // nullable: per agent, the ordinal of its group (dict insertion order)
  double rscale;   // 10^ndigits (ndigits >= 0) or 10^-ndigits (ndigits < 0)
  double rthresh;  // see py_round_nd
  double rinv;     // RN(1 / rscale) (mode 0)
  int rmode;       // 0: py_round_nd, 1: py_round_neg, 2: identity (nd > 323), 3: signed zero (nd < -308),
                   // 4: big-integer path 23 <= nd <= 323, 5: big-integer path -308 <= nd <= -16
  int rnd;         // ndigits (modes 4, 5)
  int* fault;      // device fault word: kFaultRoundOverflow (CPython's OverflowError)
  int* split;      // PART 1/2 launches: one word per wave of the (shared) grid; a PART 1 wave
                   // that leaves a tile to PART 2 writes `ticket` into its word
  int ticket;      // this launch pair's number (host counter, never 0): no reset needed
};

constexpr int kFaultRoundOverflow = 6;  // round(x, nd) too large to represent (mode 5)

// round(prediction, precision) of tiebreak.py:54 for every precision CPython accepts (see
// tb_round_mode on the host).  EXOTIC kernels (modes 4, 5: 10^|nd| not an exact double) run
// the exact big-integer restatement of py_round_big.hpp; the others never contain it.
// report: this lane's value is really rounded by the reference -- an agent of a market with
// >= 2 agents (a single agent keeps its raw prediction, tiebreak.py:89-96, and lanes without a
// market round a placeholder) -- so its OverflowError is raised.
template <bool EXOTIC>
__device__ __forceinline__ double tb_round(double x, const TbArgs& a, bool report = true) {
  if constexpr (EXOTIC) {
    if (a.rmode == 4) return bce_round::round_pos(x, a.rnd);
    bool ovf = false;
    const double r = bce_round::round_neg(x, -a.rnd, &ovf);
    if (ovf && report && a.fault) atomicCAS(a.fault, 0, kFaultRoundOverflow);
    return r;
  } else {
    switch (a.rmode) {
      case 0: return py_round_nd(x, a.rscale, a.rthresh);
      case 1: return py_round_neg(x, a.rscale);
      case 2: return x;
      default: return (x != x || fabs(x) == __builtin_inf()) ? x : copysign(0.0, x);
    }
  }
}

__device__ __forceinline__ bool key_eq(double a, double b) { return a == b; }  // -0.0 == 0.0

// (d1, m1, k1) strictly better than (d2, m2, k2) under Python tuple order of
// (density, max_reliability, -key).
__device__ __forceinline__ bool tb_better(double d1, double m1, double k1, double d2, double m2,
                                          double k2) {
  if (d1 != d2) return d1 > d2;
  if (m1 != m2) return m1 > m2;
  return (-k1) > (-k2);
}

// tb_better without short-circuit returns
__device__ __forceinline__ bool tb_better_sel(double d1, double m1, double k1, double d2, double m2,
                                              double k2) {
  const bool nd = d1 != d2, nm = m1 != m2;
  return nd ? (d1 > d2) : (nm ? (m1 > m2) : ((-k1) > (-k2)));
}

// The rare exact square (pow2_fast's near-midpoint cases) out of line: inlined, its log/exp
// polynomial constants were hoisted out of the tile loop and held in (spilled) registers.
__device__ __noinline__ double tb_pow2_full(double d) { return bce_pow::pow2_full(d); }

// x / c for a group size c in 1..32: RN(x * rc) with one FMA correction, rc = RN(1 / c)
// (Markstein; tools/check_markstein.c checks 3e9 quotients against IEEE division), exact
// for |x| in [2^-1000, 2^1000]; a wave with any other x (0, subnormal, huge, inf, NaN)
// divides those lanes.
__device__ __forceinline__ double tb_div_small(double x, int c, const double* rc_tab) {
  const double rc = rc_tab[c];
  const double b = (double)c;
  const double q0 = x * rc;
  const double q = __builtin_fma(__builtin_fma(-q0, b, x), rc, q0);
  const bool ok = ((int)(fabs(x) >= 0x1p-1000) & (int)(fabs(x) <= 0x1p1000)) != 0;
  return ballot(!ok) ? (ok ? q : x / b) : q;
}

__device__ __forceinline__ double rl_f64(double v, int l) {
  int2 x = *reinterpret_cast<int2*>(&v);
  int2 y;
  y.x = __builtin_amdgcn_readlane(x.x, l);
  y.y = __builtin_amdgcn_readlane(x.y, l);
  return *reinterpret_cast<double*>(&y);
}

template <bool EXOTIC>
__global__ __launch_bounds__(256) void tiebreak_wave_kernel(TbArgs a, const int32_t* list,
                                                            int64_t n_list) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t li = wave; li < n_list; li += nwaves) {
    const int64_t m = list ? list[li] : li;
    const int64_t off = a.offsets[m];
    const int n = (int)(a.offsets[m + 1] - off);
    // n == 0: tiebreak.py:86-87 (ValueError).  n > 64: longer than this kernel's lanes (a
    // max_len bound the caller got wrong) -- left unprocessed with the empty marker and
    // reported in the fault word, never computed from wrapped lanes
    if (n == 0 || n > 64) {
      if (n > 64) raise_fault(a.fault, kFaultTooLong);
      if (lane == 0) {
        a.winner[m] = 0.0; a.label[m] = -1; a.n_groups[m] = -1; a.variance[m] = 0.0;
      }
      continue;
    }
    const bool v = lane < n;
    double p = 0.0, c = 0.0, w = 0.0, r = 0.0;
    if (v) {
      p = a.pred[off + lane];
      c = a.conf[off + lane];
      w = a.weight[off + lane];
      r = a.rel[off + lane];
    }
    if (n == 1) {  // tiebreak.py:89-96
      if (lane == 0) {
        a.winner[m] = p; a.label[m] = BCE_TB_SINGLE_AGENT; a.n_groups[m] = 1; a.variance[m] = 0.0;
        if (a.g_key) a.g_key[off] = p;
        if (a.g_count) a.g_count[off] = 1;
        if (a.g_density) a.g_density[off] = w;
        if (a.g_avgconf) a.g_avgconf[off] = c;
        if (a.g_maxrel) a.g_maxrel[off] = r;
        if (a.g_of) a.g_of[off] = 0;
      }
      continue;
    }
    const double key = tb_round<EXOTIC>(p, a);
    // leader = first index with an equal key (dict insertion order)
    int leader = lane;
    for (int j = 0; j < n; ++j) {
      const double kj = rl_f64(key, j);
      if (v && j < leader && key_eq(kj, key)) leader = j;
    }
    const bool is_leader = v && leader == lane;
    // group metrics in input order (tiebreak.py:58-71), accumulated by the leader lane
    double tot = 0.0, cs = 0.0, mx = r;
    int cnt = 0;
    double csum_all = 0.0;
    for (int j = 0; j < n; ++j) {
      const int lj = __builtin_amdgcn_readlane(leader, j);
      const double wj = rl_f64(w, j), cj = rl_f64(c, j), rj = rl_f64(r, j);
      csum_all += cj;
      if (lj == lane) {
        tot += wj;
        cs += cj;
        ++cnt;
        if (j != lane && rj > mx) mx = rj;  // builtin max: first maximum kept
      }
    }
    const double dens = is_leader ? tot / (double)cnt : 0.0;
    const double avgc = is_leader ? cs / (double)cnt : 0.0;
    // variance of all confidences (tiebreak.py:108-110): sequential sums
    // (c - mean) ** 2 is libm pow, not d*d (glibc_pow.hpp): every lane squares its own
    // agent's deviation, then the squares are summed in agent order
    const double mean = csum_all / (double)n;
    const double sq = v ? bce_pow::pow2(c - mean) : 0.0;
    double vs = 0.0;
    for (int j = 0; j < n; ++j) vs += rl_f64(sq, j);
    const unsigned long long lm = ballot(is_leader);
    const int ng = __popcll(lm);
    // winner: lexicographic max over leaders
    int best = -1;
    double bd = 0.0, bm = 0.0, bk = 0.0;
    for (int j = 0; j < n; ++j) {
      if (!((lm >> j) & 1ull)) continue;
      const double dj = rl_f64(dens, j), mj = rl_f64(mx, j), kj = rl_f64(key, j);
      if (best < 0 || tb_better(dj, mj, kj, bd, bm, bk)) {
        best = j; bd = dj; bm = mj; bk = kj;
      }
    }
    const bool tie = is_leader && lane != best && dens == bd && mx == bm;
    int lab = BCE_TB_WEIGHT_DENSITY;
    if (ng == 1) lab = BCE_TB_UNANIMOUS;
    else if (ballot(tie)) lab = BCE_TB_PREDICTION_VALUE_SMALLEST;
    if (lane == 0) {
      a.winner[m] = bk;
      a.label[m] = lab;
      a.n_groups[m] = ng;
      a.variance[m] = vs / (double)n;
    }
    if (a.g_of && v) a.g_of[off + lane] = __popcll(lm & ((leader == 0) ? 0ull : (~0ull >> (64 - leader))));
    if (is_leader) {
      const int64_t g = off + __popcll(lm & below);
      if (a.g_key) a.g_key[g] = key;
      if (a.g_count) a.g_count[g] = cnt;
      if (a.g_density) a.g_density[g] = dens;
      if (a.g_avgconf) a.g_avgconf[g] = avgc;
      if (a.g_maxrel) a.g_maxrel[g] = mx;
    }
  }
}

// n <= 32, lane = market (64 markets per wave): every per-market step runs in one lane's
// registers, so none of the wave kernel's serial readlane loops exist and a wave's
// instructions serve 64 markets at once.
//
// Data movement (STAGED, contiguous markets): a wave's 64 markets are one contiguous CSR
// range [B, E) of <= 2048 agents.  Every input array is read ONCE with coalesced 16-B loads
// into a wave-private LDS buffer (one pad slot per 32, so lanes reading their own rows hit
// distinct bank pairs), and every per-agent / per-group output is assembled in such a buffer
// and leaves with coalesced 16-B stores (per-lane scattered stores wrote each line ~4 times:
// 5.3 GB of HBM writes for the 1.3 GB of outputs).  A group's outputs go to slot g of the
// market's row, overwriting the input of agent g in place: group g ends only after every
// group <= g, and agent g belongs to one of those (ordinals are assigned in first-seen
// order, so agent g's ordinal is <= g) -- its input has been consumed.  Slots g >= n_groups
// of a market's row receive unspecified values (include/bce.h).
// (The !STAGED path, for market lists, reads rows and writes outputs per lane.)
// Per lane:
//   1. keys round(pred, precision) (tiebreak.py:54) and each agent's group ordinal in
//      first-seen (dict insertion) order: O(n^2) key compares, == semantics (-0.0 == 0.0,
//      NaN never equal); keys (ordinal << 5 | agent) sorted by the odd-even merge network
//      with the rounded key as payload: every group becomes a run, groups in first-seen
//      order, members in input order;
//   2. walk (weight, reliability): the group's weight sum runs in input order from +0.0
//      (builtin sum from int 0), builtin max keeps the first maximum; at a run's end the
//      winner (lexicographic max of (density, max_rel, -key), tiebreak.py:113-117) and the
//      top-two tie flag (tiebreak.py:123-133) are updated;
//   3. variance (tiebreak.py:108-110; mean, then the squares -- libm pow restated,
//      glibc_pow.hpp -- summed in input order) and the per-group confidence sums.
constexpr int kTbLpmMax = 32;
constexpr int kTbLpmWaves = 4;
constexpr int kTbStage = 64 * kTbLpmMax + 64;  // doubles per wave buffer: a tile's agents + pads
constexpr int kTbStageIt = 64 * kTbLpmMax / 128;  // 16-B loads per lane for a full tile
constexpr int kTbStageBatch = 4;                  // of them in flight together (2 x 8 VGPRs each)
// A STAGED tile's arrays reach LDS as 16-B loads into registers, kTbStageBatch in flight, then
// ds_writes (two workgroups of four waves per CU).  LDS-DMA staging into the one buffer (1.070 vs
// 0.849-0.866 ms, profiles/archive/r04f/) and two DMA-filled buffers per wave (one workgroup per CU:
// 1.316 ms, profiles/archive/r04e/) were measured and removed.

__device__ __forceinline__ int tb_pad(int i) { return i + (i >> 5); }
constexpr bool kTbFullKeysInLds = true;  // FULL tiles: sort (ordinal, agent) alone, keys via LDS
// the staged general body likewise: tie-break over 1M ragged markets 0.7347-0.7364 -> 0.7201-0.7218
// ms, three interleaved reps (profiles/r06tb/)
constexpr bool kTbGeneralKeysInLds = true;
constexpr int kTbGatherBatch = 8;  // GATHER staging: passes whose row loads are in flight together
constexpr int kTbDump = 64;
// FULL tiles: 16-B loads per lane in flight while staging the predictions / confidences and the
// weights / reliabilities (8 for the latter spills ~10 VGPRs around those stages and still
// wins: 0.662 vs 0.688 ms with stage()'s 4, profiles/archive/r04q/)
constexpr int kTbFullBatchPC = 8;
constexpr int kTbFullBatchWR = 8;
constexpr bool kTbPrefetchMeta = true;
// (FULL tiles, measured and removed: the next array's first batch issued before the phase's
// output flushes -- 36 spilled VGPRs, 0.712-0.716 vs 0.664 ms, profiles/archive/r04aa/; dword touches of
// the next phase's array -- -0.5% time for +27% FETCH_SIZE, profiles/archive/r04k/, archive/r04m/.)
// nontemporal hints on the staged input loads / the flushed output stores (both off: 0.727-0.730
// ms vs 0.712 for the 1M x 32 line, profiles/archive/r04j/)
constexpr bool kTbNtLoad = true;
constexpr bool kTbNtStore = true;
typedef double tb_d2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 tb_ld2(const double* p) {
  const tb_d2 v = kTbNtLoad ? __builtin_nontemporal_load(reinterpret_cast<const tb_d2*>(p))
                            : *reinterpret_cast<const tb_d2*>(p);
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void tb_st2(double* p, double x, double y) {
  tb_d2 v;
  v.x = x;
  v.y = y;
  if constexpr (kTbNtStore) __builtin_nontemporal_store(v, reinterpret_cast<tb_d2*>(p));
  else *reinterpret_cast<tb_d2*>(p) = v;
}  // per-lane sink slots after a wave buffer (FULL tiles' masked stores)

// A per-lane bit set hidden from the compiler: each phase re-derives its run-boundary
// compares from it instead of keeping 32 lane masks (64 SGPRs) alive across the tile.
__device__ __forceinline__ unsigned tb_bits(unsigned m) {
  asm volatile("" : "+v"(m));
  return m;
}

constexpr int kTbLpmWPE = 2;  // waves per SIMD (VGPR budget 256)
// GATHER kernels size their buffers for NP positions per lane; the 8-position body fits 128
// VGPRs, so four waves per SIMD (LDS: four workgroups of 4 x 4.2 KB per CU)
constexpr int tb_wpe(int np, bool gather) { return (gather && np == 8) ? 4 : kTbLpmWPE; }  // (EXOTIC: 2)
constexpr int tb_stage(int np, bool gather) { return gather ? 64 * np + 2 * np + 8 : kTbStage + kTbDump; }

// PART (STAGED launches): 1 = only FULL tiles, 2 = every other tile; 0 = all tiles, one body.
// (Both bodies in one kernel: 21 spilled VGPRs and 190 SGPRs, so two launches.)
// GATHER (market lists, round 5): a tile is 64 list entries, each lane's market row is copied
// into the wave's LDS buffer at row NP * lane by groups of NP / 4 lanes (4 agents each, one
// contiguous row segment per group: coalesced like the contiguous staging) and the outputs
// leave the same way; the general body then runs over NP positions -- a length-bucketed plan
// (batch.tiebreak_plan: buckets of <= 8, 9..16, 17..32 agents) no longer walks 32 positions
// for a 5-agent market (verdict r04 item 5).
template <bool STAGED, bool EXOTIC, int PART = 0, int NP = kTbLpmMax, bool GATHER = false>
__global__ __launch_bounds__(64 * kTbLpmWaves) __attribute__((amdgpu_waves_per_eu(tb_wpe(NP, GATHER && !EXOTIC), tb_wpe(NP, GATHER && !EXOTIC)))) void tiebreak_lpm_kernel(TbArgs a, const int32_t* list,
                                                                         int64_t n_list, int* fault) {
  static_assert(PART == 0 || (STAGED && !EXOTIC), "FULL / rest split: staged kernels only");
  static_assert(!GATHER || (STAGED && PART == 0), "gather staging: staged general body only");
  static_assert(NP == kTbLpmMax || GATHER, "fewer positions: gathered rows only");
  static_assert(NP == 8 || NP == 16 || NP == 32, "positions per lane");
  // one buffer per wave (16.9 KB; two workgroups of four waves per CU)
  __shared__ double sBuf[STAGED ? kTbLpmWaves : 1][STAGED ? tb_stage(NP, GATHER) : 1];
  // GATHER: every lane's row start and length, for the row-segment copies
  __shared__ int64_t sRowOff[GATHER ? kTbLpmWaves : 1][GATHER ? 64 : 1];
  __shared__ int sRowN[GATHER ? kTbLpmWaves : 1][GATHER ? 64 : 1];
  // FULL tiles: RN(1 / c) for group sizes c = 1..32 (tb_div_small)
  constexpr bool kFullBody = PART == 1;
  constexpr bool kRcTab = STAGED;  // group means via the reciprocal table
  __shared__ double sRc[kRcTab ? kTbLpmMax + 1 : 1];
  if constexpr (kRcTab) {
    if (threadIdx.x <= (unsigned)kTbLpmMax) sRc[threadIdx.x] = 1.0 / (double)(threadIdx.x ? threadIdx.x : 1);
    __syncthreads();
  }
  const int lane = lane_id();
  const int wv = STAGED ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;  // uniform: LDS bases in SGPRs
  double* const buf = sBuf[wv];
  int32_t* const ibuf = reinterpret_cast<int32_t*>(buf);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // a tile's metadata: this lane's market and the tile's agent range [B, B + cnt)
  struct Meta {
    int64_t m, off;
    int n;
    bool has;
    int64_t B;
    int cnt;
    int skip;  // 0 process, 1 every market empty, 2 a market longer than kTbLpmMax inside
    bool full;  // every lane holds a market of exactly kTbLpmMax agents
  };
  // PART 1: the next tile's two offsets per lane are loaded while this tile's confidences are
  // processed (kTbPrefetchMeta), so its meta costs no round trip of its own
  int64_t pre_o0 = 0, pre_o1 = 0;
  bool pre = false;
  auto meta_pre = [&](int64_t tile) {
    const int64_t li = tile * 64 + lane;
    const bool h = tile * 64 < n_list && li < n_list;
    pre_o0 = h ? a.offsets[li] : 0;
    pre_o1 = h ? a.offsets[li + 1] : 0;
    pre = true;
  };
  auto meta_of = [&](int64_t tile) -> Meta {
    Meta t{};
    const int64_t li = tile * 64 + lane;
    t.has = tile * 64 < n_list && li < n_list;
    t.m = t.has ? (list ? (int64_t)list[li] : li) : 0;
    if (kFullBody && pre) {  // (STAGED: m = li)
      t.off = pre_o0;
      t.n = (int)(pre_o1 - pre_o0);
      pre = false;
    } else {
      t.off = t.has ? a.offsets[t.m] : 0;
      t.n = t.has ? (int)(a.offsets[t.m + 1] - t.off) : 0;
    }
    if (ballot(t.n > NP || t.n < 0)) {
      raise_fault(fault, kFaultTooLong);
      if (t.n > NP || t.n < 0) t.n = 0;
    }
    if (!ballot(t.n > 0)) {
      t.skip = 1;
      return t;
    }
    if constexpr (GATHER) return t;  // rows are copied one by one: no tile range
    // STAGED: the tile's agents [B, E) (lane 0's market starts it, the last lane's ends it)
    t.B = ((int64_t)__builtin_amdgcn_readfirstlane((int)(t.off >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)t.off);
    const int last_lane = 63 - __builtin_clzll(ballot(t.has));
    const int64_t endl = t.off + t.n;
    const int64_t E = ((int64_t)__builtin_amdgcn_readlane((int)(endl >> 32), last_lane) << 32) |
                      (uint32_t)__builtin_amdgcn_readlane((int)endl, last_lane);
    t.cnt = (int)(E - t.B);  // <= 64 * 32 unless a market inside [B, E) was too long
    // (PART 1 launches only with 16-B aligned arrays, so an even B aligns every row load)
    t.full = ballot(t.has && t.n == kTbLpmMax) == ~0ull && (t.B & 1) == 0;
    // a market longer than kTbLpmMax (already faulted and zeroed above) still lies inside
    // [B, E): staging the range would run past this wave's buffer, so the tile is skipped
    // (every market gets the empty marker; the fault word reports the call as failed)
    if (STAGED && (E - t.B > 64 * kTbLpmMax || E < t.B)) {
      raise_fault(fault, kFaultTooLong);
      t.skip = 2;
    }
    return t;
  };
  Meta cur{};
  // PART 2 has nothing to do when PART 1 found every tile full (the common uniform batch):
  // it then only counts itself out
  bool run = true;
  // (one word per wave: a single flag word took every skipping wave's store through the
  // device-coherent path to one address -- 0.55 ms of serialised stores on a ragged batch)
  // Words are shared round-robin by launch pairs (capi.hip split_slot), possibly on other
  // streams: PART 1 raises its word to its ticket with atomicMax, and PART 2 runs when the word
  // holds its own ticket or a NEWER pair's (then it may run for nothing -- it skips FULL tiles
  // itself -- but never skips a tile its own PART 1 left).  Tickets are positive and
  // increase; after a wrap split_slot clears the slot before the first pair that reuses it.
  if constexpr (PART == 2) run = a.split[wave] >= a.ticket;
  bool left = false;  // PART 1: this wave left a tile to PART 2
  for (int64_t tile = wave; run && tile * 64 < n_list; tile += nwaves) {
    cur = meta_of(tile);
    if constexpr (PART == 1) {
      if (!cur.full) {  // (skipped tiles are never full)
        left = true;
        continue;
      }
    } else if constexpr (PART == 2) {
      if (cur.full) continue;
    }
    const int64_t m = cur.m, off = cur.off;
    const bool has = cur.has;
    const int n = cur.n;
    if (cur.skip) {
      if (has) {
        a.winner[m] = 0.0; a.label[m] = -1; a.n_groups[m] = -1; a.variance[m] = 0.0;
      }
      continue;
    }
    const int64_t B = cur.B;
    const int cnt_tile = cur.cnt;
    // this lane's row in the staged buffer (GATHER: a fixed row of NP slots per lane)
    const int lrow = GATHER ? NP * lane : (int)(off - B);
    if constexpr (GATHER) {
      wave_sync_lds();  // the previous tile's row table readers are done
      sRowOff[wv][lane] = off;
      sRowN[wv][lane] = n;
      wave_sync_lds();
    }
    // GATHER: row r's agents [0, cnt) <-> global [off_r, off_r + cnt) as 16-B aligned pairs:
    // NP / 2 lanes per row, lane c of a row owns the pair starting at agent 2c - (off_r & 1)
    // (the row's aligned start), 64 / (NP / 2) rows per pass, NP / 2 passes -- one 16-B access
    // per lane and pass, as many as the contiguous staging of a full tile.  A 32-agent row
    // starting at an odd agent has one agent past its last pair (`tail`).  body(r, i, ro, rn)
    // gets the row's agent index i of the pair's first element (-1 .. NP - 1).
    constexpr int kGL = NP / 2, kGR = 64 / kGL;
    auto rows_copy = [&](auto&& body) {
#pragma unroll 4
      for (int pass = 0; pass < kGL; ++pass) {
        const int r = pass * kGR + lane / kGL, c = lane % kGL;
        const int64_t ro = sRowOff[wv][r];
        body(r, 2 * c - (int)(ro & 1), ro, sRowN[wv][r]);
      }
    };
    auto rows_tail = [&](auto&& body) {  // agent NP of an odd-start NP-agent row, one lane each
      const int r = lane;
      const int64_t ro = sRowOff[wv][r];
      if ((ro & 1) && sRowN[wv][r] == NP) body(r, NP - 1, ro);
    };
    // every lane reads inside its own row (positions past n re-read the last agent); a lane
    // with an empty market reads the tile's first agent (masked later)
    const int last = n > 0 ? n - 1 : 0;
    const int rbase = n > 0 ? lrow : 0;
    const int64_t gbase = n > 0 ? off : B;
    // global [B, E) -> LDS (padded), coalesced 16-B loads issued kTbStageBatch at a time
    // before any is written to LDS: one memory round trip per batch, not one per load (the
    // per-iteration loop paid ~16 serial HBM latencies per array and tile)
    auto stage = [&](const double* src) {
      wave_sync_lds();  // the buffer's previous readers (this wave) are done
      if constexpr (GATHER) {
        // kTbGatherBatch passes' loads issued before any is written to LDS: the loads are
        // unconditional (a pair outside its row reads agent 0 of the array, never used), so
        // they leave back to back -- one memory round trip per batch instead of one per pass
        constexpr int K = kGL < kTbGatherBatch ? kGL : kTbGatherBatch;
#pragma unroll 1
        for (int p0 = 0; p0 < kGL; p0 += K) {
          double2 v[K];
          int rr[K], ii[K], nn[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const int r = (p0 + k) * kGR + lane / kGL, c = lane % kGL;
            const int64_t ro = sRowOff[wv][r];
            const int rn = sRowN[wv][r];
            const int i = 2 * c - (int)(ro & 1);
            const bool touch = i + 1 >= 0 && i < rn;  // the pair [i, i + 1] touches the row
            v[k] = tb_ld2(src + (touch ? ro + i : 0));  // 16-B aligned: ro + i is even
            rr[k] = r;
            ii[k] = i;
            nn[k] = touch ? rn : 0;
          }
#pragma unroll
          for (int k = 0; k < K; ++k) {
            if (ii[k] >= 0 && ii[k] < nn[k]) buf[tb_pad(NP * rr[k] + ii[k])] = v[k].x;
            if (ii[k] + 1 >= 0 && ii[k] + 1 < nn[k]) buf[tb_pad(NP * rr[k] + ii[k] + 1)] = v[k].y;
          }
        }
        rows_tail([&](int r, int i, int64_t ro) { buf[tb_pad(NP * r + i)] = src[ro + i]; });
        wave_sync_lds();
        return;
      }
      if (((uintptr_t)(src + B) & 15) == 0) {
#pragma unroll 1
        for (int k0 = 0; k0 < kTbStageIt; k0 += kTbStageBatch) {
          if (k0 * 128 >= cnt_tile) break;  // wave-uniform
          double2 v[kTbStageBatch];
#pragma unroll
          for (int k = 0; k < kTbStageBatch; ++k) {
            const int e = 2 * lane + 128 * (k0 + k);
            v[k] = make_double2(0.0, 0.0);
            if (e + 1 < cnt_tile) v[k] = tb_ld2(src + B + e);
          }
#pragma unroll
          for (int k = 0; k < kTbStageBatch; ++k) {
            const int e = 2 * lane + 128 * (k0 + k);
            if (e + 1 < cnt_tile) {
              buf[tb_pad(e)] = v[k].x;
              buf[tb_pad(e + 1)] = v[k].y;
            }
          }
        }
        if ((cnt_tile & 1) && lane == 0) buf[tb_pad(cnt_tile - 1)] = src[B + cnt_tile - 1];  // odd tail
      } else {
#pragma unroll 1
        for (int k0 = 0; k0 < 2 * kTbStageIt; k0 += 2 * kTbStageBatch) {
          if (k0 * 64 >= cnt_tile) break;  // wave-uniform
          double v[2 * kTbStageBatch];
#pragma unroll
          for (int k = 0; k < 2 * kTbStageBatch; ++k) {
            const int e = lane + 64 * (k0 + k);
            v[k] = 0.0;
            if (e < cnt_tile) v[k] = src[B + e];
          }
#pragma unroll
          for (int k = 0; k < 2 * kTbStageBatch; ++k) {
            const int e = lane + 64 * (k0 + k);
            if (e < cnt_tile) buf[tb_pad(e)] = v[k];
          }
        }
      }
      wave_sync_lds();
    };
    // FULL tiles (2048 agents): no bounds checks, NB 16-B loads per lane in flight
    auto stage_full = [&](const double* src, auto nb) {
      constexpr int NB = decltype(nb)::value;  // (src + B is 16-B aligned: see Meta::full)
      wave_sync_lds();
#pragma unroll 1
      for (int k0 = 0; k0 < kTbStageIt; k0 += NB) {
        double2 v[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) v[k] = tb_ld2(src + B + 2 * lane + 128 * (k0 + k));
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int e = 2 * lane + 128 * (k0 + k);
          buf[tb_pad(e)] = v[k].x;
          buf[tb_pad(e + 1)] = v[k].y;
        }
      }
      wave_sync_lds();
    };
    // LDS (padded) -> global [B, E), coalesced 16-B stores
    auto flush = [&](double* dst) {
      wave_sync_lds();
      if constexpr (GATHER) {
        // a pair wholly inside the row leaves as one 16-B store; a pair the row shares with
        // its neighbour writes only its own agent
        rows_copy([&](int r, int i, int64_t ro, int rn) {
          if (i >= 0 && i + 1 < rn) {
            tb_st2(dst + ro + i, buf[tb_pad(NP * r + i)], buf[tb_pad(NP * r + i + 1)]);
          } else {
            if (i >= 0 && i < rn) dst[ro + i] = buf[tb_pad(NP * r + i)];
            if (i + 1 >= 0 && i + 1 < rn) dst[ro + i + 1] = buf[tb_pad(NP * r + i + 1)];
          }
        });
        rows_tail([&](int r, int i, int64_t ro) { dst[ro + i] = buf[tb_pad(NP * r + i)]; });
        wave_sync_lds();
        return;
      }
      const bool al = ((uintptr_t)(dst + B) & 15) == 0;
      for (int e = 2 * lane; e < cnt_tile; e += 128) {
        if (al && e + 1 < cnt_tile) {
          tb_st2(dst + B + e, buf[tb_pad(e)], buf[tb_pad(e + 1)]);
        } else {
          dst[B + e] = buf[tb_pad(e)];
          if (e + 1 < cnt_tile) dst[B + e + 1] = buf[tb_pad(e + 1)];
        }
      }
      wave_sync_lds();  // the buffer's next writers (this wave) come after these reads
    };
    auto flush_i32 = [&](int32_t* dst) {
      wave_sync_lds();
      if constexpr (GATHER) {
        rows_copy([&](int r, int i, int64_t ro, int rn) {
          if (i >= 0 && i < rn) dst[ro + i] = ibuf[tb_pad(NP * r + i)];
          if (i + 1 >= 0 && i + 1 < rn) dst[ro + i + 1] = ibuf[tb_pad(NP * r + i + 1)];
        });
        rows_tail([&](int r, int i, int64_t ro) { dst[ro + i] = ibuf[tb_pad(NP * r + i)]; });
        wave_sync_lds();
        return;
      }
      const bool al = ((uintptr_t)(dst + B) & 15) == 0;
      for (int e = 4 * lane; e < cnt_tile; e += 256) {
        if (al && e + 3 < cnt_tile) {
          *reinterpret_cast<int4*>(dst + B + e) =
              make_int4(ibuf[tb_pad(e)], ibuf[tb_pad(e + 1)], ibuf[tb_pad(e + 2)], ibuf[tb_pad(e + 3)]);
        } else {
          for (int q = 0; q < 4 && e + q < cnt_tile; ++q) dst[B + e + q] = ibuf[tb_pad(e + q)];
        }
      }
      wave_sync_lds();  // (as flush: the int32 reads are fenced before the next double writes)
    };
    // agent t of this lane's market
    auto at = [&](const double* src, int t) -> double {
      if constexpr (STAGED) return buf[tb_pad(rbase + t)];
      else return src[gbase + t];
    };
    // this lane's slot g (an agent's or a group's output)
    auto put = [&](double* dst, int g, double v) {
      if constexpr (STAGED) buf[tb_pad(lrow + g)] = v;
      else dst[off + g] = v;
    };
    auto put_i32 = [&](int32_t* dst, int g, int v) {
      if constexpr (STAGED) ibuf[tb_pad(lrow + g)] = v;
      else dst[off + g] = v;
    };
    const double nd = (double)(n > 0 ? n : 1);
    // a group mean: the reciprocal-table quotient where the table exists, else IEEE division
    auto tb_div_cnt = [&](double x, int c, const double* tab) -> double {
      if constexpr (kRcTab) return tb_div_small(x, c, tab);
      else return x / (double)c;
    };

    // ---- FULL tile: 64 markets of exactly kTbLpmMax agents, lane L's row at 33 L ------------
    // The same four phases as below with n a compile-time 32: no per-position validity masks,
    // row reads at immediate offsets (or one shift-add for a sorted position), and every
    // conditional store a store to a selected address (the lane's sink slot when masked).
    if constexpr (kFullBody) {
      {
        constexpr int N = kTbLpmMax;
        double* row = buf + 33 * lane;
        int32_t* irow = ibuf + 33 * lane;
        double* sink = buf + kTbStage + lane;
        int32_t* isink = ibuf + 2 * kTbStage + lane;
        auto put_sel = [&](unsigned bits, int p, unsigned g, double v) {
          *(((bits >> p) & 1u) ? row + g : sink) = v;
        };
        auto put_sel_i32 = [&](unsigned bits, int p, unsigned g, int v) {
          *(((bits >> p) & 1u) ? irow + g : isink) = v;
        };
        unsigned u[N];
        // each phase re-derives its row addresses from u (CSE across phases kept 64 address
        // registers alive through the tile and spilled)
        auto refresh_u = [&]() {
#pragma unroll
          for (int p = 0; p < N; ++p) u[p] = tb_bits(u[p]);
        };
        // 1. keys, first-seen ordinals, sort
        stage_full(a.pred, std::integral_constant<int, kTbFullBatchPC>{});
        double kp[N];  // (PART 1 runs only for round mode 0, see launch_tb_short)
#pragma unroll
        for (int t = 0; t < N; ++t) {
          bool slow;
          kp[t] = py_round_nd_fast(row[t], a.rscale, a.rinv, a.rthresh, slow);
          if (ballot(slow)) kp[t] = slow ? py_round_nd_sel(row[t], a.rscale, a.rinv, a.rthresh) : kp[t];
        }
        int ngf = 0;
        {
          int go[N];
#pragma unroll
          for (int t = 0; t < N; ++t) {
            int g = -1;
#pragma unroll
            for (int s2 = 0; s2 < t; ++s2) g = key_eq(kp[s2], kp[t]) ? go[s2] : g;
            go[t] = g < 0 ? ngf : g;
            ngf += g < 0 ? 1 : 0;
            u[t] = ((unsigned)go[t] << 5) | (unsigned)t;
          }
          if (a.g_of) {
            wave_sync_lds();
#pragma unroll
            for (int t = 0; t < N; ++t) irow[t] = go[t];
            flush_i32(a.g_of);
          }
        }
        // run boundaries: bit p of stm / enm = a run starts / ends at sorted position p
        unsigned stm = 1u, enm = 1u << (N - 1);
        if constexpr (kTbFullKeysInLds) {
          // the rounded keys wait in the lane's row while only the 32-bit (ordinal, agent)
          // keys go through the network; each sorted position then reads its run head's key
          wave_sync_lds();
#pragma unroll
          for (int t = 0; t < N; ++t) row[t] = kp[t];
          oem_sort(u);
#pragma unroll
          for (int p = 1; p < N; ++p) {
            const unsigned d = ((u[p] >> 5) != (u[p - 1] >> 5)) ? 1u : 0u;
            stm |= d << p;
            enm |= d << (p - 1);
          }
          unsigned ht = u[0] & 31u;
          kp[0] = row[ht];
#pragma unroll
          for (int p = 1; p < N; ++p) {
            ht = ((stm >> p) & 1u) ? (u[p] & 31u) : ht;
            kp[p] = row[ht];
          }
        } else {
          oem_sort_kv(u, kp);
#pragma unroll
          for (int p = 1; p < N; ++p) {
            const unsigned d = ((u[p] >> 5) != (u[p - 1] >> 5)) ? 1u : 0u;
            stm |= d << p;
            enm |= d << (p - 1);
          }
#pragma unroll
          for (int p = 1; p < N; ++p) kp[p] = ((stm >> p) & 1u) ? kp[p] : kp[p - 1];  // run head's key
        }
        // 2. group keys and counts
        if (a.g_key) {
          wave_sync_lds();
          const unsigned en_ = tb_bits(enm);
          refresh_u();
#pragma unroll
          for (int p = 0; p < N; ++p) put_sel(en_, p, u[p] >> 5, kp[p]);
          flush(a.g_key);
        }
        if (a.g_count) {
          wave_sync_lds();
          const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
          refresh_u();
          int cnt = 0;
#pragma unroll
          for (int p = 0; p < N; ++p) {
            cnt = (((st_ >> p) & 1u) ? 0 : cnt) + 1;
            put_sel_i32(en_, p, u[p] >> 5, cnt);
          }
          flush_i32(a.g_count);
        }
        // 3. densities
        double densp[N];
        stage_full(a.weight, std::integral_constant<int, kTbFullBatchWR>{});
        {
          const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
          refresh_u();
          double tot = 0.0;
          int cnt = 0;
#pragma unroll
          for (int p = 0; p < N; ++p) {
            const bool st = (st_ >> p) & 1u;
            tot = (st ? 0.0 : tot) + row[u[p] & 31u];  // tiebreak.py:60, sum from int 0
            cnt = (st ? 0 : cnt) + 1;
            densp[p] = tb_div_small(tot, cnt, sRc);
            put_sel(en_, p, u[p] >> 5, densp[p]);
          }
          if (a.g_density) flush(a.g_density);
        }
        // 4. max reliability per group, the winner and the tie flag
        double bd = 0.0, bm = 0.0, bk = 0.0;
        bool tie = false;
        stage_full(a.rel, std::integral_constant<int, kTbFullBatchWR>{});
        {
          const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
          refresh_u();
          double mx = 0.0;
#pragma unroll
          for (int p = 0; p < N; ++p) {
            const unsigned g = u[p] >> 5;
            const double r = row[u[p] & 31u];
            mx = ((st_ >> p) & 1u) ? r : ((r > mx) ? r : mx);  // tiebreak.py:62
            put_sel(en_, p, g, mx);
            const bool en = (en_ >> p) & 1u;
            const double dens = densp[p];
            const bool same = (dens == bd) && (mx == bm);
            const bool better = (g == 0) | tb_better_sel(dens, mx, kp[p], bd, bm, bk);  // tiebreak.py:113-117
            tie = en ? (better ? ((g != 0) && same) : (tie || same)) : tie;     // tiebreak.py:123-133
            const bool upd = en && better;
            bd = upd ? dens : bd;
            bm = upd ? mx : bm;
            bk = upd ? kp[p] : bk;
          }
          if (a.g_maxrel) flush(a.g_maxrel);
        }
        // 5. variance (input order), per-group mean confidences
        stage_full(a.conf, std::integral_constant<int, kTbFullBatchPC>{});
        if (kTbPrefetchMeta && (tile + nwaves) * 64 < n_list) meta_pre(tile + nwaves);
        double variance;
        {
          double cs = 0.0;
#pragma unroll
          for (int t = 0; t < N; ++t) cs += row[t];
          const double mean = cs / (double)N;
          // squares summed as they come (no array of 32): the fast square is exact unless
          // flagged; a lane with a flagged square redoes the ordered sum with exact ones
          wave_sync_lds();  // re-read the confidences instead of holding all 32
          double vs = 0.0;
          unsigned slow = 0;
#pragma unroll
          for (int t = 0; t < N; ++t) {
            bool ok;
            vs += bce_pow::pow2_fast(row[t] - mean, ok);
            slow |= ok ? 0u : (1u << t);
          }
          if (slow) {
            vs = 0.0;
#pragma unroll 1
            for (int t = 0; t < N; ++t) {
              const double d = row[t] - mean;
              bool ok;
              const double q = bce_pow::pow2_fast(d, ok);
              vs += ((slow >> t) & 1u) ? tb_pow2_full(d) : q;
            }
          }
          variance = vs / (double)N;
        }
        if (a.g_avgconf) {
          const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
          refresh_u();
          double gcs = 0.0;
          int cnt = 0;
#pragma unroll
          for (int p = 0; p < N; ++p) {
            const bool st = (st_ >> p) & 1u;
            gcs = (st ? 0.0 : gcs) + row[u[p] & 31u];  // tiebreak.py:61
            cnt = (st ? 0 : cnt) + 1;
            put_sel(en_, p, u[p] >> 5, tb_div_small(gcs, cnt, sRc));
          }
          flush(a.g_avgconf);
        }
        a.winner[m] = bk;
        a.label[m] = (ngf == 1) ? BCE_TB_UNANIMOUS : tie ? BCE_TB_PREDICTION_VALUE_SMALLEST : BCE_TB_WEIGHT_DENSITY;
        a.n_groups[m] = ngf;
        a.variance[m] = variance;
        continue;
      }
    }

    // ---- 1. keys, group ordinals (first-seen order), sort with the key as payload ---------
    // Per-lane validity is the bit set vm (bit t: t < n) and run boundaries are stm / enm
    // (bit p: a run starts / ends at sorted position p), each re-derived per phase through an
    // empty asm: kept as 32 lane masks they held 64 SGPRs through the tile and spilled.
    unsigned u[NP];
    double kp[NP];
    int ng = 0;
    const unsigned vm = (n >= NP) ? ~0u : ((1u << (n > 0 ? n : 0)) - 1u);
    auto vbit = [](unsigned bits, int p) { return ((bits >> p) & 1u) != 0u; };
    auto refresh_ug = [&]() {
#pragma unroll
      for (int p = 0; p < NP; ++p) u[p] = tb_bits(u[p]);
    };
    if constexpr (STAGED) stage(a.pred);
    const double praw0 = at(a.pred, 0);  // a single agent keeps its raw prediction (tiebreak.py:89-96)
    {
      if (!EXOTIC && a.rmode == 0) {  // the common precisions: rint fast path, exact redo if flagged
#pragma unroll
        for (int t = 0; t < NP; ++t) {
          const double x = at(a.pred, min(t, last));
          bool slow;
          kp[t] = py_round_nd_fast(x, a.rscale, a.rinv, a.rthresh, slow);
          if (ballot(slow)) kp[t] = slow ? py_round_nd_sel(x, a.rscale, a.rinv, a.rthresh) : kp[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < NP; ++t) kp[t] = tb_round<EXOTIC>(at(a.pred, min(t, last)), a, n >= 2);
      }
      const unsigned vm1 = tb_bits(vm);
      int go[NP];
#pragma unroll
      for (int t = 0; t < NP; ++t) {
        int g = -1;
#pragma unroll
        for (int s2 = 0; s2 < t; ++s2) g = key_eq(kp[s2], kp[t]) ? go[s2] : g;  // earlier equal key: its group
        const bool fresh = vbit(vm1, t) && g < 0;
        go[t] = fresh ? ng : g;
        ng += fresh ? 1 : 0;
        u[t] = vbit(vm1, t) ? (((unsigned)go[t] << 5) | (unsigned)t) : 0xFFFFFFFFu;
      }
      if (a.g_of) {  // agent t's prediction (slot t) is consumed: the ordinals go in place
        if constexpr (STAGED) wave_sync_lds();
        const unsigned vm2 = tb_bits(vm);
#pragma unroll
        for (int t = 0; t < NP; ++t)
          if (vbit(vm2, t)) put_i32(a.g_of, t, go[t]);
        if constexpr (STAGED) flush_i32(a.g_of);
      }
    }
    // STAGED (kTbGeneralKeysInLds): as the FULL body, only the 32-bit (ordinal, agent) keys go
    // through the network; the rounded keys wait in the lane's row (the predictions are
    // consumed) and each sorted position reads its run head's key back
    if constexpr (STAGED && kTbGeneralKeysInLds) {
      wave_sync_lds();  // the row's readers (keys, g_of flush) are done
      const unsigned vm3 = tb_bits(vm);
#pragma unroll
      for (int t = 0; t < NP; ++t)
        if (vbit(vm3, t)) buf[tb_pad(lrow + t)] = kp[t];
      wave_sync_lds();
      oem_sort(u);
    } else {
      oem_sort_kv(u, kp);
    }
    // run boundaries from the sorted keys alone (invalid positions hold 0xFFFFFFFF, sorted
    // last: the last valid position ends its run, no invalid position ends one)
    unsigned stm = 1u, enm = (u[NP - 1] != 0xFFFFFFFFu) ? (1u << (NP - 1)) : 0u;
#pragma unroll
    for (int p = 1; p < NP; ++p) {
      const unsigned d = ((u[p] >> 5) != (u[p - 1] >> 5)) ? 1u : 0u;
      stm |= d << p;
      enm |= d << (p - 1);
    }
    enm &= vm;
    // every member carries its run head's key: a group's dict key is its FIRST member's
    // rounded prediction (tiebreak.py:54-55), and -0.0 / 0.0 share a group with different bits
    if constexpr (STAGED && kTbGeneralKeysInLds) {
      // (an invalid position's head index is clamped into the lane's row: never used)
      unsigned ht = u[0] & (unsigned)(NP - 1);
      kp[0] = buf[tb_pad(lrow + (int)ht)];
#pragma unroll
      for (int p = 1; p < NP; ++p) {
        ht = vbit(stm, p) ? (u[p] & (unsigned)(NP - 1)) : ht;
        kp[p] = buf[tb_pad(lrow + (int)ht)];
      }
    } else {
#pragma unroll
      for (int p = 1; p < NP; ++p) kp[p] = vbit(stm, p) ? kp[p] : kp[p - 1];
    }

    // ---- 2. group keys and counts (registers only) ------------------------------------------
    if (a.g_key || a.g_count) {
      if (a.g_key) {
        const unsigned en_ = tb_bits(enm);
        refresh_ug();
#pragma unroll
        for (int p = 0; p < NP; ++p)
          if (vbit(en_, p)) put(a.g_key, (int)(u[p] >> 5), (n == 1) ? praw0 : kp[p]);
        if constexpr (STAGED) flush(a.g_key);
      }
      if (a.g_count) {
        if constexpr (STAGED) wave_sync_lds();
        const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
        refresh_ug();
        int cnt = 0;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          cnt = (vbit(st_, p) ? 0 : cnt) + 1;
          if (vbit(en_, p)) put_i32(a.g_count, (int)(u[p] >> 5), cnt);
        }
        if constexpr (STAGED) flush_i32(a.g_count);
      }
    }

    // ---- 3. weights: group densities, kept per run end for the winner -----------------------
    // A group's outputs overwrite slot g of its market's row in place: group g ends only after
    // every group <= g, and agent g (ordinal <= g) belongs to one of those -- consumed.
    // (Positions past n read slot min(31, ...) of the lane's row or the tile's slack: never used.)
    double densp[NP];
    if constexpr (STAGED) stage(a.weight);
    {
      const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
      refresh_ug();
      double tot = 0.0;
      int cnt = 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int t = min((int)(u[p] & 31u), last);
        const bool st = vbit(st_, p);
        tot = (st ? 0.0 : tot) + at(a.weight, t);  // tiebreak.py:60, sum from int 0
        cnt = (st ? 0 : cnt) + 1;
        densp[p] = tb_div_cnt(tot, cnt, sRc);
        if (vbit(en_, p) && a.g_density) put(a.g_density, (int)(u[p] >> 5), densp[p]);
      }
      if constexpr (STAGED) {
        if (a.g_density) flush(a.g_density);
      }
    }

    // ---- 4. reliabilities: max per group (first maximum kept), the winner ------------------
    double bd = 0.0, bm = 0.0, bk = 0.0;
    bool tie = false;
    if constexpr (STAGED) stage(a.rel);
    {
      const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
      refresh_ug();
      double mx = 0.0;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int t = min((int)(u[p] & 31u), last);
        const unsigned g = u[p] >> 5;
        const double r = at(a.rel, t);
        mx = vbit(st_, p) ? r : ((r > mx) ? r : mx);  // tiebreak.py:62
        if (vbit(en_, p)) {
          if (a.g_maxrel) put(a.g_maxrel, (int)g, mx);
          const double key = (n == 1) ? praw0 : kp[p], dens = densp[p];
          const bool same = (dens == bd) && (mx == bm);
          if (g == 0 || tb_better(dens, mx, key, bd, bm, bk)) {  // tiebreak.py:113-117
            tie = (g != 0) && same;
            bd = dens; bm = mx; bk = key;
          } else {
            tie = tie || same;  // tiebreak.py:123-133: does another group tie the winner?
          }
        }
      }
      if constexpr (STAGED) {
        if (a.g_maxrel) flush(a.g_maxrel);
      }
    }

    // ---- 5. confidences: variance (input order), then the per-group means -----------------
    if constexpr (STAGED) stage(a.conf);
    double variance;
    {
      const unsigned vm5 = tb_bits(vm);
      double cs = 0.0;
#pragma unroll
      for (int t = 0; t < NP; ++t) cs += vbit(vm5, t) ? at(a.conf, min(t, last)) : 0.0;
      const double mean = cs / nd;
      // squares: pow(d, 2.0) restated (glibc_pow.hpp), summed as they come; a lane with a
      // near-midpoint square (a bit in `slow`) redoes its ordered sum with the exact ones
      if constexpr (STAGED) wave_sync_lds();  // re-read the confidences instead of holding them
      const unsigned vm6 = tb_bits(vm);
      double vs = 0.0;
      unsigned slow = 0;
#pragma unroll
      for (int t = 0; t < NP; ++t) {
        bool ok;
        const double q = bce_pow::pow2_fast(at(a.conf, min(t, last)) - mean, ok);
        vs += vbit(vm6, t) ? q : 0.0;
        slow |= (vbit(vm6, t) && !ok) ? (1u << t) : 0u;
      }
      if (slow) {
        vs = 0.0;
#pragma unroll 1
        for (int t = 0; t < n; ++t) {
          const double d = at(a.conf, t) - mean;
          bool ok;
          const double q = bce_pow::pow2_fast(d, ok);
          vs += ((slow >> t) & 1u) ? tb_pow2_full(d) : q;
        }
      }
      variance = vs / nd;
    }
    if (a.g_avgconf) {
      const unsigned st_ = tb_bits(stm), en_ = tb_bits(enm);
      refresh_ug();
      double gcs = 0.0;
      int cnt = 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const bool st = vbit(st_, p);
        gcs = (st ? 0.0 : gcs) + at(a.conf, min((int)(u[p] & 31u), last));  // tiebreak.py:61
        cnt = (st ? 0 : cnt) + 1;
        if (vbit(en_, p)) put(a.g_avgconf, (int)(u[p] >> 5), tb_div_cnt(gcs, cnt, sRc));
      }
      if constexpr (STAGED) flush(a.g_avgconf);
    }
    if (has) {
      if (n == 0) {  // tiebreak.py:86-87 (ValueError)
        a.winner[m] = 0.0; a.label[m] = -1; a.n_groups[m] = -1; a.variance[m] = 0.0;
      } else {
        a.winner[m] = bk;
        a.label[m] = (n == 1) ? BCE_TB_SINGLE_AGENT
                              : (ng == 1) ? BCE_TB_UNANIMOUS
                                          : tie ? BCE_TB_PREDICTION_VALUE_SMALLEST : BCE_TB_WEIGHT_DENSITY;
        a.n_groups[m] = ng;
        a.variance[m] = (n == 1) ? 0.0 : variance;
      }
    }
  }
  if (PART == 1 && left && lane == 0) atomicMax(&a.split[wave], a.ticket);
}

// n > 64: one workgroup per market.  (rounded key, index) pairs are bitonic-sorted in
// LDS (n <= 4096) or in the workgroup's slice of a global scratch buffer (any length:
// the reference has no limit), so every group is a run whose members appear in input
// order; the run head owns the group (its first member is the dict-insertion leader).
constexpr int kTbThreads = 256;
constexpr int kTbMax = 4096;
constexpr unsigned long long kNanKey = 0xFFFFFFFFFFFFF000ull;

// (Round 6, VERDICT r05 item 4: FULL tiles on a quad of lanes per market -- 4 lanes x 8 agents,
// 16 markets per wave, rows loaded straight into registers, O(n^2) leader search over the LDS row,
// a quad-wide bitonic sort, every ordered chain run as four seeded passes -- parity green but
// 1.46-1.49 ms against 0.663-0.665 ms for this lane-per-market FULL body on the same box
// (profiles/r06p/; 128 VGPRs, 4 waves per SIMD): the per-market sequential chains cost four
// instruction slots per market instead of one and the leader search 2.7x the compares.  Removed;
// the kernel is in git history, commit "Tie-break: quad-of-lanes-per-market FULL kernel".)

template <bool IN_LDS, bool EXOTIC>
__global__ __launch_bounds__(kTbThreads) void tiebreak_block_kernel(TbArgs a, const int32_t* list,
                                                                    int64_t n_list, void* scratch,
                                                                    int64_t stride) {
  __shared__ unsigned long long lk[IN_LDS ? kTbMax : 1];
  __shared__ int32_t lIdx[IN_LDS ? kTbMax : 1];
  __shared__ int32_t lRank[IN_LDS ? kTbMax : 1];
  // global slice: keys (8 B), indices, ranks (4 B each) of `stride` entries per workgroup
  unsigned long long* const sk =
      IN_LDS ? lk : reinterpret_cast<unsigned long long*>(scratch) + (int64_t)blockIdx.x * 2 * stride;
  int32_t* const sIdx = IN_LDS ? lIdx : reinterpret_cast<int32_t*>(sk + stride);
  int32_t* const sRank = IN_LDS ? lRank : sIdx + stride;
  __shared__ double cD[kTbThreads], cM[kTbThreads], cK[kTbThreads];
  __shared__ int32_t cI[kTbThreads];
  __shared__ int32_t sW[kTbThreads / 64 + 1];
  __shared__ int32_t sFlag;
  __shared__ double sVar;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wv = tid >> 6;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t li = blockIdx.x; li < n_list; li += gridDim.x) {
    const int64_t m = list[li];
    const int64_t off = a.offsets[m];
    const int n = (int)(a.offsets[m + 1] - off);
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = tid; i < P; i += kTbThreads) {
      unsigned long long kk = ~0ull;
      if (i < n) {
        double k = tb_round<EXOTIC>(a.pred[off + i], a);
        if (k == 0.0) k = 0.0;  // -0.0 and 0.0 share one dict slot
        unsigned long long b = (unsigned long long)__double_as_longlong(k);
        kk = (b >> 63) ? ~b : (b | 0x8000000000000000ull);  // total order on doubles
        if (k != k) kk = kNanKey;                            // NaN never equals: own group
        sRank[i] = 0;
      }
      sk[i] = kk;
      sIdx[i] = i;
    }
    if (tid == 0) sFlag = 0;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int c = tid; c < (P >> 1); c += kTbThreads) {
          const int lo = ((c & ~(j - 1)) << 1) | (c & (j - 1));
          const int hi = lo | j;
          const bool up = (lo & k) == 0;
          const unsigned long long x = sk[lo], y = sk[hi];
          const int xi = sIdx[lo], yi = sIdx[hi];
          const bool gt = (x > y) || (x == y && xi > yi);
          if (gt == up) {
            sk[lo] = y; sk[hi] = x;
            sIdx[lo] = yi; sIdx[hi] = xi;
          }
        }
        __syncthreads();
      }
    }
    // run heads mark their leader (first-seen member) in original index space
    for (int t = tid; t < n; t += kTbThreads) {
      const bool head = (t == 0) || sk[t] == kNanKey || sk[t - 1] != sk[t];
      if (head) sRank[sIdx[t]] = 1;
    }
    __syncthreads();
    // exclusive scan of leader flags in original order -> first-seen group rank
    int carry = 0;
    for (int c0 = 0; c0 < n; c0 += kTbThreads) {
      const int i = c0 + tid;
      const bool f = (i < n) && sRank[i] != 0;
      const unsigned long long bm = ballot(f);
      if (lane == 0) sW[wv] = __popcll(bm);
      __syncthreads();
      int before = carry, chunk = 0;
      for (int q = 0; q < kTbThreads / 64; ++q) {
        if (q < wv) before += sW[q];
        chunk += sW[q];
      }
      if (i < n) sRank[i] = f ? before + __popcll(bm & below) : -1;
      carry += chunk;
      __syncthreads();
    }
    const int ng = carry;
    // group metrics by run heads (members in input order), winner candidates
    double bd = 0.0, bmx = 0.0, bk = 0.0;
    int bi = -1;
    for (int t = tid; t < n; t += kTbThreads) {
      const bool head = (t == 0) || sk[t] == kNanKey || sk[t - 1] != sk[t];
      if (!head) continue;
      const int i0 = sIdx[t];
      double tot = 0.0, cs = 0.0, mx = a.rel[off + i0];
      int cnt = 0;
      for (int q = t; q < n; ++q) {
        if (q > t && (sk[q] == kNanKey || sk[q] != sk[t])) break;
        const int iq = sIdx[q];
        if (a.g_of) a.g_of[off + iq] = sRank[i0];
        tot += a.weight[off + iq];
        cs += a.conf[off + iq];
        ++cnt;
        const double rq = a.rel[off + iq];
        if (q != t && rq > mx) mx = rq;
        if (sk[t] == kNanKey) break;
      }
      const double dens = tot / (double)cnt;
      const double key = tb_round<EXOTIC>(a.pred[off + i0], a);
      const int64_t g = off + sRank[i0];
      if (a.g_key) a.g_key[g] = key;
      if (a.g_count) a.g_count[g] = cnt;
      if (a.g_density) a.g_density[g] = dens;
      if (a.g_avgconf) a.g_avgconf[g] = cs / (double)cnt;
      if (a.g_maxrel) a.g_maxrel[g] = mx;
      if (bi < 0 || tb_better(dens, mx, key, bd, bmx, bk)) {
        bi = i0; bd = dens; bmx = mx; bk = key;
      }
    }
    cD[tid] = bd; cM[tid] = bmx; cK[tid] = bk; cI[tid] = bi;
    __syncthreads();
    for (int s = kTbThreads / 2; s > 0; s >>= 1) {
      if (tid < s && cI[tid + s] >= 0 &&
          (cI[tid] < 0 || tb_better(cD[tid + s], cM[tid + s], cK[tid + s], cD[tid], cM[tid], cK[tid]))) {
        cD[tid] = cD[tid + s]; cM[tid] = cM[tid + s]; cK[tid] = cK[tid + s]; cI[tid] = cI[tid + s];
      }
      __syncthreads();
    }
    const double wd = cD[0], wm = cM[0], wk = cK[0];
    const int wi = cI[0];
    // label: does another group tie the winner on (density, max_rel)?
    for (int t = tid; t < n; t += kTbThreads) {
      const bool head = (t == 0) || sk[t] == kNanKey || sk[t - 1] != sk[t];
      if (!head || sIdx[t] == wi) continue;
      double tot = 0.0, mx = a.rel[off + sIdx[t]];
      int cnt = 0;
      for (int q = t; q < n; ++q) {
        if (q > t && (sk[q] == kNanKey || sk[q] != sk[t])) break;
        const int iq = sIdx[q];
        tot += a.weight[off + iq];
        ++cnt;
        const double rq = a.rel[off + iq];
        if (q != t && rq > mx) mx = rq;
        if (sk[t] == kNanKey) break;
      }
      if (tot / (double)cnt == wd && mx == wm) sFlag = 1;
    }
    // confidence variance (tiebreak.py:108-110): the mean and the sum of squares run in
    // agent order on one lane; the squares -- libm pow(d, 2.0), glibc_pow.hpp -- are
    // computed by every thread for its agents into the (now dead) sort keys
    if (tid == 0) {
      double csum = 0.0;
      for (int i = 0; i < n; ++i) csum += a.conf[off + i];
      sVar = csum / (double)n;
    }
    __syncthreads();
    {
      const double mean = sVar;
      double* const sq = reinterpret_cast<double*>(sk);
      for (int i = tid; i < n; i += kTbThreads) sq[i] = bce_pow::pow2(a.conf[off + i] - mean);
    }
    __syncthreads();
    if (tid == 0) {
      const double* const sq = reinterpret_cast<const double*>(sk);
      double vs = 0.0;
      for (int i = 0; i < n; ++i) vs += sq[i];
      sVar = vs / (double)n;
    }
    __syncthreads();
    if (tid == 0) {
      a.winner[m] = wk;
      a.label[m] = (ng == 1) ? BCE_TB_UNANIMOUS
                             : (sFlag ? BCE_TB_PREDICTION_VALUE_SMALLEST : BCE_TB_WEIGHT_DENSITY);
      a.n_groups[m] = ng;
      a.variance[m] = sVar;
    }
    __syncthreads();
  }
}

}  // namespace bce

using namespace bce;

static double pow10_exact(int nd) {
  double s = 1.0;
  for (int i = 0; i < nd; ++i) s *= 10.0;  // exact for nd <= 22
  return s;
}
// 2^E with E = floor(52 - nd*log2(10)) + 1: the smallest power of two whose ulp exceeds 10^-nd
static double round_thresh(int nd) {
  const double y = nd * 3.321928094887362;
  const int E = (int)floor(52.0 - y) + 1;
  return ldexp(1.0, E);
}
// CPython float.__round__(x, nd): nd > 323 returns x, nd < -308 returns 0.0 * x
// (NDIGITS_MAX / NDIGITS_MIN of floatobject.c); in between the correctly rounded decimal.
// Restated with doubles for -15 <= nd <= 22 (10^|nd| exact, remainders exact) and with
// exact big integers (py_round_big.hpp, EXOTIC kernels) for the rest.
static int tb_round_mode(int nd, double* scale, double* thresh) {
  *scale = 1.0;
  *thresh = 0.0;
  if (nd > 323) return 2;
  if (nd < -308) return 3;
  if (nd >= 0 && nd <= 22) {
    *scale = pow10_exact(nd);
    *thresh = round_thresh(nd);
    return 0;
  }
  if (nd < 0 && nd >= -15) {
    *scale = pow10_exact(-nd);
    return 1;
  }
  return nd > 0 ? 4 : 5;
}

template <bool EXOTIC>
static int launch_tb_short(const TbArgs& a, const int32_t* market_list, int64_t nl, int32_t max_len, void* stream) {
  if (max_len <= kTbLpmMax) {  // lane per market: 64 markets per wave, kTbLpmWaves per workgroup
    const int64_t tiles = (nl + 63) / 64;
    int64_t blocks = (tiles + kTbLpmWaves - 1) / kTbLpmWaves;
    // contiguous markets stage each wave's agent range in LDS; a market list gathers rows
    // contiguous markets, register-batch staging: the FULL tiles (64 markets of 32 agents)
    // run a kernel specialised for them, then a second launch takes every other tile (each
    // launch only reads the offsets of the tiles it leaves to the other)
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    bool split = !EXOTIC && a.rmode == 0 && al16(a.pred) && al16(a.conf) &&
                 al16(a.weight) && al16(a.rel);
    // market lists: rows gathered into LDS as 16-B aligned pairs (every array 16-B aligned;
    // else each lane reads and writes its own row in global memory), NP = the list's bound
    // rounded up to 8 / 16 / 32
    const int np = max_len <= 8 ? 8 : max_len <= 16 ? 16 : 32;
    const bool gather = al16(a.pred) && al16(a.conf) && al16(a.weight) && al16(a.rel) &&
                        (!a.g_key || al16(a.g_key)) && (!a.g_density || al16(a.g_density)) &&
                        (!a.g_avgconf || al16(a.g_avgconf)) && (!a.g_maxrel || al16(a.g_maxrel));
    const void* fn = (market_list && !gather) ? reinterpret_cast<const void*>(&tiebreak_lpm_kernel<false, EXOTIC>)
                     : market_list ? (np == 8    ? reinterpret_cast<const void*>(&tiebreak_lpm_kernel<true, EXOTIC, 0, 8, true>)
                                    : np == 16 ? reinterpret_cast<const void*>(&tiebreak_lpm_kernel<true, EXOTIC, 0, 16, true>)
                                               : reinterpret_cast<const void*>(&tiebreak_lpm_kernel<true, EXOTIC, 0, 32, true>))
                     : split     ? reinterpret_cast<const void*>(&tiebreak_lpm_kernel<true, false, 1>)
                                 : reinterpret_cast<const void*>(&tiebreak_lpm_kernel<true, EXOTIC>);
    const int per_cu = blocks_per_cu(fn, 64 * kTbLpmWaves, 0, 1, "tiebreak_lpm_kernel");
    const int64_t cap = (int64_t)cu_count() * per_cu;
    if (blocks > cap) blocks = cap;
    split = split && blocks * kTbLpmWaves <= kSplitWords;  // one split word per wave of the grid
    hipStream_t st = as_stream(stream);
    const dim3 grid((int)blocks), block(64 * kTbLpmWaves);
    if (market_list && !gather) {
      hipLaunchKernelGGL((tiebreak_lpm_kernel<false, EXOTIC>), grid, block, 0, st, a, market_list, nl, fault_word());
    } else if (market_list) {
      if (np == 8)
        hipLaunchKernelGGL((tiebreak_lpm_kernel<true, EXOTIC, 0, 8, true>), grid, block, 0, st, a, market_list, nl,
                           fault_word());
      else if (np == 16)
        hipLaunchKernelGGL((tiebreak_lpm_kernel<true, EXOTIC, 0, 16, true>), grid, block, 0, st, a, market_list, nl,
                           fault_word());
      else
        hipLaunchKernelGGL((tiebreak_lpm_kernel<true, EXOTIC, 0, 32, true>), grid, block, 0, st, a, market_list, nl,
                           fault_word());
    } else if (split) {
      static std::atomic<int> tickets{0};
      TbArgs b = a;
      // positive; after a wrap split_slot clears the slot's stale (larger) tickets
      b.ticket = (tickets.fetch_add(1) & 0x3fffffff) + 1;
      b.split = split_slot(b.ticket, st);
      if (!b.split) {
        set_error("tiebreak: no device split words");
        return BCE_EHIP;
      }
      hipLaunchKernelGGL((tiebreak_lpm_kernel<true, false, 1>), grid, block, 0, st, b, market_list, nl, fault_word());
      if (int rc = check_launch("tiebreak_lpm_kernel<full>")) return rc;
      hipLaunchKernelGGL((tiebreak_lpm_kernel<true, false, 2>), grid, block, 0, st, b, market_list, nl, fault_word());
    } else {
      hipLaunchKernelGGL((tiebreak_lpm_kernel<true, EXOTIC>), grid, block, 0, st, a, market_list, nl, fault_word());
    }
    return check_launch("tiebreak_lpm_kernel");
  }
  int64_t blocks = (nl + 3) / 4;
  const int64_t cap = (int64_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(tiebreak_wave_kernel<EXOTIC>, dim3((int)blocks), dim3(256), 0, as_stream(stream), a,
                     market_list, nl);
  return check_launch("tiebreak_wave_kernel");
}

extern "C" int bce_tiebreak_csr(const int64_t* offsets, int64_t n_markets, const int32_t* market_list,
                                int64_t n_list, const double* pred, const double* conf,
                                const double* weight, const double* rel, int32_t max_len,
                                int32_t ndigits, double* winner, int32_t* label, int32_t* n_groups,
                                double* variance, double* g_key, int32_t* g_count, double* g_density,
                                double* g_avgconf, double* g_maxrel, int32_t* g_of, void* stream) {
  BCE_REQUIRE(n_markets >= 0, "tiebreak: n_markets < 0");
  const int64_t nl = market_list ? n_list : n_markets;
  if (nl == 0) return BCE_OK;
  BCE_REQUIRE(offsets && pred && conf && weight && rel && winner && label && n_groups && variance,
              "tiebreak: NULL argument");
  BCE_REQUIRE(max_len > 0 && max_len <= 64,
              "tiebreak: max_len must be in 1..64 (longer markets: bce_tiebreak_csr_long)");
  double rs = 1.0, rt = 0.0;
  const int rmode = tb_round_mode(ndigits, &rs, &rt);
  TbArgs a{offsets, n_markets, pred, conf, weight, rel, winner, label, n_groups, variance,
           g_key, g_count, g_density, g_avgconf, g_maxrel, g_of, rs, rt, 1.0 / rs, rmode, ndigits, fault_word(), nullptr, 0};
  return rmode >= 4 ? launch_tb_short<true>(a, market_list, nl, max_len, stream)
                    : launch_tb_short<false>(a, market_list, nl, max_len, stream);
}

template <bool EXOTIC>
static int launch_tb_long(const TbArgs& a, const int32_t* list, int64_t n_list, int64_t max_len, void* stream) {
  hipStream_t st = as_stream(stream);
  if (max_len <= kTbMax) {
    int64_t blocks = n_list;
    const int64_t cap = (int64_t)cu_count() * 2;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL((tiebreak_block_kernel<true, EXOTIC>), dim3((int)blocks), dim3(kTbThreads), 0, st, a, list,
                       n_list, nullptr, (int64_t)0);
    return check_launch("tiebreak_block_kernel<lds>");
  }
  // any longer market: sort in a global scratch slice per workgroup (16 B per entry)
  int64_t P = 1;
  while (P < max_len) P <<= 1;
  // each workgroup walks the list with a stride of the grid, so its slice must hold the
  // longest market; the grid shrinks instead of the scratch growing past 1 GiB (one
  // 10M-agent market beside other long ones would otherwise ask for CUs x 256 MB)
  int64_t blocks = n_list;
  int64_t cap = (int64_t)cu_count();
  const int64_t by_budget = ((int64_t)1 << 30) / (16 * P);
  if (cap > by_budget) cap = by_budget > 0 ? by_budget : 1;
  if (blocks > cap) blocks = cap;
  void* scratch = nullptr;
  BCE_HIP(hipMallocAsync(&scratch, (size_t)(blocks * 16 * P), st));
  hipLaunchKernelGGL((tiebreak_block_kernel<false, EXOTIC>), dim3((int)blocks), dim3(kTbThreads), 0, st, a, list, n_list,
                     scratch, P);
  const int rc = check_launch("tiebreak_block_kernel<global>");
  BCE_HIP(hipFreeAsync(scratch, st));
  return rc;
}

extern "C" int bce_tiebreak_csr_long(const int64_t* offsets, int64_t n_markets, const int32_t* list,
                                     int64_t n_list, int32_t ndigits, const double* pred,
                                     const double* conf, const double* weight, const double* rel,
                                     int64_t max_len, double* winner, int32_t* label,
                                     int32_t* n_groups, double* variance, double* g_key,
                                     int32_t* g_count, double* g_density, double* g_avgconf,
                                     double* g_maxrel, int32_t* g_of, void* stream) {
  BCE_REQUIRE(n_list >= 0 && (n_list == 0 || list), "tiebreak_long: bad list");
  if (n_list == 0) return BCE_OK;
  BCE_REQUIRE(offsets && pred && conf && weight && rel && winner && label && n_groups && variance,
              "tiebreak_long: NULL argument");
  BCE_REQUIRE(max_len > 0 && max_len < (1ll << 31), "tiebreak_long: max_len out of range");
  double rs = 1.0, rt = 0.0;
  const int rmode = tb_round_mode(ndigits, &rs, &rt);
  TbArgs a{offsets, n_markets, pred, conf, weight, rel, winner, label, n_groups, variance,
           g_key, g_count, g_density, g_avgconf, g_maxrel, g_of, rs, rt, 1.0 / rs, rmode, ndigits, fault_word(), nullptr, 0};
  return rmode >= 4 ? launch_tb_long<true>(a, list, n_list, max_len, stream)
                    : launch_tb_long<false>(a, list, n_list, max_len, stream);
}

// Host-side run of the exotic-precision rounding (the same header code the EXOTIC kernels
// run), for the CPU tests against Python round(): nd in 1..323 via round_pos, -308..-1 via
// round_neg (both also valid where the double paths are used); *overflow = 1 when CPython
// would raise OverflowError.
extern "C" double bce_debug_py_round(double x, int32_t ndigits, int32_t* overflow) {
  bool ovf = false;
  double r = x;
  if (ndigits > 0 && ndigits <= 323) r = bce_round::round_pos(x, ndigits);
  else if (ndigits < 0 && ndigits >= -308) r = bce_round::round_neg(x, -ndigits, &ovf);
  if (overflow) *overflow = ovf ? 1 : 0;
  return r;
}
