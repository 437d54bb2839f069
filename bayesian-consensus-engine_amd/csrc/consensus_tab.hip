// consensus_tab.hip -- core.compute_consensus (core.py:63-179) for contiguous markets with
// n <= 32, the source table held in LDS.
//
// Why this shape (tools/gather_probe.hip, profiles/r02_gather_probe.txt): streaming the
// C2 bytes alone takes 0.185 ms; adding one random 16-B {rel, conf} gather per signal
// from the 160 KB table in global memory takes it to 0.288 ms (the round-1 kernel's time:
// those gathers, not HBM, bound it), while the same gathers served from LDS cost almost
// nothing (0.189 ms).  So one workgroup per CU stages the whole table (16 B per source +
// the present bitmask, S <= kTabMaxSources = the 160 KB LDS) once, and everything else
// stays in VGPRs -- no LDS staging ring, no producer/consumer waves:
//
//  load       a wave owns a tile of 64 consecutive markets.  A REGULAR tile (every market
//             has 32 signals, 16-B aligned) is read with coalesced 16-B loads: eight
//             lanes (m, m+8, ..., m+56) cover one contiguous 128-B piece of a market's
//             row.  Three butterflies (v_permlane32_swap, v_permlane16_swap, row_ror:8 DPP)
//             swap those lane bits with load-index bits, leaving lane = market, register
//             index = position.  Other tiles (ragged lengths, the last tile, misaligned
//             shards) load per lane.  The next tile's offsets are read at the top of each tile.
//  sort       keys (sid << 5 | position) with the probability as payload, Batcher
//             odd-even merge network in VGPRs (branch-free, VGPR swap masks):
//             duplicates of a source stay in input order.
//  averages   duplicate runs (rare) are summed in input order and divided once per run
//             (core.py:115-116), in rounds over the wave's lanes.
//  walk       sorted positions left to right: {rel, conf} from LDS (ds_read_b128, eight
//             ahead), the reference's three left-to-right chains over unique sources
//             (core.py:120,135-143) -- each lane is one market, so the exact order is free.
//  compact    per-unique (usid, weight) pairs are emitted at their run's last sorted
//             position; the duplicates' holes are removed highest first (rounds over the
//             wave, usually one).
//  store      per-market scalars from the market's lane; per-unique outputs go back
//             through the same butterflies and leave as coalesced 16-B chunk stores
//             (chunks holding no unique are skipped; slots past n_unique inside a written
//             chunk are scratch, include/bce.h).  normalizedWeight = weight / total is
//             divided in the store layout, the market's total fetched with ds_bpermute.
// Validation (core.py:59-60: first p < 0 or p > 1, NaN passes) reads the probabilities in
// input order before the sort.  Exact mode only: every sum is the reference's own order.
//
// Measured (tools/tab_variants.py, measurements/tab_*_r0[23].txt): with nontemporal signal
// loads and per-unique stores, 8 waves per CU (two per SIMD, 256 VGPRs) beat 4; wave-major
// tile order (consecutive tiles on consecutive workgroups / XCDs) -3.3%; a wave priority
// ramp through the tile (1 walk, 2 per-market outputs, 3 per-unique stores) -4%; the
// permlane transposes -2..3% against DPP-only ones.  The per-unique stores are the largest
// phase; loading the next tile's signals ahead, unconditional chunk stores, a
// reciprocal-based normalizedWeight and nontemporal per-market stores did not help.  The
// alternatives live in tools/tab_variants.py (source patches), not here.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "consensus_common.hpp"

#pragma clang fp contract(off)

namespace bce {
namespace {

constexpr int kTabWaves = 8;  // waves per workgroup (two per SIMD); one workgroup per CU (LDS-bound)
// The next tile's metadata read at the top of a tile (true) or after its walk (false: no spill
// stores left in the tile loop, but 1.7% slower -- 0.2143-0.2146 vs 0.2109-0.2129 ms,
// profiles/archive/r05d/)
constexpr bool kTabMetaEarly = true;
constexpr int kPL = 8;         // lanes per 128-B piece of a market row (16 B each)
constexpr int kLB = 3;         // log2 kPL
constexpr int kMG = 64 / kPL;  // markets per load instruction
constexpr int kTabRing = 8;    // LDS table reads issued ahead of the walk (4/6/8 measured equal)

// Nontemporal signal loads and per-unique stores (the per-market stores stay default:
// nt there measured slower, measurements/tab_nt_variants_r02.txt).
typedef unsigned tab_u4v __attribute__((ext_vector_type(4)));
typedef double tab_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 tab_ld16(const uint32_t* p) {
  const tab_u4v v = __builtin_nontemporal_load(reinterpret_cast<const tab_u4v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void tab_st16(int32_t* p, uint4 v) {
  const tab_u4v x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<tab_u4v*>(p));
}
__device__ __forceinline__ void tab_st16(double* p, double x0, double x1) {
  const tab_d2v x = {x0, x1};
  __builtin_nontemporal_store(x, reinterpret_cast<tab_d2v*>(p));
}

// ---- lane-bit <-> register-bit butterflies -------------------------------------------
// A 128-B piece of a market row is read by eight lanes m, m+8, ..., m+56: the piece's
// eight 16-B chunks sit on lane bits 5..3 (the same addresses per instruction as eight
// consecutive lanes -- no memory cost, tools/tile_probe.hip).  For a register pair (a:
// index bit j, b: the partner with that bit set) each butterfly swaps one of those lane
// bits with the index bit: a' = bit ? b[lane ^ 2^L] : a, b' = bit ? b : a[lane ^ 2^L].
// Lane bit 5 is one v_permlane32_swap per pair, bit 4 one v_permlane16_swap, bit 3 a
// row_ror:8 DPP pair with a wave-constant select.
__device__ __forceinline__ void bfly_pl32(uint32_t& a, uint32_t& b) {  // lane bit 5
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void bfly_pl16(uint32_t& a, uint32_t& b) {  // lane bit 4
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void bfly_r8(uint32_t& a, uint32_t& b, int lane) {  // lane bit 3: l ^ 8 = row_ror:8
  const bool hi = (lane & 8) != 0;
  const uint32_t bx = (uint32_t)__builtin_amdgcn_mov_dpp((int)b, 0x128, 0xF, 0xF, true);
  const uint32_t ax = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0x128, 0xF, 0xF, true);
  const uint32_t na = hi ? bx : a;
  b = hi ? b : ax;
  a = na;
}
// Swap lane bits 5..3 with dword-index bits 4..2 of r[N] (an involution).  The three
// butterflies commute; permlane32 / permlane16 / row_ror:8 measured 4% faster than the
// reverse order on the same box (0.2090 vs 0.2184 ms median, measurements/tab_xord_r03.txt)
// although the reverse order spills fewer VGPRs.
template <int N>
__device__ __forceinline__ void xpose(uint32_t (&r)[N], int lane) {
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 16)) bfly_pl32(r[i], r[i | 16]);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 8)) bfly_pl16(r[i], r[i | 8]);
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (!(i & 4)) bfly_r8(r[i], r[i | 4], lane);
}

// Regular-tile address maps (tile = 64 markets x 32 signals from B; PL = kPL lanes per
// piece, MG = 64 / PL, load index k, q = lane >> log2 PL, c = lane & (PL-1)): every PL
// consecutive lanes read one contiguous 16·PL-byte piece of one market's row, so each
// wave-instruction is MG fully coalesced pieces (PL = 4: 64-B pieces, 8: 128-B)
//   sid   k < 8:  market MG(k&(PL-1)) + q, positions 4PL(k>>log2 PL) + 4c + d   dword 4k + d
//   prob  k < 16: market MG(k&(PL-1)) + q, positions 2PL(k>>log2 PL) + 2c + h  double 2k + h
// Swapping the log2 PL lane bits of c with the low load-index bits leaves one market per
// lane -- lane L holds market tmkt(L) = MG (L & (PL-1)) + (L >> log2 PL) -- and the
// register index = the position, for both arrays.
// (With the chunks on lane bits 5..3, lane L reads market group q = L & 7, chunk c = L >> 3,
// and after the transpose holds market L.)
__device__ __forceinline__ int tmkt(int lane) { return lane; }
// this lane's market-within-group q and chunk c in the regular-tile address maps
__device__ __forceinline__ int lq(int lane) { return lane & 7; }
__device__ __forceinline__ int lc(int lane) { return lane >> 3; }
// Odd-even merge network over 31-bit keys with a 64-bit payload, branch- and SGPR-free:
// the swap mask is the sign of y - x (keys < 2^31), the payload moves with v_bfi_b32.
// (Compare-and-select would give every comparator of a stage its own SGPR-pair condition;
// the 191-comparator network then spills SGPRs.)
__device__ __forceinline__ void oem_sort_kv31(unsigned (&key)[32], double (&val)[32]) {
  constexpr auto P = OemNet<32>::make();
#pragma unroll
  for (int c = 0; c < OemNet<32>::C; ++c) {
    const unsigned x = key[P.a[c]], y = key[P.b[c]];
    unsigned m = (unsigned)((int)(y - x) >> 31);  // all ones <=> y < x
    asm("" : "+v"(m));
    key[P.a[c]] = min(x, y);
    key[P.b[c]] = max(x, y);
    const uint64_t vx = (uint64_t)__double_as_longlong(val[P.a[c]]), vy = (uint64_t)__double_as_longlong(val[P.b[c]]);
    const uint64_t mm = ((uint64_t)m << 32) | m;
    val[P.a[c]] = __longlong_as_double((long long)((mm & vy) | (~mm & vx)));
    val[P.b[c]] = __longlong_as_double((long long)((mm & vx) | (~mm & vy)));
  }
}

__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) {
  return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ uint32_t lo32(double x) { return (uint32_t)__double_as_longlong(x); }
__device__ __forceinline__ uint32_t hi32(double x) { return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32); }

// HYB: the table is larger than the LDS; rows [0, a.tab_rows) are staged (with the whole
// present bitmask) and the walk gathers the others from the global relconf table.
template <bool HYB>
__global__ __launch_bounds__(64 * kTabWaves) void consensus_tab32_kernel(ConsArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char tab_smem[];
  const int S = a.n_sources > 0 ? a.n_sources : 1;
  const int nwords = (S + 31) >> 5;
  const int rows = HYB ? a.tab_rows : S;  // rows staged in LDS
  double2* const sT = reinterpret_cast<double2*>(tab_smem);
  uint32_t* const sB = reinterpret_cast<uint32_t*>(tab_smem + 16 * (size_t)rows);
  // ---- stage the table once per workgroup ----------------------------------------------
  if (a.n_sources > 0) {
    int i = threadIdx.x;
    for (; i + 3 * 64 * kTabWaves < rows; i += 4 * 64 * kTabWaves) {
      double2 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = a.relconf[i + q * 64 * kTabWaves];
#pragma unroll
      for (int q = 0; q < 4; ++q) sT[i + q * 64 * kTabWaves] = v[q];
    }
    for (; i < rows; i += 64 * kTabWaves) sT[i] = a.relconf[i];
    for (int j = threadIdx.x; j < nwords; j += 64 * kTabWaves) sB[j] = a.pbits[j];
  } else if (threadIdx.x == 0) {
    sT[0] = make_double2(0.5, 0.25);  // DEFAULT_RELIABILITY / _CONFIDENCE (config.py:17-18)
    sB[0] = 0u;
  }
  __syncthreads();

  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform loop
  const unsigned smax = (unsigned)(S - 1);
  const int64_t M = a.n_list;
  const int64_t n_tiles = (M + 63) >> 6;
  const int64_t stride = (int64_t)gridDim.x * kTabWaves;
  const bool do_u = a.usid != nullptr, do_w = a.weight != nullptr, do_nw = a.nweight != nullptr;
  const bool do_any = do_u || do_w || do_nw;

  // Tile metadata: this lane's market bounds, the tile base B and whether the tile is
  // regular (64 markets x 32 signals from a 16-B aligned B).
  struct Meta {
    int64_t off;
    int n;
    int64_t B;
    bool reg;
  };
  auto meta = [&](int64_t tile, int lane) -> Meta {
    Meta m{0, 0, 0, false};
    if (tile >= n_tiles) return m;
    const int j = tmkt(lane);
    const int64_t mk = tile * 64 + j;
    int64_t end = 0;
    if (mk < M) {
      m.off = a.offsets[mk];
      end = a.offsets[mk + 1];
    }
    m.n = (int)(end - m.off);
    if (ballot(mk < M && (m.n < 0 || m.n > 32))) {  // the launch promised max_len <= 32
      raise_fault(a.fault, kFaultTooLong);
      if (m.n < 0 || m.n > 32) m.n = 0;
    }
    m.B = ((int64_t)__builtin_amdgcn_readfirstlane((int)(m.off >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)m.off);  // lane 0 holds market 0
    m.reg = ballot(!(mk < M && m.n == 32 && m.off == m.B + 32 * (int64_t)j)) == 0 &&
            ((((uintptr_t)(a.sid + m.B)) | ((uintptr_t)(a.prob + m.B))) & 15) == 0;
    return m;
  };
  // Regular-tile loads (the address maps above); raw, not yet transposed.
  auto load_regular = [&](int64_t B, int lane, uint32_t (&rs)[32], uint32_t (&rp)[64]) {
    const int q = lq(lane), c = lc(lane);
    const uint32_t* sb = reinterpret_cast<const uint32_t*>(a.sid + B);
    const double* pb = a.prob + B;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = tab_ld16(sb + 32 * (kMG * (k & (kPL - 1)) + q) + 4 * kPL * (k >> kLB) + 4 * c);
      rs[4 * k] = v.x; rs[4 * k + 1] = v.y; rs[4 * k + 2] = v.z; rs[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint4 v = tab_ld16(reinterpret_cast<const uint32_t*>(pb + 32 * (kMG * (k & (kPL - 1)) + q) +
                                                                 2 * kPL * (k >> kLB) + 2 * c));
      rp[4 * k] = v.x; rp[4 * k + 1] = v.y; rp[4 * k + 2] = v.z; rp[4 * k + 3] = v.w;
    }
  };

  // The next tile's metadata is read at the top of each tile (loading the next tile's
  // signals ahead, or the first tile's under the table staging, measured slower: spills).
  // Wave-major tile order: tile = w * grid + block, so the tiles in flight at any moment
  // are spread over every workgroup (and XCD) instead of 8 consecutive tiles per CU
  // (tools/tile_probe.hip: 0.204 -> 0.195 ms for the same bytes and shapes)
  int64_t tile = (int64_t)w * gridDim.x + blockIdx.x;
  Meta cur = meta(tile, lane_id());
  uint32_t s[32], pw[64];
  for (; tile < n_tiles; tile += stride) {
    // lane-derived offsets are recomputed per tile: hoisted out of the loop, the 24 load
    // and 40 store address offsets would stay live across the whole tile
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    const int64_t m0 = tile * 64;
    const int64_t off = cur.off, B = cur.B;
    const int n = cur.n;
    const bool reg = cur.reg;
    // the next tile's metadata: read here (kTabMetaEarly) or after the walk, so its registers
    // are not live through the sort and the walk
    Meta nxt{};
    if constexpr (kTabMetaEarly) nxt = meta(tile + stride, lane);

    // ---- lane = market, s[t] = sid, pw = probabilities ------------------------------------
    if (reg) {
      load_regular(B, lane, s, pw);
      xpose<32>(s, lane);
      xpose<64>(pw, lane);
    } else if (a.n_signals > 0) {
      // per-lane rows, straight-line: positions past n re-read the market's last signal
      // (or signal 0 of the batch for an empty market) and are masked later
      const int64_t base = (n > 0) ? off : 0;
      const int last = (n > 0) ? n - 1 : 0;
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        const int64_t i = base + min(t, last);
        s[t] = (uint32_t)a.sid[i];
        const double v = a.prob[i];
        pw[2 * t] = lo32(v);
        pw[2 * t + 1] = hi32(v);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 64; ++t) pw[t] = 0u;
#pragma unroll
      for (int t = 0; t < 32; ++t) s[t] = 0u;
    }
    __builtin_amdgcn_sched_barrier(0);
    double p[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) p[t] = dbl(pw[2 * t], pw[2 * t + 1]);

    // ---- validation (core.py:59-60) in input order ----------------------------------------
    // per-position predicates are folded into lane bitmasks right away (t < n as a
    // compare would be CSE'd into 32 SGPR-pair conditions held across the sort)
    const unsigned vb = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
    unsigned badp = 0, bads = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      badp |= ((p[t] < 0.0 || p[t] > 1.0) ? 1u : 0u) << t;  // NaN passes
      bads |= ((s[t] > smax) ? 1u : 0u) << t;
    }
    badp &= vb;
    const int err = badp ? (int)__builtin_ctz(badp) : -1;
    if (ballot((bads & vb) != 0u)) raise_fault(a.fault, kFaultSid);

    // ---- sort (sid, position) with the probability as payload -----------------------------
    unsigned key[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe(vb, t, 1);
      key[t] = (m & ((min(s[t], smax) << 5) | (unsigned)t)) | (~m & 0x7FFFFFFFu);
    }
    oem_sort_kv31(key, p);
    __builtin_amdgcn_sched_barrier(0);
    unsigned nq = 0;
#pragma unroll
    for (int t = 30; t >= 0; --t) nq = (nq << 1) | ((((key[t] ^ key[t + 1]) >> 5) != 0u) ? 1u : 0u);
    const unsigned lb = (nq | 0x80000000u) & vb;  // last position of a run
    const unsigned fb = ((nq << 1) | 1u) & vb;    // first position of a run

    // ---- duplicate runs: averaged in input order (core.py:115-116) ----------------------
    // dupend = last positions of runs of two or more signals.  Each round handles every
    // lane's highest remaining run: its signals are summed left to right (the other
    // positions add +0.0, which is exact: the sum starts at +0.0 like builtin sum() from
    // int 0 and never becomes -0.0), divided once, and the average replaces the
    // probability at the run's last position.  Rounds = the wave's most duplicated market
    // (nearly always one).
    unsigned dupend = lb & ~fb;
    while (ballot(dupend != 0u)) {
      const int te = dupend ? 31 - __builtin_clz(dupend) : -1;
      const unsigned upto = (te >= 0) ? (0xFFFFFFFFu >> (31 - te)) : 0u;  // bits 0..te
      dupend &= ~(upto ^ (upto >> 1));
      const unsigned fm = fb & upto;
      const int ts = fm ? 31 - __builtin_clz(fm) : 0;
      const unsigned run = upto & ~((1u << ts) - 1u);  // bits ts..te (0 when te < 0)
      double psum = 0.0;
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        uint32_t m = (uint32_t)__builtin_amdgcn_sbfe(run, t, 1);
        asm("" : "+v"(m));
        const uint64_t m64 = ((uint64_t)m << 32) | m;
        psum += __longlong_as_double((long long)(m64 & (uint64_t)__double_as_longlong(p[t])));
      }
      const double avg = psum / (double)(te - ts + 1);
      const unsigned at = upto ^ (upto >> 1);  // bit te
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        uint32_t m = (uint32_t)__builtin_amdgcn_sbfe(at, t, 1);
        asm("" : "+v"(m));
        const uint64_t m64 = ((uint64_t)m << 32) | m;
        p[t] = __longlong_as_double((long long)((m64 & (uint64_t)__double_as_longlong(avg)) |
                                                (~m64 & (uint64_t)__double_as_longlong(p[t]))));
      }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- walk (core.py:107-144 in sorted-source order) ----------------------------------
    // wave priority ramps up through the tile (1 walk, 2 per-market outputs + compaction, 3
    // per-unique stores, back to 0 for the next tile's loads): of the two waves sharing a
    // SIMD, the one further into its tile issues first, so its stores leave while the other
    // wave's loads are in flight (-4.2% against none, tools/tab_variants.py)
    __builtin_amdgcn_s_setprio(1);
    double2 ring[kTabRing];
    uint32_t rbits[kTabRing];
    // one table row: LDS, or (hybrid, rows past the staged ones) the global table
    auto row = [&](unsigned ix) -> double2 {
      if constexpr (HYB) {
        if (ix >= (unsigned)rows) return a.relconf[ix];
      }
      return sT[ix];
    };
#pragma unroll
    for (int t = 0; t < kTabRing; ++t) {
      const unsigned ix = min(key[t] >> 5, smax);
      ring[t] = row(ix);
      rbits[t] = sB[ix >> 5];
    }
    double total = 0.0, ws = 0.0, cs = 0.0;
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      const unsigned sid = key[t] >> 5;
      const double2 rc = ring[t % kTabRing];
      const uint32_t bw = rbits[t % kTabRing];
      if (t + kTabRing < 32) {
        const unsigned ix = min(key[t + kTabRing < 32 ? t + kTabRing : t] >> 5, smax);
        ring[t % kTabRing] = row(ix);
        rbits[t % kTabRing] = sB[ix >> 5];
      }
      // p[t] at a run's last position is the source's average (a single signal: p itself;
      // -0.0 * w adds nothing); accumulate only there -- + 0.0 leaves every chain bit-exact
      const double wt = rc.x, cf = rc.y, avg = p[t];
      const bool lst = ((lb >> t) & 1u) != 0u;
      total += lst ? wt : 0.0;         // core.py:120
      ws += lst ? avg * wt : 0.0;      // core.py:135-137
      cs += lst ? cf * wt : 0.0;       // core.py:141-143
      // emitted at the run's last position: usid (cold bit, core.py:167-170) and weight
      key[t] = sid | ((((bw >> (sid & 31)) & 1u) != 0u) ? 0u : 0x80000000u);
      p[t] = wt;
      asm volatile("" : "+v"(total), "+v"(ws), "+v"(cs));
      __builtin_amdgcn_sched_barrier(0);
    }
    const int u = __builtin_popcount(lb);

    // ---- per-market results (lane = market, coalesced) -----------------------------------
    __builtin_amdgcn_s_setprio(2);
    if constexpr (!kTabMetaEarly) nxt = meta(tile + stride, lane_id());
    {
      // the market index re-derived here: held from the top of the tile, it and the five
      // output addresses built from it stay live through the sort and the walk (spills)
      int ln = lane_id();
      asm volatile("" : "+v"(ln));
      const int64_t mk2 = m0 + tmkt(ln);
      if (mk2 < M) {
        const bool null_ = (total == 0.0);  // core.py:131-133
        a.consensus[mk2] = null_ ? 0.0 : ws / total;
        a.confidence[mk2] = null_ ? 0.0 : cs / total;
        a.total_weight[mk2] = total;
        a.n_unique[mk2] = u;
        if (a.err_idx) a.err_idx[mk2] = err;
      }
    }
    if (!do_any) {
      __builtin_amdgcn_s_setprio(0);
      cur = nxt;
      continue;
    }

    // ---- compaction: unique j = the j-th emitted position ---------------------------------
    const unsigned full = (u >= 32) ? 0xFFFFFFFFu : ((1u << u) - 1u);
    if (ballot(lb != full)) {
      // holes = valid positions that are not the last of their run (duplicates).  Remove
      // the highest hole of every lane per round: slots above it move down by one, the
      // lower holes stay where they are.  Rounds = the wave's largest duplicate count
      // (nearly always 1).  Selects use VGPR masks (v_bfi_b32): compare-and-select would
      // hold 32 SGPR-pair conditions.
      unsigned holes = vb & ~lb;
      while (ballot(holes != 0u)) {
        const int h = holes ? 31 - __builtin_clz(holes) : 32;
        holes &= ~(1u << (h & 31));
#pragma unroll
        for (int i = 0; i < 31; ++i) {
          uint32_t m = (uint32_t)((h - 1 - i) >> 31);  // all ones <=> i >= h
          asm("" : "+v"(m));
          key[i] = (m & key[i + 1]) | (~m & key[i]);
          const uint64_t m64 = ((uint64_t)m << 32) | m;
          const uint64_t x = (uint64_t)__double_as_longlong(p[i + 1]), y = (uint64_t)__double_as_longlong(p[i]);
          p[i] = __longlong_as_double((long long)((m64 & x) | (~m64 & y)));
        }
      }
    }

    // ---- per-unique outputs --------------------------------------------------------------
    __builtin_amdgcn_s_setprio(3);
    __builtin_amdgcn_sched_barrier(0);
    if (reg) {
      // re-derive the tile base and the lane offsets here: without the opaque copies the
      // compiler hoists all 40 store addresses to the top of the tile (SGPR/VGPR spills)
      uint32_t blo = (uint32_t)B, bhi = (uint32_t)((uint64_t)B >> 32);
      asm volatile("" : "+s"(blo), "+s"(bhi));
      const int64_t B = (int64_t)(((uint64_t)bhi << 32) | blo);
      int lane = lane_id();
      asm volatile("" : "+v"(lane));
      const int q = lq(lane), c = lc(lane);
      int uk[kPL];
      double tk[kPL];
#pragma unroll
      for (int k = 0; k < kPL; ++k) {  // market MG·k + q of load index k sits in lane PL·q + k
        const int src = ((k << 3) | (lane & 7)) << 2;
        uk[k] = __builtin_amdgcn_ds_bpermute(src, u);
        tk[k] = dbl((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)lo32(total)),
                    (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)hi32(total)));
      }
      // whole 16-byte chunks holding at least one unique (the rest of the chunk is scratch)
      if (do_u) {
        uint32_t o[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) o[t] = key[t];
        xpose<32>(o, lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int slot = 4 * kPL * (k >> kLB) + 4 * c;
          if (uk[k & (kPL - 1)] > slot)
            tab_st16(a.usid + B + 32 * (kMG * (k & (kPL - 1)) + q) + slot,
                     make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]));
        }
      }
      if (do_w || do_nw) {
        uint32_t o[64];
#pragma unroll
        for (int t = 0; t < 32; ++t) {
          o[2 * t] = lo32(p[t]);
          o[2 * t + 1] = hi32(p[t]);
        }
        xpose<64>(o, lane);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int slot = 2 * kPL * (k >> kLB) + 2 * c;
          const int64_t pos = B + 32 * (kMG * (k & (kPL - 1)) + q) + slot;
          const double w0 = dbl(o[4 * k], o[4 * k + 1]), w1 = dbl(o[4 * k + 2], o[4 * k + 3]);
          const double tot = tk[k & (kPL - 1)];
          if (uk[k & (kPL - 1)] > slot) {
            if (do_w) tab_st16(a.weight + pos, w0, w1);
            if (do_nw) tab_st16(a.nweight + pos, tot > 0.0 ? w0 / tot : 0.0, tot > 0.0 ? w1 / tot : 0.0);  // core.py:151
          }
        }
      }
    } else {
      // per-lane rows (irregular tiles): weight first, then normalizedWeight.  The row start
      // is read again here (L2) rather than held through the tile.
      int ln = lane_id();
      asm volatile("" : "+v"(ln));
      const int64_t mk2 = m0 + tmkt(ln);
      const int64_t off = (mk2 < M) ? a.offsets[mk2] : 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (j < u) {
          if (do_u) a.usid[off + j] = (int32_t)key[j];
          if (do_w) a.weight[off + j] = p[j];
        }
      }
      if (do_nw) {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const double v = total > 0.0 ? p[j] / total : 0.0;
          if (j < u) a.nweight[off + j] = v;
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    cur = nxt;
  }
}

}  // namespace


template <bool HYB>
int launch_tab32_t(ConsArgs a, hipStream_t st) {
  const int64_t tiles = (a.n_list + 63) / 64;
  if (tiles == 0) return BCE_OK;
  const int S = a.n_sources > 0 ? a.n_sources : 1;
  const size_t bits = 4 * (size_t)((S + 31) / 32);
  // hybrid: as many rows as fit beside the whole bitmask (16-B aligned)
  a.tab_rows = HYB ? (int)std::min<size_t>(((size_t)kTabLdsBytes - bits) / 16, (size_t)S) : S;
  const size_t lds = 16 * (size_t)a.tab_rows + bits;
  const void* fn = reinterpret_cast<const void*>(&consensus_tab32_kernel<HYB>);
  const int rc = ensure_dynamic_lds(fn, kTabLdsBytes);
  if (rc) return rc;
  const int per_cu = blocks_per_cu(fn, 64 * kTabWaves, lds, 1, HYB ? "consensus_tab32_kernel<hybrid>"
                                                                  : "consensus_tab32_kernel");
  const int64_t blocks = (tiles + kTabWaves - 1) / kTabWaves;
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(blocks < cap ? blocks : cap);
  hipLaunchKernelGGL((consensus_tab32_kernel<HYB>), dim3(grid), dim3(64 * kTabWaves), lds, st, a);
  return check_launch("consensus_tab32_kernel");
}

int launch_tab32(const ConsArgs& a, hipStream_t st) {
  return (a.n_sources <= kTabMaxSources) ? launch_tab32_t<false>(a, st) : launch_tab32_t<true>(a, st);
}

}  // namespace bce
