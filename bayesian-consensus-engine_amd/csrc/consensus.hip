// consensus.hip -- batched core.compute_consensus (core.py:63-179) over CSR markets: every
// kernel except the LDS-table one (consensus_tab.hip), the launchers and the C ABI.
//
// Kernels by market length (launch_seg_for_len / launch_wide_for_len pick them):
//  consensus_pipe_kernel<G>    contiguous markets, n <= G in {8,16,32}, S <= 16384: one
//                              loader wave streams tiles into an LDS ring (LDS-DMA), four
//                              compute waves (lane = market) sort keys in VGPRs and walk
//                              them with 16-B {rel, conf} gathers from global memory.
//  consensus_flat_kernel<G>    contiguous markets, n <= 32, larger tables or compact
//                              outputs: the same arithmetic, each wave loads its own tile.
//  consensus_lpm_kernel<G>     market lists (planned ragged batches), n <= 32: lane per
//                              market, rows staged per market by LDS-DMA.
//  consensus_seg_kernel<64,8>  33 <= n <= 64: cooperative lane-per-signal phase (bitonic
//                              sort, ballots) then lane-per-market ordered sums from LDS.
//  consensus_wide_kernel       64 < n <= 4096 (consensus_wide.hip): one workgroup per
//                              market, register bitonic network over packed (sid, index)
//                              keys, exact chains or BCE_MODE_FAST fixed-order trees.
//  consensus_long_kernel<LDS>  fallback for long markets (LDS or global-scratch sort),
//                              BCE_MODE_FAST fixed-order trees.
// Every kernel sums in the reference's order in BCE_MODE_EXACT (bit-exact outputs).
// FP contraction is off for the whole file: every mul/add rounds like CPython.
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>
#include <algorithm>

#include "consensus_common.hpp"

#pragma clang fp contract(off)

constexpr int kSegWPE = 1;    // __launch_bounds__ min waves per SIMD for the segment kernel
constexpr int kFlatTM = 64;   // flat kernel: markets per wave tile
constexpr int kFlatRing = 8;  // flat kernel: relconf gathers in flight per lane
constexpr int kFlatWPE = 1;   // flat kernel: min waves per SIMD (register budget)
constexpr int kFlatWPB = 2;   // flat kernel: waves per workgroup

namespace bce {

// ------------------------------------------------------------------------------------
// short markets: wave-per-tile, lane-per-signal then lane-per-market
// ------------------------------------------------------------------------------------
template <int G, int TM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kSegWPE, 8)))
void consensus_seg_kernel(ConsArgs a) {
  dev_range(a);
  static_assert(G == 8 || G == 16 || G == 32 || G == 64, "segment width");
  constexpr int SPR = kWave / G;   // segments (markets) per round
  constexpr int R = TM / SPR;      // rounds per tile
  static_assert(R * SPR == TM, "tile must be a whole number of rounds");
  constexpr int LOGG = (G == 8) ? 3 : (G == 16) ? 4 : (G == 32) ? 5 : 6;
  constexpr int RS = G + 1;        // padded LDS row stride (conflict-free transposed reads)
  constexpr int NI = (TM * G + 3 + 4 * kWave - 1) / (4 * kWave);  // 16-B sid chunks per lane
  constexpr int NP = (TM * G + 1 + 2 * kWave - 1) / (2 * kWave);  // 16-B prob chunks per lane

  // One LDS array, carved by hand (cdna guide §5 trap 4a): W | A | B rows (fp64,
  // TM x RS each), then usid rows, per-market scalars and the present bitmask.
  constexpr int ROWS = TM * RS;
  __shared__ double sWAB[3 * ROWS];
  __shared__ int32_t sU[ROWS];
  __shared__ int64_t sOff[TM];
  __shared__ int32_t sN[TM];
  __shared__ int32_t sM[TM];
  __shared__ int32_t sNU[TM];
  __shared__ int32_t sErr[TM];
  __shared__ double sTot[TM];
  __shared__ uint32_t sBits[kBitsLds];
  double* const sW = sWAB;
  double* const sA = sWAB + ROWS;
  double* const sB = sWAB + 2 * ROWS;

  const int lane = lane_id();
  const int seg = lane / G;
  const int t = lane & (G - 1);
  const int seg_base = seg * G;
  const unsigned long long segmask =
      (G >= 64) ? ~0ull : (((1ull << (G & 63)) - 1ull) << seg_base);
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  // present bitmask: staged once per (persistent) workgroup when it fits in LDS
  const int nwords = (a.n_sources + 31) >> 5;
  const bool bits_in_lds = nwords <= kBitsLds;
  if (bits_in_lds)
    for (int i = lane; i < nwords; i += kWave) sBits[i] = a.pbits[i];
  // input staging for contiguous tiles, aliased onto the W|A|B rows (dead until the
  // cooperative phase): sids at sStageI[e - a0] in W, probabilities at sStageP[e - a0p]
  // from A on.
  static_assert(ROWS * 8 >= NI * 4 * kWave * 4, "sid staging fits in the W rows");
  static_assert(2 * ROWS * 8 >= NP * 2 * kWave * 8, "prob staging fits in the A|B rows");
  int32_t* sStageI = reinterpret_cast<int32_t*>(sW);
  double* sStageP = sA;

  const int64_t n_tiles = (a.n_list + TM - 1) / TM;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    // ---- tile metadata -------------------------------------------------------------
    if (lane < TM) {
      const int64_t li = tile * TM + lane;
      int32_t m = -1;
      int64_t off = 0;
      int32_t n = 0;
      if (li < a.n_list) {
        m = a.list ? a.list[li] : (int32_t)li;
        off = a.offsets[m];
        n = (int32_t)(a.offsets[m + 1] - off);
        if (n < 0 || n > G) {  // longer than the launch's max_len: report, skip
          if (a.fault) atomicCAS(a.fault, 0, kFaultTooLong);
          n = 0;
        }
      }
      sM[lane] = m;
      sOff[lane] = off;
      sN[lane] = n;
    }
    __syncthreads();

    // ---- load every round's signals; all loads in flight before the first use -------
    int32_t sidv[R];
    double pv[R];
    bool valid[R];
    if (a.list == nullptr) {
      // contiguous tile: [base, end) streamed with 16-B loads into LDS, then each lane
      // picks its (market, slot) element.
      const int64_t base = sOff[0];
      int64_t end = base;
#pragma unroll
      for (int q = 0; q < TM; ++q) end = (sN[q] > 0) ? sOff[q] + sN[q] : end;
      const int64_t a0 = base & ~3ll, a0p = base & ~1ll;
      int4 vi[NI];
      double2 vp[NP];
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int64_t e = a0 + 4 * (lane + kWave * q);
        vi[q] = make_int4(0, 0, 0, 0);
        if (e < end) {
          if (e + 4 <= a.n_signals) {
            vi[q] = *reinterpret_cast<const int4*>(a.sid + e);
          } else {
            vi[q].x = a.sid[e];
            if (e + 1 < a.n_signals) vi[q].y = a.sid[e + 1];
            if (e + 2 < a.n_signals) vi[q].z = a.sid[e + 2];
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int64_t e = a0p + 2 * (lane + kWave * q);
        vp[q] = make_double2(0.0, 0.0);
        if (e < end) {
          if (e + 2 <= a.n_signals) vp[q] = *reinterpret_cast<const double2*>(a.prob + e);
          else vp[q].x = a.prob[e];
        }
      }
#pragma unroll
      for (int q = 0; q < NI; ++q)
        *reinterpret_cast<int4*>(sStageI + 4 * (lane + kWave * q)) = vi[q];
#pragma unroll
      for (int q = 0; q < NP; ++q)
        *reinterpret_cast<double2*>(sStageP + 2 * (lane + kWave * q)) = vp[q];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int mk = r * SPR + seg;
        valid[r] = t < sN[mk];
        const int64_t p = sOff[mk] + t;
        sidv[r] = valid[r] ? sStageI[p - a0] : 0;
        pv[r] = valid[r] ? sStageP[p - a0p] : 0.0;
      }
      __syncthreads();  // staging (aliased on sA/sB) is dead from here on
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int mk = r * SPR + seg;
        const int32_t n = sN[mk];
        valid[r] = t < n;
        sidv[r] = 0;
        pv[r] = 0.0;
        if (valid[r]) {
          const int64_t p = sOff[mk] + t;
          sidv[r] = a.sid[p];
          pv[r] = a.prob[p];
        }
      }
    }

    // ---- source-table gathers for every round, by ORIGINAL lane, all in flight ------
    // (core.py:110-112): one 16-B {reliability, confidence} load per signal; the sorted
    // lanes later pull the values of the lane that holds the same sid (ds_bpermute), so
    // no L2 round trip sits inside the per-round dependency chain.
    double2 rc[R];
    uint32_t pw[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      rc[r] = make_double2(0.5, 0.25);
      pw[r] = 0xffffffffu;
      if (valid[r]) {
        rc[r] = a.relconf[sidv[r]];
        if (!bits_in_lds) pw[r] = a.pbits[sidv[r] >> 5];
      }
    }

    // ---- cooperative phase -----------------------------------------------------------
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int mk = r * SPR + seg;
      unsigned key = valid[r] ? (((unsigned)sidv[r] << LOGG) | (unsigned)t) : kSent32;
      key = bitonic_sort_seg<G>(key, t);
      const bool kv = key != kSent32;
      const int ssid = (int)(key >> LOGG);
      const int src = seg_base + (int)(key & (G - 1));  // lane holding this signal
      const double ps = pull_f64(pv[r], src);            // probability in sorted order
      const int prev = wave_shr1(ssid, -1);
      const bool first = kv && (t == 0 || prev != ssid);
      const unsigned long long fm = ballot(first);
      const unsigned long long vm = ballot(kv);
      const int j = __popcll(fm & segmask & below);
      // run length of a leader: distance to the next leader / invalid lane / segment end
      const unsigned long long bnd = fm | ~vm;
      const unsigned long long above = (lane == 63) ? 0ull : (bnd >> (lane + 1));
      const int seg_end = seg_base + G;
      int run = above ? (__builtin_ctzll(above) + 1) : (64 - lane);
      if (lane + run > seg_end) run = seg_end - lane;
      const int myrun = first ? run : 1;
      double s = 0.0 + ps;  // builtin sum() starts from int 0 (core.py:116)
      double avg = s;
      if (ballot(myrun > 1)) {  // duplicates: sum the run in input order
        for (int k = 1; k < G; ++k) {
          const int sl = (lane + k < 64) ? lane + k : 63;
          const double pk = pull_f64(ps, sl);
          if (k < myrun) s += pk;
          if (!ballot(k + 1 < myrun)) break;
        }
        avg = (myrun > 1) ? s / (double)myrun : s;
      }
      const double w = pull_f64(rc[r].x, src);  // core.py:111,119
      const double c = pull_f64(rc[r].y, src);  // core.py:112
      const uint32_t word = bits_in_lds ? sBits[ssid >> 5] : (uint32_t)pull_i32((int)pw[r], src);
      if (first) {
        const bool cold = ((word >> (ssid & 31)) & 1u) == 0;  // core.py:167-170
        const int o = mk * RS + j;
        sW[o] = w;
        sA[o] = avg * w;  // core.py:136
        sB[o] = c * w;    // core.py:142
        sU[o] = ssid | (cold ? (int32_t)0x80000000 : 0);
      }
      // validate_input_payload range check (core.py:59-60) on the ORIGINAL order
      const unsigned long long bad =
          ballot(valid[r] && (pv[r] < 0.0 || pv[r] > 1.0)) & segmask;
      if (t == 0) {
        sNU[mk] = __popcll(fm & segmask);
        sErr[mk] = bad ? (int)(__builtin_ctzll(bad) - seg_base) : -1;
      }
    }
    __syncthreads();

    // ---- serial phase: lane = market, exact left-to-right sums (core.py:107-144) ----
    // Fixed trip count with predication so every LDS read can be issued ahead of the
    // dependent adds; adding nothing for j >= u keeps the exact order.
    if (lane < TM) {
      const int u = sNU[lane];
      double total = 0.0, ws = 0.0, cs = 0.0;
      const int base = lane * RS;
      {
#pragma unroll
        for (int jj = 0; jj < G; ++jj) {
          if (jj < u) {
            total += sW[base + jj];
            ws += sA[base + jj];
            cs += sB[base + jj];
          }
        }
      }
      sTot[lane] = total;
      const int32_t m = sM[lane];
      if (m >= 0) {
        const bool null_ = (total == 0.0);
        a.consensus[m] = null_ ? 0.0 : ws / total;
        a.confidence[m] = null_ ? 0.0 : cs / total;
        a.total_weight[m] = total;
        a.n_unique[m] = u;
        if (a.err_idx) a.err_idx[m] = sErr[lane];
      }
    }
    __syncthreads();

    // ---- per-unique outputs (coalesced at CSR offsets) --------------------------------
    if ((a.usid || a.weight || a.nweight)) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int mk = r * SPR + seg;
        if (t < sNU[mk]) {
          const int64_t p = sOff[mk] + t;
          const double w = sW[mk * RS + t];
          const double tot = sTot[mk];
          if (a.usid) a.usid[p] = sU[mk * RS + t];
          if (a.weight) a.weight[p] = w;
          if (a.nweight) a.nweight[p] = (tot > 0.0) ? w / tot : 0.0;  // core.py:151
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// short markets, lane per market: consensus_lpm_kernel<G>  (n <= G, G in {8, 16, 32})
// ------------------------------------------------------------------------------------
// LDS ordering inside a single-wave workgroup: the wave's LDS instructions execute in
// order, so a compiler barrier + lgkmcnt drain is all a cross-lane hand-off needs.
__device__ __forceinline__ void wave_sync() {
  __syncthreads();
}

__device__ __forceinline__ void dma4(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

template <int G>
__global__ __launch_bounds__(64) void consensus_lpm_kernel(ConsArgs a) {
  dev_range(a);
  static_assert(G == 8 || G == 16 || G == 32, "lane-per-market widths");
  constexpr int LOGG = (G == 8) ? 3 : (G == 16) ? 4 : 5;
  constexpr int SST = G + 1;       // sid / usid row stride (dwords): conflict-free b32 reads
  constexpr int PST = 2 * G + 2;   // prob / weight row stride (dwords, even -> 8-B aligned)
  constexpr int RING = 8;          // gathers issued this many sorted positions ahead
  constexpr int MPI = kWave / G;   // markets per copy-out iteration

  __shared__ uint32_t sS[kWave * SST];  // sid rows; after the walk: usid rows
  __shared__ uint32_t sP[kWave * PST];  // prob rows; after the sorted read: weight rows
  __shared__ int64_t sOff[kWave];
  __shared__ int32_t sU[kWave];
  __shared__ double sTot[kWave];

  const int lane = lane_id();
  const int64_t n_tiles = (a.n_list + kWave - 1) / kWave;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    // ---- this lane's market ---------------------------------------------------------
    const int64_t li = tile * kWave + lane;
    int32_t mk = -1;
    int64_t off = 0;
    int n = 0;
    if (li < a.n_list) {
      mk = a.list ? a.list[li] : (int32_t)li;
      off = a.offsets[mk];
      n = (int)(a.offsets[mk + 1] - off);
    }
    if (ballot(n < 0 || n > G)) {  // longer than the launch's max_len: report, skip
      raise_fault(a.fault, kFaultTooLong);
      if (n < 0 || n > G) n = 0;
    }

    unsigned key[G];
    double sp[G];
    int err = -1;
    // ---- rows -> LDS by LDS-DMA: one dword per lane, market by market --------------
    for (int q = 0; q < kWave; ++q) {
      const int nq = __builtin_amdgcn_readlane(n, q);
      if (nq == 0) continue;
      const int64_t oq = ((int64_t)__builtin_amdgcn_readlane((int)(off >> 32), q) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)off, q);
      if (lane < nq) dma4(a.sid + oq + lane, sS + q * SST);
      if (lane < 2 * nq) dma4(reinterpret_cast<const uint32_t*>(a.prob + oq) + lane, sP + q * PST);
      if (2 * nq > kWave && lane < 2 * nq - kWave)
        dma4(reinterpret_cast<const uint32_t*>(a.prob + oq) + kWave + lane, sP + q * PST + kWave);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    const uint32_t* rowS = sS + lane * SST;
    const double* rowP = reinterpret_cast<const double*>(sP + lane * PST);
    // keys (sid, slot) and the validation scan in input order
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const bool v = t < n;
      key[t] = v ? ((rowS[t] << LOGG) | (unsigned)t) : kSent32;
      const double p = rowP[t];
      if (v && err < 0 && (p < 0.0 || p > 1.0)) err = t;  // core.py:59-60 (NaN passes)
    }
    oem_sort<G>(key);
    // probabilities in sorted order (registers); the rows become output staging
#pragma unroll
    for (int t = 0; t < G; ++t) sp[t] = rowP[key[t] & (G - 1)];
    wave_sync();
    // ---- walk in sorted order: runs summed in input order (core.py:116), then the
    //      reference's left-to-right totals over unique sources (core.py:107-144) -----
    uint32_t* outS = sS + lane * SST;                         // usid of unique j
    double* outW = reinterpret_cast<double*>(sP + lane * PST);  // weight of unique j
    double2 rc[RING];
    uint32_t pw[RING];
#pragma unroll
    for (int t = 0; t < RING && t < G; ++t) {
      const bool kv = key[t] != kSent32;
      const int sid = (int)(key[t] >> LOGG);
      const bool fst = kv && (t == 0 || sid != (int)(key[t - 1 > 0 ? t - 1 : 0] >> LOGG));
      if (fst) {
        rc[t] = a.relconf[sid];
        pw[t] = a.pbits[sid >> 5];
      } else {
        rc[t] = make_double2(0.5, 0.25);
        pw[t] = 0xffffffffu;
      }
    }
    double total = 0.0, ws = 0.0, cs = 0.0;
    double psum = 0.0;
    int cnt = 0, j = 0, psid = 0;
    double2 prc = make_double2(0.0, 0.0);
    uint32_t ppw = 0;
    auto finalize = [&]() {
      double avg = psum;
      if (ballot(cnt > 1)) {  // duplicates: avg = sum / len (core.py:116), rare
        if (cnt > 1) avg = psum / (double)cnt;
      }
      const double w = prc.x, c = prc.y;
      total += w;          // core.py:120
      ws += avg * w;       // core.py:135-137
      cs += c * w;         // core.py:141-143
      const bool cold = ((ppw >> (psid & 31)) & 1u) == 0;  // core.py:167-170
      outS[j] = (uint32_t)psid | (cold ? 0x80000000u : 0u);
      outW[j] = w;
      ++j;
    };
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const bool kv = key[t] != kSent32;
      const int sid = (int)(key[t] >> LOGG);
      const bool fst = kv && (t == 0 || sid != (int)(key[t > 0 ? t - 1 : 0] >> LOGG));
      if (fst) {
        if (cnt > 0) finalize();
        psid = sid;
        prc = rc[t % RING];
        ppw = pw[t % RING];
        psum = 0.0 + sp[t];  // builtin sum() starts from int 0
        cnt = 1;
      } else if (kv) {
        psum += sp[t];
        ++cnt;
      }
      if (t + RING < G) {  // refill the ring slot just consumed
        const int tt = t + RING;
        const bool kv2 = key[tt] != kSent32;
        const int sid2 = (int)(key[tt] >> LOGG);
        const bool fst2 = kv2 && sid2 != (int)(key[tt - 1] >> LOGG);
        if (fst2) {
          rc[tt % RING] = a.relconf[sid2];
          pw[tt % RING] = a.pbits[sid2 >> 5];
        }
      }
    }
    if (cnt > 0) finalize();

    // ---- per-market results (lane = market: coalesced) ------------------------------
    if (mk >= 0) {
      const bool null_ = (total == 0.0);  // core.py:131-133
      a.consensus[mk] = null_ ? 0.0 : ws / total;
      a.confidence[mk] = null_ ? 0.0 : cs / total;
      a.total_weight[mk] = total;
      a.n_unique[mk] = j;
      if (a.err_idx) a.err_idx[mk] = err;
    }
    sOff[lane] = off;
    sU[lane] = (mk >= 0) ? j : 0;
    sTot[lane] = total;
    wave_sync();

    // ---- per-unique outputs: MPI markets per iteration, lane = slot (coalesced) ------
    if ((a.usid || a.weight || a.nweight)) {
      const int slot = lane & (G - 1);
#pragma unroll 4
      for (int it = 0; it < G; ++it) {
        const int q = it * MPI + lane / G;
        if (slot < sU[q]) {
          const int64_t p = sOff[q] + slot;
          const double w = reinterpret_cast<const double*>(sP + q * PST)[slot];
          const double tot = sTot[q];
          if (a.usid) a.usid[p] = (int32_t)sS[q * SST + slot];
          if (a.weight) a.weight[p] = w;
          if (a.nweight) a.nweight[p] = (tot > 0.0) ? w / tot : 0.0;  // core.py:151
        }
      }
    }
    wave_sync();
  }
}

// ------------------------------------------------------------------------------------
// contiguous short markets, lane per market: consensus_flat_kernel<G, TM, WPB>
// ------------------------------------------------------------------------------------
// The headline path (list == NULL, every n <= G).  WPB independent waves per workgroup
// share only the present bitmask; each wave owns a tile of TM consecutive markets whose
// signals form ONE contiguous range [B, E):
//   1. B, E by scalar loads; the range is streamed into the wave's LDS image with 16-B
//      LDS-DMA (global_load_lds_dwordx4): ceil(TM*G*12 / 1 KiB) wave-instructions, no
//      per-market loop, no VGPR staging.
//   2. lane = market: its sids -> 32-bit keys (sid << log2 G | slot), Batcher odd-even
//      merge network in VGPRs.
//   3. walk in sorted order (branch-free): probability of the sorted slot from LDS,
//      duplicate runs summed in input order (core.py:115-116), one 16-B relconf gather
//      per position (ring RING ahead), and the reference's left-to-right totals over
//      unique sources (core.py:120, 135-143) gated by "last of its run".  The range
//      check of core.py:59-60 is the minimum failing slot.  Per unique j the packed
//      (sid | slot << 25) goes to the (dead) sid image at j and the weight over the
//      (consumed) probability cell of that slot.
//   4. per-market scalars (lane = market, coalesced); per-unique outputs with G/2 lanes
//      per market, two slots per lane: 8-B usid pairs and 16-B weight/nweight pairs.
constexpr int kPackSlot = 25;  // packed = sid | slot << 25 (sid < 2^25)
// global (not constant) address space: selected against the relconf argument, a constant
// pointer would turn the gathers into flat loads (vmcnt + lgkmcnt, out of order)
__device__ double2 kColdRow[1] = {{0.5, 0.25}};  // DEFAULT_RELIABILITY / _CONFIDENCE

template <int G, int TM, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(kFlatWPE, 8)))
void consensus_flat_kernel(ConsArgs a) {
  static_assert(G == 8 || G == 16 || G == 32, "flat widths");
  static_assert(TM == 32 || TM == 64, "markets per wave tile");
  constexpr int LOGG = (G == 8) ? 3 : (G == 16) ? 4 : 5;
  constexpr int TS = TM * G;           // max signals per tile
  constexpr int SW = TS + 8 + G;       // sid image (dwords): alignment slack, row overrun, sink
  constexpr int PW = TS + 4 + G;       // prob image (doubles)
  constexpr int RING = kFlatRing;
  constexpr int P = G / 2;             // lanes per market in the copy-out (2 slots each)
  constexpr int MPI = kWave / P;       // markets per copy-out iteration

  __shared__ uint32_t sBits[kBitsLds];
  __shared__ __attribute__((aligned(16))) uint32_t sSid[WPB][SW];
  __shared__ __attribute__((aligned(16))) double sProb[WPB][PW];
  __shared__ double sTot[WPB][TM];
  __shared__ int32_t sU[WPB][TM];
  __shared__ int32_t sRs[WPB][TM];

  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwords = (a.n_sources + 31) >> 5;
  const bool bits_in_lds = nwords <= kBitsLds;
  if (bits_in_lds)
    for (int i = threadIdx.x; i < nwords; i += 64 * WPB) sBits[i] = a.pbits[i];
  __syncthreads();  // the only workgroup barrier: waves are independent from here on

  uint32_t* const iS = sSid[w];
  double* const iP = sProb[w];
  const int64_t M = a.n_list;
  const int64_t n_tiles = (M + TM - 1) / TM;
  for (int64_t tile = (int64_t)blockIdx.x * WPB + w; tile < n_tiles; tile += (int64_t)gridDim.x * WPB) {
    const int64_t m0 = tile * TM;
    const int64_t m1 = (m0 + TM < M) ? m0 + TM : M;
    const int64_t B = a.offsets[m0];   // wave-uniform: scalar loads
    const int64_t E = a.offsets[m1];
    const int64_t Bs = B & ~3ll, Bp = B & ~1ll;

    // ---- this lane's market ------------------------------------------------------------
    const int64_t mk = m0 + lane;
    const bool has = lane < TM && mk < M;
    int64_t off = B;
    int n = 0;
    if (has) {
      off = a.offsets[mk];
      n = (int)(a.offsets[mk + 1] - off);
    }
    if (ballot(n < 0 || n > G)) {  // longer than the launch's max_len: report, skip
      raise_fault(a.fault, kFaultTooLong);
      if (n < 0 || n > G) n = 0;
    }

    // ---- 1. stream [B, E) into the LDS image (16-B LDS-DMA, full chunks in bounds) -------
    {
      const int64_t Nf4 = a.n_signals & ~3ll;                  // last full 4-sid chunk end
      const int64_t es = (E < Nf4) ? ((E + 3) & ~3ll) : Nf4;   // DMA end (sids)
      const int nci = (int)((es - Bs) >> 2);                   // 16-B chunks
      for (int i = 0; i * kWave < nci; ++i) {
        const int c = i * kWave + lane;
        if (c < nci)
          __builtin_amdgcn_global_load_lds(a.sid + Bs + 4 * c,
                                           (__attribute__((address_space(3))) void*)(iS + i * 256), 16, 0, 0);
      }
      const int64_t Nf2 = a.n_signals & ~1ll;
      const int64_t ep = (E < Nf2) ? ((E + 1) & ~1ll) : Nf2;
      const int ncp = (int)((ep - Bp) >> 1);
      for (int i = 0; i * kWave < ncp; ++i) {
        const int c = i * kWave + lane;
        if (c < ncp)
          __builtin_amdgcn_global_load_lds(a.prob + Bp + 2 * c,
                                           (__attribute__((address_space(3))) void*)(iP + i * 128), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // tail of the arrays that does not fill a 16-B chunk (last tile only)
      if (E > es && lane < (int)(E - es)) iS[es - Bs + lane] = (uint32_t)a.sid[es + lane];
      if (E > ep && lane < (int)(E - ep)) iP[ep - Bp + lane] = a.prob[ep + lane];
      wave_sync_lds();
    }

    // ---- 2. keys + sort ------------------------------------------------------------------
    const int rs = (int)(off - B);            // row start relative to B
    const int rsi = rs + (int)(B - Bs);       // ... in the sid image
    const int rsp = rs + (int)(B - Bp);       // ... in the prob image
    unsigned key[G];
    if (ballot(has && (rsi & 3) != 0) == 0) {
#pragma unroll
      for (int c = 0; c < G / 4; ++c) {
        const uint4 v = *reinterpret_cast<const uint4*>(iS + rsi + 4 * c);
        key[4 * c] = v.x; key[4 * c + 1] = v.y; key[4 * c + 2] = v.z; key[4 * c + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < G; ++t) key[t] = iS[rsi + t];
    }
#pragma unroll
    for (int t = 0; t < G; ++t) key[t] = (t < n) ? ((key[t] << LOGG) | (unsigned)t) : kSent32;
    oem_sort<G>(key);
    // run structure as bit masks in one VGPR each (bit t: position t is the first / last
    // position of its sid run); valid positions are exactly t < n after the sort
    unsigned fb = 0, lb = 0;
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const unsigned s = key[t] >> LOGG;
      const bool kv = key[t] != kSent32;
      const bool f = kv && (t == 0 || s != (key[t > 0 ? t - 1 : 0] >> LOGG));
      const bool l = kv && (t == G - 1 || s != (key[t < G - 1 ? t + 1 : t] >> LOGG));
      fb |= (f ? 1u : 0u) << t;
      lb |= (l ? 1u : 0u) << t;
    }
    unsigned vb = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);  // valid positions
    // opaque to the optimiser: otherwise it folds the bit tests back into the per-position
    // compare masks and keeps ~3*G of them alive in SGPRs across the walk (spills)
    asm volatile("" : "+v"(fb), "+v"(lb), "+v"(vb));
    // ---- 3. walk: every input of every position in registers before the ordered sums -----
    wave_sync_lds();  // every lane has read its sids: rows may be rewritten
    double sp[G];
#pragma unroll
    for (int t = 0; t < G; ++t) sp[t] = iP[rsp + (int)(key[t] & (G - 1))];  // sentinel: slot G-1, in the image
    // gathers: index clamped into the table (sentinels and out-of-range sids never fault;
    // their values are never used), no per-position branch
    const unsigned smax = (unsigned)(a.n_sources > 0 ? a.n_sources - 1 : 0);
    const bool have_tab = a.n_sources > 0;
    constexpr int NG = (G < RING) ? G : RING;  // gathers in flight
    double2 ring[NG];
#pragma unroll
    for (int t = 0; t < NG; ++t) {
      const unsigned ix = min(key[t] >> LOGG, smax);
      ring[t] = (have_tab) ? a.relconf[ix] : make_double2(0.5, 0.25);
    }
    const int dumS = SW - 1, dumP = PW - 1;  // write sinks for invalid positions
    double total = 0.0, ws = 0.0, cs = 0.0, psum = 0.0;
    int cnt = 0, j = 0, err = G;
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const bool kv = (vb >> t) & 1u;
      const unsigned sid = key[t] >> LOGG;
      const int slot = (int)(key[t] & (G - 1));
      const bool fst = (fb >> t) & 1u;
      const bool lst = (lb >> t) & 1u;
      const double p = sp[t];
      const double2 rc = ring[t % NG];
      if (t + NG < G) {
        const unsigned ix = min(key[t + NG < G ? t + NG : t] >> LOGG, smax);
        if (have_tab) ring[t % NG] = a.relconf[ix];
      }
      if (kv && (p < 0.0 || p > 1.0)) err = (slot < err) ? slot : err;  // core.py:59-60
      psum = (fst ? 0.0 : psum) + p;   // builtin sum() from int 0 (core.py:116)
      cnt = fst ? 1 : cnt + 1;
      double avg = psum;
      if (ballot(lst && cnt > 1)) {     // duplicates: sum / len (core.py:116), rare
        if (lst && cnt > 1) avg = psum / (double)cnt;
      }
      const double wt = rc.x, cf = rc.y;
      // accumulate only at the last position of a run; +0.0 leaves every chain bit-exact
      // (the chains start at +0.0 and can never become -0.0)
      total += lst ? wt : 0.0;          // core.py:120
      ws += lst ? avg * wt : 0.0;       // core.py:135-137
      cs += lst ? cf * wt : 0.0;        // core.py:141-143
      // j <= t: the row cell is dead; the slot's probability is already in registers
      iS[kv ? rsi + j : dumS] = sid | ((unsigned)slot << kPackSlot);
      iP[kv ? rsp + slot : dumP] = wt;
      j += lst ? 1 : 0;
      // pin the chains here: left alone the compiler sinks every add to the end of the
      // walk and keeps all per-position operands and masks alive
      asm volatile("" : "+v"(total), "+v"(ws), "+v"(cs), "+v"(psum), "+v"(j), "+v"(cnt), "+v"(err));
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- 4a. per-market results --------------------------------------------------------
    if (has) {
      const bool null_ = (total == 0.0);  // core.py:131-133
      a.consensus[mk] = null_ ? 0.0 : ws / total;
      a.confidence[mk] = null_ ? 0.0 : cs / total;
      a.total_weight[mk] = total;
      a.n_unique[mk] = j;
      if (a.err_idx) a.err_idx[mk] = (err < G) ? err : -1;
    }
    if (lane < TM) {
      sTot[w][lane] = total;
      sU[w][lane] = has ? j : 0;
      sRs[w][lane] = rs;
    }
    wave_sync_lds();

    // ---- 4b. per-unique outputs ---------------------------------------------------------
    if ((a.usid || a.weight || a.nweight)) {
      const int dB = (int)(B - Bs), dP = (int)(B - Bp);
      const bool vec_ok = (((uintptr_t)a.usid & 7) | ((uintptr_t)a.weight & 15) | ((uintptr_t)a.nweight & 15)) == 0;
      if (vec_ok && ballot(has && (off & 1) != 0) == 0 && (B & 1) == 0) {
        // even offsets: slot pairs are 8-B (usid) / 16-B (weights) aligned
        const int k2 = 2 * (lane % P);
#pragma unroll 1
        for (int it = 0; it < TM / MPI; ++it) {
          const int q = it * MPI + lane / P;
          const int u = sU[w][q];
          if (k2 < u) {
            const int r = sRs[w][q];
            const double tot = sTot[w][q];
            const int64_t pos = B + r + k2;
            const bool two = k2 + 1 < u;
            const unsigned pk0 = iS[dB + r + k2];
            const unsigned pk1 = two ? iS[dB + r + k2 + 1] : 0u;
            const unsigned s0 = pk0 & ((1u << kPackSlot) - 1), s1 = pk1 & ((1u << kPackSlot) - 1);
            const double w0 = iP[dP + r + (int)(pk0 >> kPackSlot)];
            const double w1 = iP[dP + r + (int)(pk1 >> kPackSlot)];
            const bool p0 = bits_in_lds ? is_present(sBits, (int)s0) : is_present(a.pbits, (int)s0);
            const bool p1 = two && (bits_in_lds ? is_present(sBits, (int)s1) : is_present(a.pbits, (int)s1));
            const unsigned u0 = s0 | (p0 ? 0u : 0x80000000u);  // core.py:167-170
            const unsigned u1 = s1 | (p1 ? 0u : 0x80000000u);
            const double n0 = (tot > 0.0) ? w0 / tot : 0.0;    // core.py:151
            const double n1 = (tot > 0.0) ? w1 / tot : 0.0;
            if (two) {
              if (a.usid) *reinterpret_cast<uint2*>(a.usid + pos) = make_uint2(u0, u1);
              if (a.weight) *reinterpret_cast<double2*>(a.weight + pos) = make_double2(w0, w1);
              if (a.nweight) *reinterpret_cast<double2*>(a.nweight + pos) = make_double2(n0, n1);
            } else {
              if (a.usid) a.usid[pos] = (int32_t)u0;
              if (a.weight) a.weight[pos] = w0;
              if (a.nweight) a.nweight[pos] = n0;
            }
          }
        }
      } else {
        const int slot = lane % G;
#pragma unroll 1
        for (int it = 0; it < TM / (kWave / G); ++it) {
          const int q = it * (kWave / G) + lane / G;
          if (slot < sU[w][q]) {
            const int r = sRs[w][q];
            const double tot = sTot[w][q];
            const unsigned pk = iS[dB + r + slot];
            const unsigned s = pk & ((1u << kPackSlot) - 1);
            const double wt = iP[dP + r + (int)(pk >> kPackSlot)];
            const bool pr = bits_in_lds ? is_present(sBits, (int)s) : is_present(a.pbits, (int)s);
            const int64_t pos = B + r + slot;
            if (a.usid) a.usid[pos] = (int32_t)(s | (pr ? 0u : 0x80000000u));
            if (a.weight) a.weight[pos] = wt;
            if (a.nweight) a.nweight[pos] = (tot > 0.0) ? wt / tot : 0.0;
          }
        }
      }
    }
    wave_sync_lds();  // the next tile's DMA overwrites the images
  }
}

// ------------------------------------------------------------------------------------
// consensus_pipe_kernel<G, C, R>: one loader wave + C compute waves per workgroup
// ------------------------------------------------------------------------------------
// The headline schedule.  Per workgroup (one per CU) an LDS ring of R tile slots:
//   loader wave   streams tile after tile into free slots with LDS-DMA, a FIXED number
//                 of 16-B wave-instructions per tile (lanes past the tile's range re-read
//                 its first chunk into the slot's slack), so `s_waitcnt vmcnt(NDMA)`
//                 publishes tile i-1 while tile i is still in flight (two tiles deep);
//   compute waves grab tiles in sequence (LDS counter), wait for the slot's ready flag,
//                 and run the flat kernel's arithmetic on it: keys + odd-even merge sort
//                 in VGPRs, the walk with 16 relconf gathers in flight and the sorted-slot
//                 probabilities read from the slot just ahead of use, per-unique results
//                 staged in place (packed sid|slot over the dead sid row, the weight over
//                 the consumed probability cell), coalesced copy-out with 16-B pairs, then
//                 release the slot.
// A compute wave never issues an LDS-DMA, so none of its waits covers one; the loader
// never touches registers the compute waves need.  Flags live in LDS (one workgroup).
// Progress: the loader only waits for the release of sequence i-R, which a compute wave
// is processing or has released (sequences are grabbed in order and R > C).
constexpr int kPipeRing = 16;  // relconf gathers in flight per compute lane

constexpr int kPipeC32 = 4;  // compute waves at G = 32
constexpr int kPipeR32 = 6;  // slots at G = 32 (LDS: ~25 KB each)
// Slots R >= C + 2: with one spare slot the ring is load-latency bound (a released slot
// must be refilled within tile_time / C); two spares keep two tiles in flight.
template <int G>
struct PipeCfg {
  static constexpr int L = 1;  // one loader wave (two measured slower: TA contention)
  static constexpr int C = (G == 32) ? kPipeC32 : 6;
  static constexpr int R = (G == 32) ? kPipeR32 : C + 3;
};

template <int G>
__global__ __launch_bounds__(64 * (PipeCfg<G>::C + PipeCfg<G>::L))
void consensus_pipe_kernel(ConsArgs a) {
  static_assert(G == 8 || G == 16 || G == 32, "pipe widths");
  constexpr int C = PipeCfg<G>::C, R = PipeCfg<G>::R, NL = PipeCfg<G>::L;
  constexpr int TM = kWave;
  constexpr int LOGG = (G == 8) ? 3 : (G == 16) ? 4 : 5;
  constexpr int TS = TM * G;
  // Fixed DMA shape per tile: body instructions cover chunks [64k, 64k + 64) of the
  // tile's range, one tail instruction covers its LAST 64 chunks [n - 64, n) (the same
  // bytes again where they overlap), so the image is only as long as the largest range
  // and the wave-instruction count never depends on the data.
  constexpr int SCH = (TS + 6) / 4 + 1;   // max 16-B sid chunks of a tile (misaligned start)
  constexpr int PCH = (TS + 2) / 2 + 1;   // max 16-B prob chunks
  constexpr int OCH = 2 * (TM + 1);       // offsets block dwords
  constexpr int NSI = SCH / kWave + 1;    // body + tail
  constexpr int NPI = PCH / kWave + 1;
  constexpr int NOI = OCH / kWave + 1;
  constexpr int NDMA = NSI + NPI + NOI;
  static_assert(NDMA < 64, "vmcnt field");
  constexpr int SW = (4 * SCH > TS + 4 + G) ? 4 * SCH : TS + 4 + G;  // sid image dwords (row overrun)
  constexpr int PW = (2 * PCH > TS + 4 + G) ? 2 * PCH : TS + 4 + G;  // prob image doubles
  constexpr int OW = OCH + 2;
  static_assert(4 * kWave * (NSI - 1) <= SW && 2 * kWave * (NPI - 1) <= PW && kWave * (NOI - 1) <= OW,
                "every body-instruction lane lands inside its image");
  constexpr int RING = kPipeRing;
  constexpr int NG = (G < RING) ? G : RING;
  constexpr int PA = 4;          // probabilities read this many positions ahead

  __shared__ uint32_t sBits[kBitsLds];
  __shared__ __attribute__((aligned(16))) uint32_t sSid[R][SW];
  __shared__ __attribute__((aligned(16))) double sProb[R][PW];
  __shared__ __attribute__((aligned(16))) uint32_t sOffs[R][OW];
  __shared__ int64_t sTile[R];
  __shared__ int sReady[R];  // sequence + 1 once the slot holds it
  __shared__ int sFree[R];   // sequence + 1 once the slot's tile has been released
  __shared__ int sNext;
  __shared__ uint32_t sBad[R][TS / 32 + 2];  // bit i: prob of tile position i outside [0, 1]
  __shared__ uint4 sInfo[C][TM];  // per market: {rs, u | n << 8 | rot << 16, total (lo, hi)}

  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // present bits staged in LDS up to 16384 sources; larger tables read them from global
  // memory (one 4-B gather per unique source, L2-resident: S/8 bytes)
  const int nwords = (a.n_sources + 31) >> 5;
  const bool bits_in_lds = nwords <= kBitsLds;
  if (bits_in_lds)
    for (int i = threadIdx.x; i < nwords; i += 64 * (C + NL)) sBits[i] = a.pbits[i];
  if (threadIdx.x < R) {
    sReady[threadIdx.x] = 0;
    sFree[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) sNext = 0;
  __syncthreads();  // the only workgroup barrier

  const int64_t M = a.n_list;
  const int64_t n_tiles = (M + TM - 1) / TM;

  if (w < NL) {
    // ================================ loaders =========================================
    // loader w owns sequences i = w, w + NL, ... (slot i % R); k counts its own tiles
    const int64_t Nf4 = a.n_signals & ~3ll, Nf2 = a.n_signals & ~1ll;
    const int64_t clamp_s = (Nf4 - 4 > 0) ? Nf4 - 4 : 0;  // host: n_signals >= 4
    const int64_t clamp_p = (Nf2 - 2 > 0) ? Nf2 - 2 : 0;
    int64_t tbB = 0, tbE = 0;
    auto load_bounds = [&](int64_t kbase) {
      const int64_t t = (int64_t)blockIdx.x + (w + (kbase + lane) * NL) * gridDim.x;
      if (t < n_tiles) {
        const int64_t m0 = t * TM;
        tbB = a.offsets[m0];
        tbE = a.offsets[(m0 + TM < M) ? m0 + TM : M];
      }
    };
    auto rl = [&](int64_t v, int i) -> int64_t {
      return ((int64_t)__builtin_amdgcn_readlane((int)(v >> 32), i) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)v, i);
    };
    // validation (core.py:59-60) for the compute waves: the tail of the arrays that no
    // 16-B chunk covers is loaded here, then every position's range check becomes one bit
    // of sBad (ballot per 64 positions, contiguous conflict-free reads); NaN passes
    auto finish = [&](int s, int64_t B, int64_t E) {
      const int64_t Bs = B & ~3ll, Bp = B & ~1ll;
      const int64_t es = (E < Nf4) ? ((E + 3) & ~3ll) : Nf4;
      const int64_t ep = (E < Nf2) ? ((E + 1) & ~1ll) : Nf2;
      if (E > es && lane < (int)(E - es)) sSid[s][es - Bs + lane] = (uint32_t)a.sid[es + lane];
      if (E > ep && lane < (int)(E - ep)) sProb[s][ep - Bp + lane] = a.prob[ep + lane];
      wave_sync_lds();
      const int nb = (int)(E - B), d = (int)(B - Bp);
#pragma unroll 4
      for (int k = 0; k < TS / kWave; ++k) {
        const int i = k * kWave + lane;
        const double p = sProb[s][d + ((i < nb) ? i : 0)];
        const unsigned long long m = ballot(i < nb && (p < 0.0 || p > 1.0));
        sBad[s][2 * k] = (uint32_t)m;
        sBad[s][2 * k + 1] = (uint32_t)(m >> 32);
      }
      wave_sync_lds();
    };
    auto publish = [&](int seq, int64_t t) {
      const int s = seq % R;
      // every lane stores the same words: no lane-0-only region inside the loop (the
      // structurizer splits loops around such regions and breaks wave-uniform state)
      sTile[s] = t;
      __hip_atomic_store(&sReady[s], seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    const int64_t my_tiles = (n_tiles > (int64_t)blockIdx.x) ? (n_tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    int pending = -1;  // sequence whose DMA is in flight and not yet published
    int64_t pend_t = -1, pend_B = 0, pend_E = 0;
    for (int64_t i = w, k = 0; i < my_tiles + C; i += NL, ++k) {
      const int s = (int)(i % R);
      // wait for the release of sequence i - R (publish what is in flight first)
      if (i >= R) {
        const int need = (int)(i - R) + 1;
        if (ldsflag(&sFree[s]) < need) {
          if (pending >= 0) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            finish(pending % R, pend_B, pend_E);
            publish(pending, pend_t);
            pending = -1;
          }
          int spins = 0;
          while (ldsflag(&sFree[s]) < need) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > a.spin_cap) {  // never expected: bounded so a bug cannot hang the GPU,
              raise_fault(a.fault, kFaultSpinLoader);  // and reported (bce_fault_check)
              return;
            }
          }
        }
      }
      if (i >= my_tiles) {  // end markers: one per compute wave
        if (pending >= 0) {
          __builtin_amdgcn_s_waitcnt(0x0F70);
          finish(pending % R, pend_B, pend_E);
            publish(pending, pend_t);
          pending = -1;
        }
        publish((int)i, -1);
        continue;
      }
      if ((k & 63) == 0) {
        load_bounds(k);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // (drains in-flight DMA too; once per 64 tiles)
        if (pending >= 0) {
          finish(pending % R, pend_B, pend_E);
            publish(pending, pend_t);
          pending = -1;
        }
      }
      const int64_t t = (int64_t)blockIdx.x + i * gridDim.x;
      const int64_t B = rl(tbB, (int)(k & 63)), E = rl(tbE, (int)(k & 63));
      const int64_t m0 = t * TM, m1 = (m0 + TM < M) ? m0 + TM : M;
      const int64_t Bs = B & ~3ll, Bp = B & ~1ll;
      const int64_t es = (E < Nf4) ? ((E + 3) & ~3ll) : Nf4;
      const int64_t ep = (E < Nf2) ? ((E + 1) & ~1ll) : Nf2;
      const int nci = (int)((es - Bs) >> 2), ncp = (int)((ep - Bp) >> 1);
      const int ndw = (int)(2 * (m1 - m0 + 1));
      const int64_t fs = (Bs < clamp_s) ? Bs : clamp_s, fp = (Bp < clamp_p) ? Bp : clamp_p;
      // body instruction k covers chunks [64k, 64k + 64) (lanes past the range re-read the
      // first chunk into slack the range never reaches); once the range is exhausted a body
      // instruction repeats instruction 0 (same bytes to the same places); the tail
      // instruction covers the range's last 64 chunks (from 0 if it is shorter)
#pragma unroll
      for (int k = 0; k < NSI - 1; ++k) {
        const int kk = (k * kWave < nci) ? k : 0;
        const int c = kk * kWave + lane;
        dma_b128(a.sid + ((c < nci) ? Bs + 4 * c : fs), &sSid[s][kk * 256]);
      }
      {
        const int tb = (nci > kWave) ? nci - kWave : 0;
        const int c = tb + lane;
        dma_b128(a.sid + ((c < nci) ? Bs + 4 * c : fs), &sSid[s][tb * 4]);
      }
#pragma unroll
      for (int k = 0; k < NPI - 1; ++k) {
        const int kk = (k * kWave < ncp) ? k : 0;
        const int c = kk * kWave + lane;
        dma_b128(a.prob + ((c < ncp) ? Bp + 2 * c : fp), &sProb[s][kk * 128]);
      }
      {
        const int tb = (ncp > kWave) ? ncp - kWave : 0;
        const int c = tb + lane;
        dma_b128(a.prob + ((c < ncp) ? Bp + 2 * c : fp), &sProb[s][tb * 2]);
      }
      const uint32_t* og = reinterpret_cast<const uint32_t*>(a.offsets + m0);
#pragma unroll
      for (int k = 0; k < NOI - 1; ++k) {
        const int kk = (k * kWave < ndw) ? k : 0;
        const int d = kk * kWave + lane;
        dma_b32(og + ((d < ndw) ? d : 0), &sOffs[s][kk * 64]);
      }
      {
        const int tb = (ndw > kWave) ? ndw - kWave : 0;
        const int d = tb + lane;
        dma_b32(og + ((d < ndw) ? d : 0), &sOffs[s][tb]);
      }
      if (pending >= 0) {  // the previous tile has landed once only this one is in flight
        __builtin_amdgcn_s_waitcnt((NDMA & 15) | (7 << 4) | (15 << 8) | ((NDMA >> 4) << 14));
        finish(pending % R, pend_B, pend_E);
        publish(pending, pend_t);
      }
      pending = (int)i;
      pend_t = t;
      pend_B = B;
      pend_E = E;
    }
    if (pending >= 0) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      finish(pending % R, pend_B, pend_E);
      publish(pending, pend_t);
    }
    return;
  }

  // ================================ compute waves =====================================
  const int cw = w - NL;
  const unsigned smax = (unsigned)(a.n_sources > 0 ? a.n_sources - 1 : 0);
  const double2* const tab = (a.n_sources > 0) ? a.relconf : kColdRow;
  const int64_t Nf4 = a.n_signals & ~3ll, Nf2 = a.n_signals & ~1ll;
  for (;;) {
    // every lane takes a ticket (one aggregated ds_add of 64 per wave): the wave's
    // sequence number is its first ticket / 64
    const int tk = __hip_atomic_fetch_add(&sNext, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int seq = __builtin_amdgcn_readfirstlane(tk) >> 6;
    const int s = seq % R;
    int spins = 0;
    while (ldsflag(&sReady[s]) != seq + 1) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > a.spin_cap) {  // never expected: bounded so a bug cannot hang the GPU,
        raise_fault(a.fault, kFaultSpinCompute);  // and reported (bce_fault_check)
        return;
      }
    }
    const int64_t tile0 = sTile[s];
    const int64_t tile = ((int64_t)__builtin_amdgcn_readfirstlane((int)(tile0 >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)tile0);  // uniform
    if (tile < 0) {
      __hip_atomic_store(&sFree[s], seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    uint32_t* const iS = sSid[s];
    double* const iP = sProb[s];
    const uint32_t* const iO = sOffs[s];
    int ln = lane_id();
    asm volatile("" : "+v"(ln));  // per-tile addresses (no loop-invariant hoisting)
    const int64_t m0 = tile * TM;
    const int64_t B = ((int64_t)iO[1] << 32) | iO[0];
    const int64_t mlast = ((m0 + TM < M) ? m0 + TM : M) - m0;
    const int64_t E = ((int64_t)iO[2 * mlast + 1] << 32) | iO[2 * mlast];
    const int64_t Bs = B & ~3ll, Bp = B & ~1ll;
    const int64_t es = (E < Nf4) ? ((E + 3) & ~3ll) : Nf4;
    const int64_t ep = (E < Nf2) ? ((E + 1) & ~1ll) : Nf2;
    (void)es;
    (void)ep;
    const int64_t mk = m0 + ln;
    const bool has = mk < M;
    int64_t off = B;
    int n = 0;
    if (has) {
      off = ((int64_t)iO[2 * ln + 1] << 32) | iO[2 * ln];
      n = (int)((((int64_t)iO[2 * ln + 3] << 32) | iO[2 * ln + 2]) - off);
    }
    if (ballot(n < 0 || n > G)) {  // longer than the launch's max_len: report, skip
      raise_fault(a.fault, kFaultTooLong);
      if (n < 0 || n > G) n = 0;
    }
    const int rs = (int)(off - B);
    const int rsi = rs + (int)(B - Bs);
    const int rsp = rs + (int)(B - Bp);

    // ---- keys + sort ---------------------------------------------------------------------
    unsigned key[G];
    if (ballot(has && (rsi & 3) != 0) == 0) {
#pragma unroll
      for (int c = 0; c < G / 4; ++c) {
        const uint4 v = *reinterpret_cast<const uint4*>(iS + rsi + 4 * c);
        key[4 * c] = v.x; key[4 * c + 1] = v.y; key[4 * c + 2] = v.z; key[4 * c + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < G; ++t) key[t] = iS[rsi + t];
    }
#pragma unroll
    for (int t = 0; t < G; ++t) key[t] = (t < n) ? ((key[t] << LOGG) | (unsigned)t) : kSent32;
    oem_sort<G>(key);
    // run boundaries: bit t of nq = (sid_t != sid_t+1); sentinels sort last and never
    // equal a sid, so lst = nq | top bit, fst = nq << 1 | 1, both masked to t < n
    unsigned nq = 0;
#pragma unroll
    for (int t = G - 2; t >= 0; --t) nq = (nq << 1) | (((key[t] ^ key[t + 1]) >> LOGG) != 0u ? 1u : 0u);
    unsigned vb = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
    unsigned lb = (nq | (1u << (G - 1))) & vb;
    unsigned fb = ((nq << 1) | 1u) & vb;
    asm volatile("" : "+v"(fb), "+v"(lb), "+v"(vb));
    wave_sync_lds();  // every lane has its sids: rows become usid staging

    double2 ring[NG];
#pragma unroll
    for (int t = 0; t < NG; ++t) {
      const unsigned ix = min(key[t] >> LOGG, smax);
      ring[t] = tab[ix];
    }
    double pq[PA];
#pragma unroll
    for (int t = 0; t < PA; ++t) pq[t] = iP[rsp + (int)(key[t] & (G - 1))];

    // ---- walk (core.py:107-144 in sorted-source order) ----------------------------------
    double total = 0.0, ws = 0.0, cs = 0.0, psum = 0.0;
    int cnt = 0, j = 0;
    // single positions: valid, first AND last of their run -- on random ids ~97 % of all
    // positions, and at ~83 % of positions every lane of the wave is single
    unsigned sb = fb & lb & vb;
    asm volatile("" : "+v"(sb));
    // unique j is staged at row cell (j + lane) mod n: rows of equal length sit at a
    // stride of n dwords, so cell j alone would put every lane on one bank (32-way);
    // rotating by the lane spreads them (cells < n only: neighbours' rows untouched)
    const int rotn = (n > 0) ? ln % n : 0;
    auto rot = [&](int jj) { const int x = jj + rotn; return (x >= n) ? x - n : x; };
#pragma unroll
    for (int t = 0; t < G; ++t) {
      const unsigned sid = key[t] >> LOGG;
      const int slot = (int)(key[t] & (G - 1));
      const double p = pq[t % PA];
      if (t + PA < G) pq[t % PA] = iP[rsp + (int)(key[t + PA < G ? t + PA : t] & (G - 1))];
      const double2 rc = ring[t % NG];
      if (t + NG < G) {
        const unsigned ix = min(key[t + NG < G ? t + NG : t] >> LOGG, smax);
        ring[t % NG] = tab[ix];
      }
      const double wt = rc.x, cf = rc.y;
      const bool kv = __builtin_amdgcn_ubfe(vb, t, 1) != 0u;
      if (ballot(__builtin_amdgcn_ubfe(sb, t, 1) == 0u) == 0) {
        // every lane: a source seen once (avg = 0 + p) -- plain left-to-right adds
        total += wt;                      // core.py:120
        ws += p * wt;                     // core.py:135-137 (0 + p == p bit for bit,
        cs += cf * wt;                    //   except -0.0 -> +0.0, which * w changes nothing)
        iS[rsi + rot(j)] = sid | ((unsigned)slot << kPackSlot);
        iP[rsp + slot] = wt;
        j += 1;
      } else {
        const bool fst = __builtin_amdgcn_ubfe(fb, t, 1) != 0u;
        const bool lst = __builtin_amdgcn_ubfe(lb, t, 1) != 0u;
        psum = (fst ? 0.0 : psum) + p;   // builtin sum() from int 0 (core.py:116)
        cnt = fst ? 1 : cnt + 1;
        double avg = psum;
        if (ballot(lst && cnt > 1)) {     // duplicates: sum / len (core.py:116), rare
          if (lst && cnt > 1) avg = psum / (double)cnt;
        }
        // accumulate only at the last position of a run; +0.0 leaves every chain
        // bit-exact (the chains start at +0.0 and can never become -0.0)
        total += lst ? wt : 0.0;          // core.py:120
        ws += lst ? avg * wt : 0.0;       // core.py:135-137
        cs += lst ? cf * wt : 0.0;        // core.py:141-143
        if (kv) {  // j <= t: the row cell is dead; the slot's probability has been read
          iS[rsi + rot(j)] = sid | ((unsigned)slot << kPackSlot);
          iP[rsp + slot] = wt;
        }
        j += lst ? 1 : 0;
      }
      asm volatile("" : "+v"(total), "+v"(ws), "+v"(cs), "+v"(psum), "+v"(cnt), "+v"(j));
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- per-market results --------------------------------------------------------------
    if (has) {
      const bool null_ = (total == 0.0);  // core.py:131-133
      a.consensus[mk] = null_ ? 0.0 : ws / total;
      a.confidence[mk] = null_ ? 0.0 : cs / total;
      a.total_weight[mk] = total;
      a.n_unique[mk] = j;
      if (a.err_idx) {  // first bad input index (the loader's range-check bits)
        const int w0 = rs >> 5, sh = rs & 31;
        const uint32_t lo = sBad[s][w0], hi = sBad[s][w0 + 1];
        const uint32_t bits = ((sh ? (hi << (32 - sh)) : 0u) | (lo >> sh)) & vb;
        a.err_idx[mk] = bits ? (int)__builtin_ctz(bits) : -1;
      }
    }
    {
      const uint2 tb = *reinterpret_cast<const uint2*>(&total);
      sInfo[cw][ln] = make_uint4((unsigned)rs, (unsigned)(has ? j : 0) | ((unsigned)((n > 0) ? n : 1) << 8) |
                                                   ((unsigned)rotn << 16), tb.x, tb.y);
    }
    wave_sync_lds();

    // ---- per-unique outputs from the in-place staging ------------------------------------
    // lane = (market q, slot pair k2), batches of CB iterations: the three dependent LDS
    // round trips (info -> packed usid -> weight cell / present bit) are issued for the
    // whole batch before any result is used, and no load sits under a branch.
    {
      const int dB = (int)(B - Bs), dP = (int)(B - Bp);
      auto copy_out = [&](auto npl) {
        constexpr int NPL = decltype(npl)::value;  // 2: slot pairs (16-B stores), 1: single slots
        constexpr int LPM = G / NPL;               // lanes per market
        constexpr int MPX = kWave / LPM;           // markets per iteration
        constexpr int NIT = TM / MPX;
        constexpr int CB = (NIT < 4) ? NIT : 4;
        const int k2 = NPL * (ln % LPM), g = ln / LPM;
#pragma unroll 1
        for (int i0 = 0; i0 < NIT; i0 += CB) {
          uint4 inf[CB];
#pragma unroll
          for (int b = 0; b < CB; ++b) inf[b] = sInfo[cw][(i0 + b) * MPX + g];
          int r[CB], c0[CB], c1[CB];
          bool v0[CB], v1[CB];
#pragma unroll
          for (int b = 0; b < CB; ++b) {
            r[b] = (int)inf[b].x;
            const int u = (int)(inf[b].y & 255u), nq = (int)((inf[b].y >> 8) & 255u), rq = (int)(inf[b].y >> 16);
            v0[b] = k2 < u;
            v1[b] = NPL == 2 && k2 + 1 < u;
            int x0 = k2 + rq;
            x0 -= (x0 >= nq) ? nq : 0;
            int x1 = x0 + 1;
            x1 -= (x1 >= nq) ? nq : 0;
            c0[b] = v0[b] ? x0 : 0;
            c1[b] = v1[b] ? x1 : 0;
          }
          unsigned pk0[CB], pk1[CB];
#pragma unroll
          for (int b = 0; b < CB; ++b) {
            pk0[b] = iS[dB + r[b] + c0[b]];
            pk1[b] = (NPL == 2) ? iS[dB + r[b] + c1[b]] : 0u;
          }
          double w0[CB], w1[CB];
          unsigned u0[CB], u1[CB], bw0[CB], bw1[CB];
#pragma unroll
          for (int b = 0; b < CB; ++b) {
            u0[b] = pk0[b] & ((1u << kPackSlot) - 1);
            u1[b] = pk1[b] & ((1u << kPackSlot) - 1);
            w0[b] = iP[dP + r[b] + (int)((pk0[b] >> kPackSlot) & (G - 1))];
            w1[b] = (NPL == 2) ? iP[dP + r[b] + (int)((pk1[b] >> kPackSlot) & (G - 1))] : 0.0;
            const unsigned i0 = min(u0[b], smax) >> 5, i1 = min(u1[b], smax) >> 5;
            bw0[b] = bits_in_lds ? sBits[i0] : a.pbits[i0];
            bw1[b] = (NPL == 2) ? (bits_in_lds ? sBits[i1] : a.pbits[i1]) : 0u;
          }
          // materialise the batch here: left alone, loads used only under the store
          // branches are sunk into them and serialise again
#pragma unroll
          for (int b = 0; b < CB; ++b) asm volatile("" : "+v"(w0[b]), "+v"(w1[b]), "+v"(bw0[b]), "+v"(bw1[b]));
#pragma unroll
          for (int b = 0; b < CB; ++b) {
            const double tot = __hiloint2double((int)inf[b].w, (int)inf[b].z);
            const unsigned x0 = u0[b] | ((((bw0[b] >> (min(u0[b], smax) & 31)) & 1u) != 0u) ? 0u : 0x80000000u);
            const unsigned x1 = u1[b] | ((((bw1[b] >> (min(u1[b], smax) & 31)) & 1u) != 0u) ? 0u : 0x80000000u);
            const double n0 = (tot > 0.0) ? w0[b] / tot : 0.0;  // core.py:151
            const double n1 = (tot > 0.0) ? w1[b] / tot : 0.0;  // (cold bit: core.py:167-170)
            const int64_t pos = B + r[b] + k2;
            if (v1[b]) {
              *reinterpret_cast<uint2*>(a.usid + pos) = make_uint2(x0, x1);
              *reinterpret_cast<double2*>(a.weight + pos) = make_double2(w0[b], w1[b]);
              *reinterpret_cast<double2*>(a.nweight + pos) = make_double2(n0, n1);
            } else if (v0[b]) {
              a.usid[pos] = (int32_t)x0;
              a.weight[pos] = w0[b];
              a.nweight[pos] = n0;
            }
          }
        }
      };
      const bool vec_ok = (((uintptr_t)a.usid & 7) | ((uintptr_t)a.weight & 15) | ((uintptr_t)a.nweight & 15)) == 0;
      if (vec_ok && ballot(has && (off & 1) != 0) == 0 && (B & 1) == 0)
        copy_out(std::integral_constant<int, 2>{});
      else
        copy_out(std::integral_constant<int, 1>{});
    }
    wave_sync_lds();  // every read of the slot has returned
    __hip_atomic_store(&sFree[s], seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// ------------------------------------------------------------------------------------
// long markets: workgroup per market
// ------------------------------------------------------------------------------------
constexpr int kLongThreads = 256;
constexpr int kLongMaxLds = 4096;

// Fixed-order (deterministic) tree sum over the workgroup (BCE_MODE_FAST).
__device__ __forceinline__ double block_sum_tree(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = kLongThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] = red[tid] + red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// Pass structure per market (all arrays length P = next pow2 >= n):
//   0  keys[t] = sid<<32 | t, Pr[t] = prob (input order); first out-of-range index
//   1  bitonic sort of keys (ascending sid, then input index == core.py:103,115)
//   2  leaders (first position of each sid run) sum their run's probabilities in input
//      order (core.py:116), compact index j by block scan -> Av[j] = avg, Sj[j] = sid
//   3  per unique j: w = rel, W[j] = w, A[j] = avg*w, C[j] = conf*w, per-unique outputs
//   4  ordered sums over j (exact: one lane per chain; fast: fixed tree)
//   5  normalizedWeight[j] = W[j] / total
template <bool IN_LDS>
__global__ __launch_bounds__(kLongThreads) void consensus_long_kernel(ConsArgs a) {
  constexpr int NT = kLongThreads;
  constexpr int NW = NT / kWave;
  constexpr int CAP = IN_LDS ? kLongMaxLds : 1;
  __shared__ unsigned long long lKeys[CAP];  // keys, then W (double)
  __shared__ double lP[CAP];                 // probabilities, then A
  __shared__ double lC[CAP];                 // avg, then C
  __shared__ int32_t lS[CAP];                // sid of unique j
  __shared__ double red[NT];
  __shared__ int32_t sInt[NW + 2];
  __shared__ double sTot[4];

  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wv = tid / kWave;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  for (int64_t li = blockIdx.x; li < a.n_list; li += gridDim.x) {
    const int32_t m = a.list ? a.list[li] : (int32_t)li;
    const int64_t off = a.offsets[m];
    const int32_t n = (int32_t)(a.offsets[m + 1] - off);
    int P = 1;
    while (P < n) P <<= 1;

    unsigned long long* keys;
    double* Pr;
    double* Cv;
    int32_t* Sj;
    if constexpr (IN_LDS) {
      keys = lKeys;
      Pr = lP;
      Cv = lC;
      Sj = lS;
    } else {
      unsigned long long* base = reinterpret_cast<unsigned long long*>(a.scratch) +
                                 (int64_t)blockIdx.x * 4 * a.scratch_stride;
      keys = base;
      Pr = reinterpret_cast<double*>(base + a.scratch_stride);
      Cv = reinterpret_cast<double*>(base + 2 * a.scratch_stride);
      Sj = reinterpret_cast<int32_t*>(base + 3 * a.scratch_stride);
    }
    double* Wv = reinterpret_cast<double*>(keys);

    // ---- pass 0 ------------------------------------------------------------------------
    if (tid == 0) sInt[0] = 0x7fffffff;
    __syncthreads();
    int myerr = 0x7fffffff;
    for (int i = tid; i < P; i += NT) {
      if (i < n) {
        const double p = a.prob[off + i];
        keys[i] = ((unsigned long long)(unsigned)a.sid[off + i] << 32) | (unsigned)i;
        Pr[i] = p;
        if ((p < 0.0 || p > 1.0) && i < myerr) myerr = i;  // core.py:59-60
      } else {
        keys[i] = kSent64;
      }
    }
    if (myerr != 0x7fffffff) atomicMin(&sInt[0], myerr);
    __syncthreads();
    const int errv = sInt[0];

    // ---- pass 1: bitonic sort ----------------------------------------------------------
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int c = tid; c < (P >> 1); c += NT) {
          const int lo = ((c & ~(j - 1)) << 1) | (c & (j - 1));
          const int hi = lo | j;
          const bool up = (lo & k) == 0;
          const unsigned long long x = keys[lo], y = keys[hi];
          if ((x > y) == up) {
            keys[lo] = y;
            keys[hi] = x;
          }
        }
        __syncthreads();
      }
    }

    // ---- pass 2: leaders, run sums in input order, compact index ------------------------
    int u = 0;
    for (int c0 = 0; c0 < n; c0 += NT) {
      const int tpos = c0 + tid;
      bool first = false;
      int ssid = 0;
      double avg = 0.0;
      if (tpos < n) {
        ssid = (int)(keys[tpos] >> 32);
        first = (tpos == 0) || ((int)(keys[tpos - 1] >> 32) != ssid);
        if (first) {
          double s = 0.0;  // builtin sum() from 0 (core.py:116)
          int cnt = 0;
          for (int q = tpos; q < n; ++q) {
            const unsigned long long kq = keys[q];
            if ((int)(kq >> 32) != ssid) break;
            s += Pr[(int)(kq & 0xffffffffu)];
            ++cnt;
          }
          avg = (cnt > 1) ? s / (double)cnt : s;
        }
      }
      const unsigned long long bm = ballot(first);
      if (lane == 0) sInt[2 + wv] = __popcll(bm);
      __syncthreads();
      int before = u, chunk = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int cq = sInt[2 + q];
        if (q < wv) before += cq;
        chunk += cq;
      }
      if (first) {
        const int j = before + __popcll(bm & below);
        Cv[j] = avg;
        Sj[j] = ssid;
      }
      u += chunk;
      __syncthreads();
    }

    // ---- pass 3: gather + per-unique products (keys/probs are dead now) -----------------
    for (int j = tid; j < u; j += NT) {
      const int s = Sj[j];
      const double2 rc = a.relconf[s];
      const double w = rc.x;  // core.py:111,119
      const double c = rc.y;  // core.py:112
      const double avg = Cv[j];
      Wv[j] = w;
      Pr[j] = avg * w;  // core.py:136
      Cv[j] = c * w;    // core.py:142
      const int64_t p = off + j;
      if (a.usid) a.usid[p] = s | (is_present(a.pbits, s) ? 0 : (int32_t)0x80000000);
      if (a.weight) a.weight[p] = w;
    }
    __syncthreads();

    // ---- pass 4: ordered sums ----------------------------------------------------------
    if (a.mode == BCE_MODE_EXACT) {
      if (tid < 3) {  // three independent chains on three lanes of wave 0
        const double* arr = (tid == 0) ? Wv : (tid == 1) ? Pr : Cv;
        double acc = 0.0;
        for (int j = 0; j < u; ++j) acc += arr[j];
        sTot[tid] = acc;
      }
      __syncthreads();
    } else {
      double pw = 0.0, pa = 0.0, pc = 0.0;
      for (int j = tid; j < u; j += NT) {
        pw += Wv[j];
        pa += Pr[j];
        pc += Cv[j];
      }
      const double tw = block_sum_tree(pw, red);
      const double ta = block_sum_tree(pa, red);
      const double tc = block_sum_tree(pc, red);
      if (tid == 0) {
        sTot[0] = tw;
        sTot[1] = ta;
        sTot[2] = tc;
      }
      __syncthreads();
    }
    const double total = sTot[0];
    if (tid == 0) {
      const bool null_ = (n == 0) || (total == 0.0);
      a.consensus[m] = null_ ? 0.0 : sTot[1] / total;
      a.confidence[m] = null_ ? 0.0 : sTot[2] / total;
      a.total_weight[m] = total;
      a.n_unique[m] = u;
      if (a.err_idx) a.err_idx[m] = (errv == 0x7fffffff) ? -1 : errv;
    }

    // ---- pass 5: normalizedWeight (core.py:151) ----------------------------------------
    if (a.nweight) {
      for (int j = tid; j < u; j += NT) a.nweight[off + j] = (total > 0.0) ? Wv[j] / total : 0.0;
    }
    __syncthreads();
  }
}


}  // namespace bce

// ======================================================================================
// host launchers
// ======================================================================================
namespace bce {
namespace {

template <int G, int TM>
int launch_seg(const ConsArgs& a, hipStream_t st) {
  const int64_t tiles = (a.n_list + TM - 1) / TM;
  if (tiles == 0) return BCE_OK;
  // persistent grid: every workgroup resident at once, tiles dealt round-robin
  const int per_cu = blocks_per_cu(reinterpret_cast<const void*>(&consensus_seg_kernel<G, TM>), 64, 0, 8);
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(tiles < cap ? tiles : cap);
  hipLaunchKernelGGL((consensus_seg_kernel<G, TM>), dim3(grid), dim3(64), 0, st, a);
  return check_launch("consensus_seg_kernel");
}

template <int G>
int launch_lpm(const ConsArgs& a, hipStream_t st) {
  const int64_t tiles = (a.n_list + kWave - 1) / kWave;
  if (tiles == 0) return BCE_OK;
  const int per_cu = blocks_per_cu(reinterpret_cast<const void*>(&consensus_lpm_kernel<G>), 64, 0, 4);
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(tiles < cap ? tiles : cap);
  hipLaunchKernelGGL((consensus_lpm_kernel<G>), dim3(grid), dim3(64), 0, st, a);
  return check_launch("consensus_lpm_kernel");
}

template <int G>
int launch_pipe(const ConsArgs& a, hipStream_t st) {
  constexpr int TM = 64;
  const int64_t tiles = (a.n_list + TM - 1) / TM;
  if (tiles == 0) return BCE_OK;
  const int per_cu = blocks_per_cu(reinterpret_cast<const void*>(&consensus_pipe_kernel<G>),
                                   64 * (PipeCfg<G>::C + PipeCfg<G>::L), 0, 1, "consensus_pipe_kernel");
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(tiles < cap ? tiles : cap);
  hipLaunchKernelGGL((consensus_pipe_kernel<G>), dim3(grid), dim3(64 * (PipeCfg<G>::C + PipeCfg<G>::L)), 0, st,
                     a);
  return check_launch("consensus_pipe_kernel");
}

template <int G>
int launch_flat(const ConsArgs& a, hipStream_t st) {
  constexpr int TM = kFlatTM, WPB = kFlatWPB;
  const int64_t tiles = (a.n_list + TM - 1) / TM;
  if (tiles == 0) return BCE_OK;
  const int per_cu = blocks_per_cu(reinterpret_cast<const void*>(&consensus_flat_kernel<G, TM, WPB>), 64 * WPB, 0, 2,
                                   "consensus_flat_kernel");
  const int64_t blocks = (tiles + WPB - 1) / WPB;
  const int64_t cap = (int64_t)cu_count() * per_cu;
  const int grid = (int)(blocks < cap ? blocks : cap);
  hipLaunchKernelGGL((consensus_flat_kernel<G, TM, WPB>), dim3(grid), dim3(64 * WPB), 0, st, a);
  return check_launch("consensus_flat_kernel");
}

// Markets with n <= 64 (a.list == NULL: contiguous CSR; else a planned market list).
//   contiguous, 16 < n <= 32, S <= kTabMaxSources   consensus_tab32_kernel (table in LDS)
//   ... S <= kTabHybMaxSources                       consensus_tab32_kernel<hybrid> (LDS rows + global rest)
//   contiguous, n <= 32, S < 2^25, all outputs       consensus_pipe_kernel<G> (loader + compute waves)
//   contiguous, n <= 32, otherwise                   consensus_flat_kernel<G>
//   market list, n <= 32                             consensus_lpm_kernel<G> (lane per market)
//   33 <= n <= 64                                    consensus_seg_kernel<64, 8>
int launch_seg_for_len(int max_len, const ConsArgs& a, hipStream_t st) {
  if (a.list == nullptr && max_len <= 32) {
    if (max_len > 16 && a.n_sources <= kTabHybMaxSources) return launch_tab32(a, st);
    if (a.n_sources < (1 << 25) && a.n_signals >= 4 && a.usid && a.weight && a.nweight) {
      if (max_len <= 8) return launch_pipe<8>(a, st);
      if (max_len <= 16) return launch_pipe<16>(a, st);
      return launch_pipe<32>(a, st);
    }
    if (max_len <= 8) return launch_flat<8>(a, st);
    if (max_len <= 16) return launch_flat<16>(a, st);
    return launch_flat<32>(a, st);
  }
  if (max_len <= 8) return launch_lpm<8>(a, st);
  if (max_len <= 16) return launch_lpm<16>(a, st);
  if (max_len <= 32) return launch_lpm<32>(a, st);
  return launch_seg<64, 8>(a, st);
}

int launch_long_lds(const ConsArgs& a, hipStream_t st) {
  if (a.n_list == 0) return BCE_OK;
  const int64_t cap = (int64_t)cu_count() * 2;
  const int grid = (int)(a.n_list < cap ? a.n_list : cap);
  hipLaunchKernelGGL((consensus_long_kernel<true>), dim3(grid), dim3(kLongThreads), 0, st, a);
  return check_launch("consensus_long_kernel<lds>");
}

// Markets with 64 < n <= 4096: the register-sort kernel (consensus_wide.hip), with packed
// 32-bit (sid, index) keys when they fit and 64-bit keys for larger tables.
int launch_wide_for_len(int64_t max_len, const ConsArgs& a, hipStream_t st) {
  return launch_wide_len(max_len, a, st);
}

constexpr int kHugeGrid = 512;

int64_t next_pow2(int64_t n) {
  int64_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

int launch_long_global(ConsArgs a, int64_t max_len, void* scratch, int64_t scratch_bytes,
                       hipStream_t st) {
  if (a.n_list == 0) return BCE_OK;
  const int grid = (int)(a.n_list < kHugeGrid ? a.n_list : kHugeGrid);
  const int64_t P = next_pow2(max_len);
  const int64_t need = (int64_t)grid * 4 * P * 8;
  BCE_REQUIRE(scratch && scratch_bytes >= need, "consensus: scratch too small (%lld < %lld)",
              (long long)scratch_bytes, (long long)need);
  a.scratch = scratch;
  a.scratch_stride = P;
  hipLaunchKernelGGL((consensus_long_kernel<false>), dim3(grid), dim3(kLongThreads), 0, st, a);
  return check_launch("consensus_long_kernel<global>");
}

__global__ void max_len_kernel(const int64_t* offsets, int64_t n, const int32_t* list, int64_t n_list,
                               unsigned long long* out) {
  int64_t best = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_list;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = list ? list[i] : i;
    const int64_t len = offsets[m + 1] - offsets[m];
    best = len > best ? len : best;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t x = __shfl_xor(best, o);
    best = x > best ? x : best;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)best);
}

int check_common(const int64_t* offsets, int64_t n_markets, const int32_t* sid, const double* prob,
                 const double* relconf, const uint32_t* present_bits, int32_t n_sources,
                 double* consensus, double* confidence, double* total_weight, int32_t* n_unique) {
  BCE_REQUIRE(n_markets >= 0, "consensus: n_markets < 0");
  BCE_REQUIRE(n_markets == 0 || offsets, "consensus: offsets is NULL");
  BCE_REQUIRE(n_markets == 0 || (consensus && confidence && total_weight && n_unique),
              "consensus: per-market outputs must be non-NULL");
  BCE_REQUIRE(n_sources >= 0 && (n_sources == 0 || (relconf && present_bits)),
              "consensus: source table is NULL");
  BCE_REQUIRE((uintptr_t)relconf % 16 == 0, "consensus: relconf must be 16-byte aligned");
  (void)sid;
  (void)prob;
  return BCE_OK;
}

}  // namespace
}  // namespace bce

using namespace bce;

extern "C" int bce_consensus_csr(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                                 const double* prob, int64_t n_signals, const double* relconf,
                                 const uint32_t* present_bits, int32_t n_sources,
                                 const int32_t* market_list, int64_t n_list, int32_t max_len,
                                 int32_t mode, double* consensus, double* confidence,
                                 double* total_weight, int32_t* n_unique, int32_t* err_idx,
                                 int32_t* usid, double* weight, double* nweight, void* stream) {
  int rc = check_common(offsets, n_markets, sid, prob, relconf, present_bits, n_sources, consensus,
                        confidence, total_weight, n_unique);
  if (rc) return rc;
  BCE_REQUIRE(mode == BCE_MODE_EXACT || mode == BCE_MODE_FAST, "consensus: bad mode %d", mode);
  BCE_REQUIRE(n_signals == 0 || (sid && prob), "consensus: sid/prob NULL");
  hipStream_t st = as_stream(stream);
  ConsArgs a{};
  a.offsets = offsets; a.sid = sid; a.prob = prob;
  a.relconf = reinterpret_cast<const double2*>(relconf); a.pbits = present_bits;
  a.n_sources = n_sources; a.n_signals = n_signals;
  a.list = market_list; a.n_list = market_list ? n_list : n_markets;
  a.consensus = consensus; a.confidence = confidence; a.total_weight = total_weight;
  a.n_unique = n_unique; a.err_idx = err_idx; a.usid = usid; a.weight = weight; a.nweight = nweight;
  a.mode = mode;
  a.fault = fault_word();
  a.spin_cap = spin_cap();
  if (a.n_list == 0) return BCE_OK;
  int64_t L = max_len;
  if (L <= 0) {  // unknown: measure on device (synchronises)
    unsigned long long* d = nullptr;
    BCE_HIP(hipMallocAsync((void**)&d, sizeof(unsigned long long), st));
    BCE_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(max_len_kernel, dim3(256), dim3(256), 0, st, offsets, n_markets, market_list,
                       a.n_list, d);
    unsigned long long h = 0;
    BCE_HIP(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st));
    BCE_HIP(hipFreeAsync(d, st));
    BCE_HIP(hipStreamSynchronize(st));
    L = (int64_t)h;
  }
  // the 32-bit (sid, index) key of the segment kernel needs sid < 2^(31 - log2 G)
  if (L <= 64 && n_sources <= (1 << 25)) return launch_seg_for_len((int)(L < 1 ? 1 : L), a, st);
  if (L <= kLongMaxLds) return launch_wide_for_len(L, a, st);
  const int grid = (int)(a.n_list < kHugeGrid ? a.n_list : kHugeGrid);
  const int64_t bytes = (int64_t)grid * 4 * next_pow2(L) * 8;
  void* scratch = nullptr;
  BCE_HIP(hipMallocAsync(&scratch, (size_t)bytes, st));
  rc = launch_long_global(a, L, scratch, bytes, st);
  BCE_HIP(hipFreeAsync(scratch, st));
  return rc;
}

static_assert(BCE_NBINS == 13, "bin table");
static constexpr int64_t kBinMax[BCE_NBINS - 1] = {8, 16, 32, 64, 128, 256, 512, 1024, 1536, 2048, 3072, kLongMaxLds};
constexpr int kBinNp2Lo = 8, kBinNp2Hi = 10;  // the 1536 and 3072 bins
static_assert(kBinMax[kBinNp2Lo] == 1536 && kBinMax[kBinNp2Hi] == 3072, "non-power-of-two bins");
constexpr int kPlanSideLast = 3;  // bins 0..3 (n <= 64) run on the side stream
constexpr double kMergeRounds = 6.0;  // merge a small call's bins below this many resident rounds
static int bin_of(int64_t n) {
  for (int b = 0; b < BCE_NBINS - 1; ++b)
    if (n <= kBinMax[b]) return b;
  return BCE_NBINS - 1;
}

extern "C" int bce_plan_bins(const int64_t* offsets_host, int64_t n_markets, int32_t* order_host,
                             int64_t* bin_start_host, int32_t* max_len_host) {
  BCE_REQUIRE(n_markets >= 0 && offsets_host && order_host && bin_start_host,
              "plan_bins: NULL argument");
  int64_t cnt[BCE_NBINS] = {0};
  int64_t mx = 0;
  for (int64_t m = 0; m < n_markets; ++m) {
    const int64_t n = offsets_host[m + 1] - offsets_host[m];
    BCE_REQUIRE(n >= 0, "plan_bins: offsets not monotone at market %lld", (long long)m);
    cnt[bin_of(n)]++;
    mx = n > mx ? n : mx;
  }
  bin_start_host[0] = 0;
  for (int b = 0; b < BCE_NBINS; ++b) bin_start_host[b + 1] = bin_start_host[b] + cnt[b];
  int64_t pos[BCE_NBINS];
  for (int b = 0; b < BCE_NBINS; ++b) pos[b] = bin_start_host[b];
  for (int64_t m = 0; m < n_markets; ++m) {
    const int64_t n = offsets_host[m + 1] - offsets_host[m];
    order_host[pos[bin_of(n)]++] = (int32_t)m;
  }
  // Wide bins (65..4096) longest market first (LPT order, ties by market index): a
  // persistent workgroup takes its next market as it finishes one, so the last round of
  // workgroups gets the short ones and the launch's tail shrinks (C3 fast -0.7%, exact
  // -0.6%, one of 8 market shards -1.3%: profiles/r03ae/).
  for (int b = kPlanSideLast + 1; b < BCE_NBINS - 1; ++b)
    std::stable_sort(order_host + bin_start_host[b], order_host + bin_start_host[b + 1], [&](int32_t x, int32_t y) {
      return offsets_host[x + 1] - offsets_host[x] > offsets_host[y + 1] - offsets_host[y];
    });
  if (max_len_host) *max_len_host = (int32_t)(mx > 0x7fffffff ? 0x7fffffff : mx);
  return BCE_OK;
}

extern "C" int64_t bce_consensus_scratch_bytes(const int64_t* offsets_host, const int32_t* order_host,
                                               const int64_t* bin_start_host) {
  const int64_t b0 = bin_start_host[BCE_NBINS - 1], b1 = bin_start_host[BCE_NBINS];
  if (b1 <= b0) return 0;
  int64_t mx = 0;
  for (int64_t i = b0; i < b1; ++i) {
    const int32_t m = order_host[i];
    const int64_t n = offsets_host[m + 1] - offsets_host[m];
    mx = n > mx ? n : mx;
  }
  const int64_t cnt = b1 - b0;
  const int grid = (int)(cnt < kHugeGrid ? cnt : kHugeGrid);
  return (int64_t)grid * 4 * next_pow2(mx) * 8;
}

// ======================================================================================
// The device planner (bce_plan_bins_device): the plan of bce_plan_bins built from device
// offsets, no D2H copy of the CSR.  A market's bin and its LPT position are one 12-bit key
//   bins 0..3 (n <= 64)           key = bin                (market order inside the bin)
//   wide bin b, lengths lo..hi    key = 4 + (lo - 65) + (hi - n)   (bins ascending, longest first)
//   n > 4096                      key = kPlanKeys - 1
// so the plan is a STABLE sort of the market indices by key: two LSD passes of 6-bit digits,
// each a per-chunk digit count, one exclusive scan of the [digit][chunk] counts and a stable
// scatter (the rank inside a chunk from a [thread][digit] count matrix in LDS).  Stable at
// every pass, hence market order inside equal keys: exactly bce_plan_bins' order.
// ======================================================================================
namespace bce {
constexpr int kPlanKeys = 4 + (4096 - 65 + 1) + 1;  // 4037 < 2^12
constexpr int kPlanThreads = 256;
constexpr int kPlanPer = 4;                          // markets per thread
constexpr int kPlanChunk = kPlanThreads * kPlanPer;  // markets per workgroup
constexpr int kPlanDigits = 64;                      // 6-bit digits, two passes
constexpr int kPlanScanThreads = 1024;
static_assert(kPlanKeys <= kPlanDigits * kPlanDigits, "two 6-bit passes");

struct PlanInfo {
  unsigned long long bins[BCE_NBINS];
  unsigned long long max_len;
  unsigned long long long_max;  // longest market of the > 4096 bin (scratch sizing)
  unsigned long long badrev;    // M - (first market whose offsets decrease), 0 = none
};

__device__ __forceinline__ int plan_bin(int64_t n) {
  return n <= 8 ? 0 : n <= 16 ? 1 : n <= 32 ? 2 : n <= 64 ? 3 : n <= 128 ? 4 : n <= 256 ? 5 : n <= 512 ? 6
       : n <= 1024 ? 7 : n <= 1536 ? 8 : n <= 2048 ? 9 : n <= 3072 ? 10 : n <= 4096 ? 11 : 12;
}

__device__ __forceinline__ int plan_key(int64_t n, int b) {
  if (b <= 3) return b;
  if (b == 12) return kPlanKeys - 1;
  const int lo = b == 4 ? 65 : b == 5 ? 129 : b == 6 ? 257 : b == 7 ? 513 : b == 8 ? 1025 : b == 9 ? 1537
               : b == 10 ? 2049 : 3073;
  const int hi = b == 4 ? 128 : b == 5 ? 256 : b == 6 ? 512 : b == 7 ? 1024 : b == 8 ? 1536 : b == 9 ? 2048
               : b == 10 ? 3072 : 4096;
  return 4 + (lo - 65) + (hi - (int)n);
}

template <typename T>
__device__ __forceinline__ T wave_max_u64(T v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const T o = (T)__shfl_xor((unsigned long long)v, m);
    v = o > v ? o : v;
  }
  return v;
}

// Pass PASS digit counts of chunk blockIdx.x -> counts[digit * nchunks + chunk].  Pass 0 reads
// the offsets (striped: coalesced) and also writes the chunk's record for PlanInfo (bin counts,
// longest market, longest > 4096 market, first decreasing offset) -- no global atomics: the
// pass-0 scan reduces the records (800 same-address atomicMax per call cost ~10 us).
constexpr int kPlanRec = 16;  // int64 per chunk record: bins[13], max_len, long_max, badrev
template <int PASS, bool CM>
__global__ __launch_bounds__(kPlanThreads) void plan_count_kernel(const int64_t* __restrict__ offsets, int64_t M,
                                                                  const uint16_t* __restrict__ keys_in,
                                                                  int32_t* __restrict__ counts, int64_t nchunks,
                                                                  int64_t* __restrict__ crec) {
  __shared__ int cnt[kPlanDigits];
  __shared__ int bincnt[BCE_NBINS];
  __shared__ unsigned long long wmax[kPlanThreads / kWave][3];
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  if (t < kPlanDigits) cnt[t] = 0;
  if (PASS == 0 && t < BCE_NBINS) bincnt[t] = 0;
  __syncthreads();
  unsigned long long mx = 0, lmx = 0, badrev = 0;
#pragma unroll
  for (int k = 0; k < kPlanPer; ++k) {
    const int64_t i = c * kPlanChunk + k * kPlanThreads + t;
    if (i < M) {
      int key;
      if constexpr (PASS == 0) {
        const int64_t n = offsets[i + 1] - offsets[i];
        if (n < 0) badrev = (unsigned long long)(M - i) > badrev ? (unsigned long long)(M - i) : badrev;
        const int b = plan_bin(n);
        key = plan_key(n < 0 ? 0 : n, n < 0 ? 0 : b);
        atomicAdd(&bincnt[n < 0 ? 0 : b], 1);
        const unsigned long long un = n < 0 ? 0ull : (unsigned long long)n;
        mx = un > mx ? un : mx;
        if (b == 12) lmx = un > lmx ? un : lmx;
      } else {
        key = keys_in[i];
      }
      atomicAdd(&cnt[(key >> (6 * PASS)) & (kPlanDigits - 1)], 1);
    }
  }
  if constexpr (PASS == 0) {
    mx = wave_max_u64(mx);
    lmx = wave_max_u64(lmx);
    badrev = wave_max_u64(badrev);
    if (lane_id() == 0) {
      wmax[t / kWave][0] = mx;
      wmax[t / kWave][1] = lmx;
      wmax[t / kWave][2] = badrev;
    }
  }
  __syncthreads();
  if (t < kPlanDigits) counts[CM ? c * kPlanDigits + t : (int64_t)t * nchunks + c] = cnt[t];
  if constexpr (PASS == 0) {
    int64_t* r = crec + c * kPlanRec;
    if (t < BCE_NBINS) r[t] = bincnt[t];
    if (t >= BCE_NBINS && t < BCE_NBINS + 3) {
      unsigned long long v = 0;
      for (int w = 0; w < kPlanThreads / kWave; ++w) v = wmax[w][t - BCE_NBINS] > v ? wmax[w][t - BCE_NBINS] : v;
      r[t] = (int64_t)v;
    }
  }
}

// Reduce the count pass's chunk records into PlanInfo; with bin_start_dev also the device bin
// boundaries and the device-driven faults (decreasing offsets: every bin empty + kFaultOffsets;
// raise_long: a market > 4096 raises kFaultTooLong).  Called by one whole workgroup.
__device__ __forceinline__ void plan_reduce_info(const int64_t* __restrict__ crec, int64_t nchunks, PlanInfo* info,
                                                 int64_t* bin_start_dev, int* fault, int raise_long,
                                                 unsigned long long* sacc, int t, int nthreads) {
  if (t < BCE_NBINS + 3) sacc[t] = 0;
  __syncthreads();
  unsigned long long b[BCE_NBINS] = {}, m0 = 0, m1 = 0, m2 = 0;
  for (int64_t c = t; c < nchunks; c += nthreads) {
    const int64_t* r = crec + c * kPlanRec;
#pragma unroll
    for (int k = 0; k < BCE_NBINS; ++k) b[k] += (unsigned long long)r[k];
    m0 = (unsigned long long)r[BCE_NBINS] > m0 ? (unsigned long long)r[BCE_NBINS] : m0;
    m1 = (unsigned long long)r[BCE_NBINS + 1] > m1 ? (unsigned long long)r[BCE_NBINS + 1] : m1;
    m2 = (unsigned long long)r[BCE_NBINS + 2] > m2 ? (unsigned long long)r[BCE_NBINS + 2] : m2;
  }
  // wave reductions first: one LDS atomic per wave and counter
#pragma unroll
  for (int k = 0; k < BCE_NBINS; ++k) {
    unsigned long long v = b[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += (unsigned long long)__shfl_xor((long long)v, o);
    b[k] = v;
  }
  m0 = wave_max_u64(m0);
  m1 = wave_max_u64(m1);
  m2 = wave_max_u64(m2);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < BCE_NBINS; ++k)
      if (b[k]) atomicAdd(&sacc[k], b[k]);
    if (m0) atomicMax(&sacc[BCE_NBINS], m0);
    if (m1) atomicMax(&sacc[BCE_NBINS + 1], m1);
    if (m2) atomicMax(&sacc[BCE_NBINS + 2], m2);
  }
  __syncthreads();
  if (t == 0) {
    for (int k = 0; k < BCE_NBINS; ++k) info->bins[k] = sacc[k];
    info->max_len = sacc[BCE_NBINS];
    info->long_max = sacc[BCE_NBINS + 1];
    info->badrev = sacc[BCE_NBINS + 2];
    if (bin_start_dev) {
      const bool bad = sacc[BCE_NBINS + 2] != 0;
      int64_t run = 0;
      bin_start_dev[0] = 0;
      for (int k = 0; k < BCE_NBINS; ++k) {
        run += bad ? 0 : (int64_t)sacc[k];
        bin_start_dev[k + 1] = run;
      }
      if (fault && bad) atomicCAS(fault, 0, kFaultOffsets);
      if (fault && !bad && raise_long && sacc[BCE_NBINS - 1]) atomicCAS(fault, 0, kFaultTooLong);
    }
  }
}

// In-place exclusive scan of counts[0..E) by one workgroup (E = 64 x chunks), in tiles of 8
// consecutive counts per thread (the loads of a tile in flight together).  INFO (pass 0): also
// reduces the chunk records into PlanInfo and, with bin_start_dev, writes the device bin
// boundaries (decreasing offsets: every bin empty + kFaultOffsets; raise_long: a market > 4096
// raises kFaultTooLong -- the device-driven launch does not compute those).
template <bool INFO>
__global__ __launch_bounds__(kPlanScanThreads) void plan_scan_kernel(int32_t* __restrict__ counts, int64_t E,
                                                                     const int64_t* __restrict__ crec, int64_t nchunks,
                                                                     PlanInfo* info, int64_t* bin_start_dev, int* fault,
                                                                     int raise_long) {
  constexpr int V = 8;
  constexpr int NW = kPlanScanThreads / kWave;
  __shared__ int64_t wsum[NW];
  __shared__ int64_t tile_total;
  __shared__ unsigned long long sacc[BCE_NBINS + 3];
  const int t = threadIdx.x;
  const int w = t / kWave;
  if constexpr (INFO) plan_reduce_info(crec, nchunks, info, bin_start_dev, fault, raise_long, sacc, t, kPlanScanThreads);
  int64_t carry = 0;
  for (int64_t base = 0; base < E; base += (int64_t)kPlanScanThreads * V) {
    const int64_t i0 = base + (int64_t)t * V;
    int v[V];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      v[k] = (i0 + k < E) ? counts[i0 + k] : 0;
      s += v[k];
    }
    int64_t inc = s;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int64_t o = __shfl_up(inc, d);
      if (lane_id() >= d) inc += o;
    }
    if (lane_id() == kWave - 1) wsum[w] = inc;
    __syncthreads();
    if (t == 0) {
      int64_t run = 0;
      for (int k = 0; k < NW; ++k) {
        const int64_t x = wsum[k];
        wsum[k] = run;
        run += x;
      }
      tile_total = run;
    }
    __syncthreads();
    int64_t run = carry + wsum[w] + inc - s;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (i0 + k < E) counts[i0 + k] = (int32_t)run;
      run += v[k];
    }
    carry += tile_total;
    __syncthreads();  // wsum / tile_total are rewritten by the next tile
  }
}

// Stable scatter of chunk blockIdx.x by its pass-PASS digit.  Thread t holds markets
// 4t..4t+3 of the chunk (blocked: thread order == input order); mat[t][d] counts thread t's
// items of digit d, and its exclusive scan in (d, t) order gives every item its rank among the
// chunk's items of smaller digit or equal digit and earlier position.
// INKB (<= kPlanInkbMax chunks): the counts are chunk-major [chunk][digit] and every workgroup
// derives its own 64 bases from all of them (a wave reads one 256-B chunk row per step), so no
// scan launch sits between the passes; PASS 0 runs one extra workgroup that reduces the chunk
// records (plan_reduce_info) alongside.  Otherwise `base` is the digit-major exclusive scan of plan_scan_kernel.
constexpr int64_t kPlanInkbMax = 1024;
template <int PASS, bool INKB>
__global__ __launch_bounds__(kPlanThreads) void plan_scatter_kernel(const int64_t* __restrict__ offsets, int64_t M,
                                                                    const uint16_t* __restrict__ keys_in,
                                                                    const int32_t* __restrict__ idx_in,
                                                                    const int32_t* __restrict__ base, int64_t nchunks,
                                                                    uint16_t* __restrict__ keys_out,
                                                                    int32_t* __restrict__ idx_out,
                                                                    const int64_t* __restrict__ crec, PlanInfo* info,
                                                                    int64_t* bin_start_dev, int* fault, int raise_long) {
  __shared__ int mat[kPlanThreads * kPlanDigits];  // [t][d], 64 KB
  __shared__ int part[kPlanThreads];
  __shared__ int sTot[kPlanDigits], sPre[kPlanDigits];
  __shared__ unsigned long long sacc[BCE_NBINS + 3];
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  if constexpr (INKB) {
    if (PASS == 0 && c == nchunks) {  // the extra workgroup of pass 0: PlanInfo, in parallel with the scatter
      plan_reduce_info(crec, nchunks, info, bin_start_dev, fault, raise_long, sacc, t, kPlanThreads);
      return;
    }
    if (t < kPlanDigits) {
      sTot[t] = 0;
      sPre[t] = 0;
    }
    __syncthreads();
    const int dd = t & (kPlanDigits - 1), qq = t / kPlanDigits;
    int tot = 0, pre = 0;
#pragma unroll 4
    for (int64_t c2 = qq; c2 < nchunks; c2 += kPlanThreads / kPlanDigits) {
      const int v = base[c2 * kPlanDigits + dd];
      tot += v;
      pre += (c2 < c) ? v : 0;
    }
    atomicAdd(&sTot[dd], tot);
    atomicAdd(&sPre[dd], pre);
    __syncthreads();
    if (t < kWave) {  // exclusive scan of the digit totals (one wave, lane = digit), + this chunk's prefix
      const int v = sTot[t];
      int inc = v;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane_id() >= o) inc += y;
      }
      sPre[t] += inc - v;
    }
  }
#pragma unroll 8
  for (int j = 0; j < kPlanDigits; ++j) mat[j * kPlanThreads + t] = 0;
  int key[kPlanPer], idx[kPlanPer], before[kPlanPer];
  const int64_t i0 = c * kPlanChunk + (int64_t)t * kPlanPer;
#pragma unroll
  for (int k = 0; k < kPlanPer; ++k) {
    const int64_t i = i0 + k;
    key[k] = -1;
    idx[k] = 0;
    if (i < M) {
      if constexpr (PASS == 0) {
        int64_t n = offsets[i + 1] - offsets[i];
        n = n < 0 ? 0 : n;
        key[k] = plan_key(n, plan_bin(n));
        idx[k] = (int)i;
      } else {
        key[k] = keys_in[i];
        idx[k] = idx_in[i];
      }
    }
  }
  __syncthreads();
  int* row = mat + t * kPlanDigits;
#pragma unroll
  for (int k = 0; k < kPlanPer; ++k) {
    if (key[k] >= 0) {
      const int d = (key[k] >> (6 * PASS)) & (kPlanDigits - 1);
      before[k] = row[d];
      row[d] = before[k] + 1;
    }
  }
  __syncthreads();
  // column sums: thread j = (q, d) sums mat[64q .. 64q+63][d] (a wave reads consecutive words)
  const int d = t & (kPlanDigits - 1), q = t / kPlanDigits;
  int s = 0;
#pragma unroll 8
  for (int r = 0; r < kPlanDigits; ++r) s += mat[(q * kPlanDigits + r) * kPlanDigits + d];
  part[d * (kPlanThreads / kPlanDigits) + q] = s;
  __syncthreads();
  if (t < kWave) {  // exclusive scan of part[] (256 values, 4 per lane) by one wave
    int v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[k] = part[4 * t + k]; sum += v[k]; }
    int inc = sum;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(inc, o);
      if (lane_id() >= o) inc += y;
    }
    int run = inc - sum;
#pragma unroll
    for (int k = 0; k < 4; ++k) { part[4 * t + k] = run; run += v[k]; }
  }
  __syncthreads();
  int run = part[d * (kPlanThreads / kPlanDigits) + q];
#pragma unroll 8
  for (int r = 0; r < kPlanDigits; ++r) {
    int* p = &mat[(q * kPlanDigits + r) * kPlanDigits + d];
    const int v = *p;
    *p = run;
    run += v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPlanPer; ++k) {
    if (key[k] >= 0) {
      const int dg = (key[k] >> (6 * PASS)) & (kPlanDigits - 1);
      const int64_t pos = (INKB ? (int64_t)sPre[dg] : (int64_t)base[(int64_t)dg * nchunks + c]) + (row[dg] - mat[dg]) +
                          before[k];
      if constexpr (PASS == 0) keys_out[pos] = (uint16_t)key[k];
      idx_out[pos] = idx[k];
    }
  }
}
}  // namespace bce

static int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }
static int plan_device_launch(const int64_t* offsets, int64_t n_markets, int32_t* order, void* scratch,
                              hipStream_t st, PlanInfo** info_out, int64_t* bin_start_dev, int raise_long);

extern "C" int64_t bce_plan_device_scratch_bytes(int64_t n_markets) {
  if (n_markets <= 0) return 0;
  const int64_t chunks = (n_markets + kPlanChunk - 1) / kPlanChunk;
  return align256(sizeof(PlanInfo)) + align256(2 * n_markets) + align256(4 * n_markets) +
         align256(4 * kPlanDigits * chunks) + align256(8 * kPlanRec * chunks);
}

extern "C" int bce_plan_bins_device(const int64_t* offsets, int64_t n_markets, int32_t* order,
                                    int64_t* bin_start_host, int32_t* max_len_host,
                                    int64_t* long_scratch_bytes_host, void* scratch, int64_t scratch_bytes,
                                    void* stream) {
  BCE_REQUIRE(n_markets >= 0 && n_markets < ((int64_t)1 << 31), "plan_bins_device: bad n_markets %lld",
              (long long)n_markets);
  BCE_REQUIRE(bin_start_host, "plan_bins_device: bin_start_host NULL");
  if (long_scratch_bytes_host) *long_scratch_bytes_host = 0;
  if (max_len_host) *max_len_host = 0;
  for (int b = 0; b <= BCE_NBINS; ++b) bin_start_host[b] = 0;
  if (n_markets == 0) return BCE_OK;
  BCE_REQUIRE(offsets && order && scratch, "plan_bins_device: NULL argument");
  BCE_REQUIRE(scratch_bytes >= bce_plan_device_scratch_bytes(n_markets), "plan_bins_device: scratch too small");
  hipStream_t st = as_stream(stream);
  PlanInfo* info = nullptr;
  int rc = plan_device_launch(offsets, n_markets, order, scratch, st, &info, nullptr, 0);
  if (rc) return rc;
  PlanInfo h{};
  BCE_HIP(hipMemcpyAsync(&h, info, sizeof h, hipMemcpyDeviceToHost, st));
  BCE_HIP(hipStreamSynchronize(st));
  BCE_REQUIRE(h.badrev == 0, "plan_bins: offsets not monotone at market %lld",
              (long long)(n_markets - (int64_t)h.badrev));
  for (int b = 0; b < BCE_NBINS; ++b) bin_start_host[b + 1] = bin_start_host[b] + (int64_t)h.bins[b];
  if (max_len_host) *max_len_host = (int32_t)(h.max_len > 0x7fffffffull ? 0x7fffffff : h.max_len);
  const int64_t n_long = (int64_t)h.bins[BCE_NBINS - 1];
  if (long_scratch_bytes_host && n_long > 0) {
    const int grid = (int)(n_long < kHugeGrid ? n_long : kHugeGrid);
    *long_scratch_bytes_host = (int64_t)grid * 4 * next_pow2((int64_t)h.long_max) * 8;
  }
  return BCE_OK;
}


static int plan_device_launch(const int64_t* offsets, int64_t n_markets, int32_t* order, void* scratch,
                              hipStream_t st, PlanInfo** info_out, int64_t* bin_start_dev, int raise_long) {
  const int64_t chunks = (n_markets + kPlanChunk - 1) / kPlanChunk;
  char* p = static_cast<char*>(scratch);
  PlanInfo* info = reinterpret_cast<PlanInfo*>(p);
  p += align256(sizeof(PlanInfo));
  uint16_t* keys = reinterpret_cast<uint16_t*>(p);
  p += align256(2 * n_markets);
  int32_t* idx = reinterpret_cast<int32_t*>(p);
  p += align256(4 * n_markets);
  int32_t* counts = reinterpret_cast<int32_t*>(p);
  p += align256(4 * kPlanDigits * chunks);
  int64_t* crec = reinterpret_cast<int64_t*>(p);
  const dim3 g((unsigned)chunks), blk(kPlanThreads), sg(1), sblk(kPlanScanThreads);
  int* fw = fault_word();
  if (chunks <= kPlanInkbMax) {  // 4 launches: bases derived inside the scatter kernels
    hipLaunchKernelGGL((plan_count_kernel<0, true>), g, blk, 0, st, offsets, n_markets, nullptr, counts, chunks, crec);
    hipLaunchKernelGGL((plan_scatter_kernel<0, true>), dim3((unsigned)chunks + 1), blk, 0, st, offsets, n_markets,
                       nullptr, nullptr, counts, chunks, keys, idx, crec, info, bin_start_dev, fw, raise_long);
    hipLaunchKernelGGL((plan_count_kernel<1, true>), g, blk, 0, st, offsets, n_markets, keys, counts, chunks, nullptr);
    hipLaunchKernelGGL((plan_scatter_kernel<1, true>), g, blk, 0, st, offsets, n_markets, keys, idx, counts, chunks,
                       nullptr, order, nullptr, nullptr, nullptr, nullptr, 0);
  } else {  // huge batches: one digit-major scan launch per pass
    hipLaunchKernelGGL((plan_count_kernel<0, false>), g, blk, 0, st, offsets, n_markets, nullptr, counts, chunks, crec);
    hipLaunchKernelGGL((plan_scan_kernel<true>), sg, sblk, 0, st, counts, kPlanDigits * chunks, crec, chunks, info,
                       bin_start_dev, fw, raise_long);
    hipLaunchKernelGGL((plan_scatter_kernel<0, false>), g, blk, 0, st, offsets, n_markets, nullptr, nullptr, counts,
                       chunks, keys, idx, nullptr, nullptr, nullptr, nullptr, 0);
    hipLaunchKernelGGL((plan_count_kernel<1, false>), g, blk, 0, st, offsets, n_markets, keys, counts, chunks, nullptr);
    hipLaunchKernelGGL((plan_scan_kernel<false>), sg, sblk, 0, st, counts, kPlanDigits * chunks, nullptr, (int64_t)0,
                       nullptr, nullptr, nullptr, 0);
    hipLaunchKernelGGL((plan_scatter_kernel<1, false>), g, blk, 0, st, offsets, n_markets, keys, idx, counts, chunks,
                       nullptr, order, nullptr, nullptr, nullptr, nullptr, 0);
  }
  *info_out = info;
  return check_launch("plan_bins_device");
}

extern "C" int bce_plan_bins_device_async(const int64_t* offsets, int64_t n_markets, int32_t* order,
                                          int64_t* bin_start_dev, void* scratch, int64_t scratch_bytes,
                                          void* stream) {
  BCE_REQUIRE(n_markets >= 0 && n_markets < ((int64_t)1 << 31), "plan_bins_device_async: bad n_markets %lld",
              (long long)n_markets);
  BCE_REQUIRE(bin_start_dev, "plan_bins_device_async: bin_start_dev NULL");
  hipStream_t st = as_stream(stream);
  if (n_markets == 0) {
    BCE_HIP(hipMemsetAsync(bin_start_dev, 0, (BCE_NBINS + 1) * sizeof(int64_t), st));
    return BCE_OK;
  }
  BCE_REQUIRE(offsets && order && scratch, "plan_bins_device_async: NULL argument");
  BCE_REQUIRE(scratch_bytes >= bce_plan_device_scratch_bytes(n_markets), "plan_bins_device_async: scratch too small");
  PlanInfo* info = nullptr;
  return plan_device_launch(offsets, n_markets, order, scratch, st, &info, bin_start_dev, 1);
}

extern "C" int bce_consensus_planned(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                                     const double* prob, int64_t n_signals, const double* relconf,
                                     const uint32_t* present_bits, int32_t n_sources,
                                     const int32_t* order, const int64_t* bin_start_host,
                                     int32_t mode, double* consensus, double* confidence,
                                     double* total_weight, int32_t* n_unique, int32_t* err_idx,
                                     int32_t* usid, double* weight, double* nweight, void* scratch,
                                     int64_t scratch_bytes, void* stream) {
  int rc = check_common(offsets, n_markets, sid, prob, relconf, present_bits, n_sources, consensus,
                        confidence, total_weight, n_unique);
  if (rc) return rc;
  BCE_REQUIRE(bin_start_host && (order || n_markets == 0), "planned: missing plan");
  BCE_REQUIRE(mode == BCE_MODE_EXACT || mode == BCE_MODE_FAST, "planned: bad mode %d", mode);
  BCE_REQUIRE(n_signals == 0 || (sid && prob), "planned: sid/prob NULL");
  hipStream_t st = as_stream(stream);
  ConsArgs base{};
  base.offsets = offsets; base.sid = sid; base.prob = prob;
  base.relconf = reinterpret_cast<const double2*>(relconf); base.pbits = present_bits;
  base.n_sources = n_sources; base.n_signals = n_signals; base.consensus = consensus; base.confidence = confidence;
  base.total_weight = total_weight; base.n_unique = n_unique; base.err_idx = err_idx;
  base.usid = usid; base.weight = weight; base.nweight = nweight; base.mode = mode;
  base.fault = fault_word();
  base.spin_cap = spin_cap();
  const bool seg_ok = n_sources <= (1 << 25);
  // The short-market bins (n <= 64) are small latency-bound launches: they run on a side
  // stream while the long bins run on st, longest first (joined before return).  Measured
  // on C3: 1.73 -> 1.65 ms; moving wide bins to the side stream too, or forking every bin
  // over 2-8 streams, was slower (profiles/r02_c3_plan_streams.jsonl); so was dealing every
  // bin over 2 or 4 streams with the resident grid shared out by estimated work (round 5,
  // profiles/archive/r05b/: one 8th of C3 0.233 -> 0.294 / 0.307 ms), and a small call's 65..1024
  // launches on a second side stream (0.2188 -> 0.2325 ms, profiles/archive/r05f/).
  hipStream_t side = st;
  std::unique_lock<std::mutex> fork_lock;
  constexpr int side_last = kPlanSideLast;
  // fork only when both streams get work: a batch of only short or only long markets runs on st
  // alone, without the fork / join events (~10 us of step boundary)
  const int nside = (bin_start_host[side_last + 1] > bin_start_host[0] &&
                     bin_start_host[BCE_NBINS] > bin_start_host[side_last + 1]) ? 1 : 0;
  rc = side_fork(st, nside, &side, &fork_lock);
  if (rc) return rc;
  // Launches: bin b runs with the markets of bins lo[b]..b in one kernel sized for bin b (its
  // own markets first, then the shorter bins' -- consensus_wide_kernel's list_hi).
  //   EXACT: the non-power-of-two bins (1025..1536, 2049..3072) always ride in the launch of the
  //   power-of-two bin above them: the exact kernel's LDS chain buffers allow two workgroups per
  //   CU at 3/6 waves as at 4/8, so the smaller workgroup only loses latency hiding, and a
  //   separate launch adds a tail.
  //   Small calls (a market shard, kMergeRounds): a launch whose markets would fill fewer than
  //   kMergeRounds rounds of its resident grid costs a ramp and a tail for little work, so FAST
  //   merges the non-power-of-two bins the same way and the 65..512 bins run as one 1-wave
  //   launch -- fewer, fuller launches for a 1/8 shard of C3.
  int lo[BCE_NBINS];
  for (int b = 0; b < BCE_NBINS; ++b) lo[b] = b;
  auto cnt = [&](int b0, int b1) { return bin_start_host[b1 + 1] - bin_start_host[b0]; };
  auto few = [&](int b0, int b1) {
    return cnt(b0, b1) > 0 && (double)cnt(b0, b1) < kMergeRounds * (double)wide_resident(kBinMax[b1], mode, n_sources);
  };
  for (int b : {kBinNp2Lo + 1, kBinNp2Hi + 1})
    if (mode == BCE_MODE_EXACT || few(b - 1, b)) lo[b] = b - 1;
  if (few(kPlanSideLast + 1, kPlanSideLast + 3)) lo[kPlanSideLast + 3] = kPlanSideLast + 1;  // 65..512 as one
  bool merged_away[BCE_NBINS] = {};
  for (int b = 0; b < BCE_NBINS; ++b)
    for (int k = lo[b]; k < b; ++k) merged_away[k] = true;
  // Launch order: longest bins first, except that the 2049..3072 bin precedes the 3073..4096
  // one: its 6-wave workgroups leave 4 of a CU's 16 wave slots free (two per CU at 128 VGPRs),
  // which the side stream's short-market kernels then fill (C3 fast -1.3%,
  // profiles/archive/r03x/order_ab.txt) -- and every main-stream launch that fills fewer than
  // kMergeRounds rounds of its resident grid (a shard's cut piece of a bin) moves behind the
  // full ones.  A small launch first ends while the side stream still holds CUs, and the big
  // persistent launch behind it, whose workgroups stride statically over its markets, then
  // starts part of its grid late and drags a tail (a planned C3 shard: 0.226 vs 0.15 ms for the
  // same bin-11 markets, profiles/r06c/).  Ordering every launch by estimated work instead cost
  // the full C3 batch 2% (1.325 vs 1.298 ms, profiles/r06e/).
  static const int kClassic[BCE_NBINS] = {12, 10, 11, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};
  int kOrder[BCE_NBINS];
  {
    int k = 0;
    for (int pass = 0; pass < 3; ++pass)
      for (int oi = 0; oi < BCE_NBINS; ++oi) {
        const int b = kClassic[oi];
        const bool side = b <= side_last;
        const bool small = !side && b < BCE_NBINS - 1 && !merged_away[b] && few(lo[b], b);
        if ((pass == 0 && !side && !small) || (pass == 1 && small) || (pass == 2 && side)) kOrder[k++] = b;
      }
  }
  for (int oi = 0; oi < BCE_NBINS && !rc; ++oi) {
    const int b = kOrder[oi];
    if (merged_away[b]) continue;
    const int b0 = lo[b];
    ConsArgs a = base;
    a.list = order + bin_start_host[b0];
    a.n_list = bin_start_host[b + 1] - bin_start_host[b0];
    if (b0 != b) {  // merged: this bin's (longer) markets first, then the bins below
      a.list_hi = order + bin_start_host[b];
      a.n_hi = bin_start_host[b + 1] - bin_start_host[b];
    }
    if (a.n_list == 0) continue;
    hipStream_t sb = (b <= side_last) ? side : st;
    if (b <= 3 && seg_ok) {
      static const int lens[4] = {8, 16, 32, 64};
      rc = launch_seg_for_len(lens[b], a, sb);
    } else if (b <= BCE_NBINS - 2) {
      rc = (b <= 3) ? launch_long_lds(a, sb) : launch_wide_for_len(kBinMax[b], a, sb);
    } else {
      // scratch stride from the caller's sizing (bce_consensus_scratch_bytes)
      const int grid = (int)(a.n_list < kHugeGrid ? a.n_list : kHugeGrid);
      const int64_t P = scratch_bytes / ((int64_t)grid * 4 * 8);
      if (P <= kLongMaxLds) {  // not BCE_REQUIRE: the side stream must still be joined
        set_error("planned: scratch too small for the >4096 bin");
        rc = BCE_EINVAL;
        break;
      }
      a.scratch = scratch;
      a.scratch_stride = P;
      hipLaunchKernelGGL((consensus_long_kernel<false>), dim3(grid), dim3(kLongThreads), 0, st, a);
      rc = check_launch("consensus_long_kernel<global>");
    }
    if (rc) break;
  }
  const int rj = side_join(st, nside);  // join even after a failed launch: st must not run ahead
  if (!rc) rc = rj;
  return rc;
}

// The planned launch driven by device bin boundaries (bce_plan_bins_device_async): no host
// sync between planning and consensus.  Every bin's kernel is launched with its resident grid
// (its market count is not known on the host) and reads its range of the plan order at entry
// (dev_range); an empty bin's launch exits at once.  The launch structure is the full batch's:
// EXACT runs the non-power-of-two bins in the launch of the bin above, FAST gives every bin its
// own launch (no small-call merges: the counts are on the device), longest bins first, bins
// 0..3 on the side stream.  Markets longer than 4096 are not computed: they raise the device
// fault word (a caller with such markets uses the host-synchronised plan).
extern "C" int bce_consensus_planned_device(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                                            const double* prob, int64_t n_signals, const double* relconf,
                                            const uint32_t* present_bits, int32_t n_sources, const int32_t* order,
                                            const int64_t* bin_start_dev, int32_t mode, double* consensus,
                                            double* confidence, double* total_weight, int32_t* n_unique,
                                            int32_t* err_idx, int32_t* usid, double* weight, double* nweight,
                                            void* stream) {
  int rc = check_common(offsets, n_markets, sid, prob, relconf, present_bits, n_sources, consensus,
                        confidence, total_weight, n_unique);
  if (rc) return rc;
  if (n_markets == 0) return BCE_OK;
  BCE_REQUIRE(bin_start_dev && order, "planned_device: missing plan");
  BCE_REQUIRE(mode == BCE_MODE_EXACT || mode == BCE_MODE_FAST, "planned_device: bad mode %d", mode);
  BCE_REQUIRE(n_signals == 0 || (sid && prob), "planned_device: sid/prob NULL");
  hipStream_t st = as_stream(stream);
  ConsArgs base{};
  base.offsets = offsets; base.sid = sid; base.prob = prob;
  base.relconf = reinterpret_cast<const double2*>(relconf); base.pbits = present_bits;
  base.n_sources = n_sources; base.n_signals = n_signals; base.consensus = consensus; base.confidence = confidence;
  base.total_weight = total_weight; base.n_unique = n_unique; base.err_idx = err_idx;
  base.usid = usid; base.weight = weight; base.nweight = nweight; base.mode = mode;
  base.fault = fault_word();
  base.spin_cap = spin_cap();
  base.list = order;           // the whole plan order: each launch's range is read on the device
  base.n_list = n_markets;     // upper bound: sizes the launch grids
  base.dev_bins = bin_start_dev;
  const bool seg_ok = n_sources <= (1 << 25);
  hipStream_t side = st;
  std::unique_lock<std::mutex> fork_lock;
  rc = side_fork(st, 1, &side, &fork_lock);
  if (rc) return rc;
  static const int kOrderDev[BCE_NBINS - 1] = {10, 11, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};
  for (int oi = 0; oi < BCE_NBINS - 1 && !rc; ++oi) {
    const int b = kOrderDev[oi];
    const bool np2 = (b == kBinNp2Lo || b == kBinNp2Hi);
    if (mode == BCE_MODE_EXACT && np2) continue;  // rides in the launch of the bin above
    ConsArgs a = base;
    a.dev_b1 = b;
    a.dev_b0 = (mode == BCE_MODE_EXACT && (b == kBinNp2Lo + 1 || b == kBinNp2Hi + 1)) ? b - 1 : b;
    hipStream_t sb = (b <= kPlanSideLast) ? side : st;
    if (b <= 3 && seg_ok) {
      static const int lens[4] = {8, 16, 32, 64};
      rc = launch_seg_for_len(lens[b], a, sb);
    } else if (b <= 3) {
      rc = BCE_EUNSUPPORTED;  // (n_sources > 2^25: the long-LDS kernel has no device range)
      set_error("planned_device: more than 2^25 sources -- use bce_consensus_planned");
    } else {
      rc = launch_wide_for_len(kBinMax[b], a, sb);
    }
  }
  const int rj = side_join(st, 1);
  if (!rc) rc = rj;
  return rc;
}

// ======================================================================================
// validation only: core.validate_input_payload range check (core.py:59-60)
// ======================================================================================
namespace bce {
__global__ __launch_bounds__(256) void validate_kernel(const int64_t* offsets, int64_t n_markets,
                                                       const double* prob, int32_t* err_idx) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t m = wave; m < n_markets; m += nwaves) {
    const int64_t a = offsets[m], b = offsets[m + 1];
    int32_t e = -1;
    for (int64_t base = a; base < b; base += 64) {
      const int64_t i = base + lane;
      const double p = (i < b) ? prob[i] : 0.5;
      const unsigned long long bad = ballot(p < 0.0 || p > 1.0);  // NaN passes
      if (bad) {
        e = (int32_t)(base - a) + __builtin_ctzll(bad);
        break;
      }
    }
    if (lane == 0) err_idx[m] = e;
  }
}
}  // namespace bce


extern "C" int bce_validate_csr(const int64_t* offsets, int64_t n_markets, const double* prob,
                                int32_t* err_idx, void* stream) {
  BCE_REQUIRE(n_markets >= 0, "validate: n_markets < 0");
  if (n_markets == 0) return BCE_OK;
  BCE_REQUIRE(offsets && prob && err_idx, "validate: NULL argument");
  int64_t blocks = (n_markets + 3) / 4;
  const int64_t cap = (int64_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(validate_kernel, dim3((int)blocks), dim3(256), 0, as_stream(stream), offsets,
                     n_markets, prob, err_idx);
  return check_launch("validate_kernel");
}

// ======================================================================================
// source-table packing: separate (rel, conf, present) -> the consensus layout
// ======================================================================================
namespace bce {
__global__ __launch_bounds__(256) void table_pack_kernel(int64_t n, const double* rel, const double* conf,
                                                         const uint8_t* present, double2* relconf,
                                                         uint32_t* bits) {
  const int lane = lane_id();
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < ((n + 63) & ~63ll);
       s += (int64_t)gridDim.x * blockDim.x) {
    const bool in = s < n;
    if (in) relconf[s] = make_double2(rel[s], conf[s]);
    const unsigned long long b = ballot(in && (present == nullptr || present[s] != 0));
    if (lane == 0 && s < n) bits[s >> 5] = (uint32_t)b;
    if (lane == 32 && s < n) bits[s >> 5] = (uint32_t)(b >> 32);
  }
}
}  // namespace bce

extern "C" int bce_table_pack(int64_t n, const double* rel, const double* conf, const uint8_t* present,
                              double* relconf, uint32_t* present_bits, void* stream) {
  BCE_REQUIRE(n >= 0, "table_pack: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(rel && conf && relconf && present_bits, "table_pack: NULL argument");
  BCE_REQUIRE((uintptr_t)relconf % 16 == 0, "table_pack: relconf must be 16-byte aligned");
  int64_t blocks = (n + 255) / 256;
  const int64_t cap = (int64_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(table_pack_kernel, dim3((int)blocks), dim3(256), 0, as_stream(stream), n, rel, conf,
                     present, reinterpret_cast<double2*>(relconf), present_bits);
  return check_launch("table_pack_kernel");
}
