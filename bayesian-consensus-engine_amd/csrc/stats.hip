// stats.hip -- per-source agreement statistics and the dense re-estimation passes.
//
//   agreement_stats        CrossMarketAggregator.summarize_sources counts
//                          (market.py:279-304): int32 atomics, exact and order-free.
//   reestimate_consensus   config 5 pass 1: c_m = sum_a P[a][m] w_a / sum_a w_a, lane per
//                          market column of the agent-major matrix -> every load is
//                          coalesced AND each lane sums in agent order, which is the
//                          reference's sorted-source order (core.py:130-144): exact.
//   reestimate_agreement   config 5 pass 2: per-agent count of markets whose binary vote
//                          matches the consensus vote (market.py:298-304), ballot+popcount
//                          over (agent tile x market tile) blocks, LDS-collected counts.
//   reestimate_consensus_votes / reestimate_agreement_votes
//                          the single-read iteration: pass 1 also records every cell's vote
//                          (P >= 0.5) as one bit, 64 markets per word, plus the consensus
//                          votes and resolved masks per word; pass 2 then counts agreement
//                          from the bits (A*M/8 bytes) instead of re-reading P (8*A*M).
#include <type_traits>

#include "bce_device.hpp"
#include "bce_internal.hpp"

#pragma clang fp contract(off)

namespace bce {

__global__ __launch_bounds__(256) void agreement_kernel(const int64_t* offsets, int64_t n_markets,
                                                        const int32_t* sid, const double* prob,
                                                        const int8_t* outcome, int32_t* correct,
                                                        int32_t* total) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t m = wave; m < n_markets; m += nwaves) {
    const int8_t o = outcome[m];
    if (o < 0) continue;
    const int64_t a = offsets[m], b = offsets[m + 1];
    for (int64_t i = a + lane; i < b; i += 64) {
      const int s = sid[i];
      const bool predicted_true = prob[i] >= 0.5;  // market.py:298-299
      atomicAdd(&total[s], 1);
      if (predicted_true == (o != 0)) atomicAdd(&correct[s], 1);
    }
  }
}

// sum_a w[a] in agent order (the reference's total_weight loop, core.py:107-120).
__global__ void weight_total_kernel(const double* w, int64_t A, double* out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double t = 0.0;
    for (int64_t a = 0; a < A; ++a) t += w[a];
    *out = t;
  }
}

// Lane per market column; 4 columns per lane-group of loads would break the exact
// per-lane order, so each lane keeps one column and the wave streams 512-B rows.
__global__ __launch_bounds__(256) void reestimate_consensus_kernel(const double* __restrict__ P,
                                                                   int64_t A, int64_t M, int64_t ld,
                                                                   const double* __restrict__ w,
                                                                   const double* __restrict__ tot,
                                                                   double* __restrict__ cons,
                                                                   uint8_t* __restrict__ null_out) {
  const int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (m >= M) return;
  const double total = *tot;
  double ws = 0.0;
  const double* col = P + m;
  int64_t a = 0;
  for (; a + 8 <= A; a += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = col[(a + q) * ld];
#pragma unroll
    for (int q = 0; q < 8; ++q) ws += (0.0 + v[q]) * w[a + q];  // avg of one signal = 0 + p
  }
  for (; a < A; ++a) ws += (0.0 + col[a * ld]) * w[a];
  const bool isnull = (total == 0.0);
  cons[m] = isnull ? 0.0 : ws / total;
  null_out[m] = isnull ? 1 : 0;
}

// Block = a tile of 256*kAgMT markets x kAgAT agents.  Each thread keeps its markets'
// consensus votes in registers, streams the tile's agent rows with 4 rows x kAgMT loads
// in flight (coalesced across lanes), reduces each row's hits with ballots, collects the
// per-agent counts of the block in LDS and adds them to global memory once per block.
// (Counting is exact and order-free.)
constexpr int kAgMT = 8;    // markets per thread
constexpr int kAgAT = 256;  // agents per block

__global__ __launch_bounds__(256) void reestimate_agreement_kernel(const double* __restrict__ P,
                                                                   int64_t A, int64_t M, int64_t ld,
                                                                   const double* __restrict__ cons,
                                                                   const uint8_t* __restrict__ nul,
                                                                   long long* __restrict__ agree,
                                                                   long long* __restrict__ resolved) {
  __shared__ int32_t cntS[kAgAT];
  __shared__ int32_t part[4];
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wv = tid >> 6;
  const int64_t n_mt = (M + 256 * kAgMT - 1) / (256 * kAgMT);
  const int64_t mt = blockIdx.x % n_mt;
  const int64_t a0 = (blockIdx.x / n_mt) * kAgAT;
  const int64_t a1 = (A < a0 + kAgAT) ? A : a0 + kAgAT;
  const int64_t m0 = mt * 256 * kAgMT;
  cntS[tid] = 0;
  bool cv[kAgMT], ok[kAgMT], in[kAgMT];
  int nres = 0;
#pragma unroll
  for (int q = 0; q < kAgMT; ++q) {
    const int64_t m = m0 + q * 256 + tid;
    in[q] = m < M;
    ok[q] = in[q] && nul[m] == 0;
    cv[q] = ok[q] && cons[m] >= 0.5;  // market.py:298-299 with the consensus as outcome
    nres += ok[q] ? 1 : 0;
  }
  if (a0 == 0) {  // resolved-market count, once per market tile
    int c = nres;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) part[wv] = c;
  }
  __syncthreads();
  if (a0 == 0 && tid == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(resolved),
              (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
  const double* base = P + m0 + tid;
  for (int64_t a = a0; a < a1; a += 4) {
    double v[4][kAgMT];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int q = 0; q < kAgMT; ++q) v[k][q] = (a + k < a1 && in[q]) ? base[(a + k) * ld + q * 256] : 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < kAgMT; ++q) cnt += __popcll(ballot(ok[q] && ((v[k][q] >= 0.5) == cv[q])));
      if (lane == 0 && cnt && a + k < a1) atomicAdd(&cntS[a + k - a0], cnt);
    }
  }
  __syncthreads();
  if (tid < a1 - a0 && cntS[tid]) atomicAdd(reinterpret_cast<unsigned long long*>(&agree[a0 + tid]),
                                           (unsigned long long)cntS[tid]);
}

// Pass 1 with votes.  Lane per market column m = kVoteBlock*block + tid, so wave w of a block
// covers the 64 markets of vote word k = (kVoteBlock / 64)*block + w.  Agents are streamed kVoteRows rows
// at a time (coalesced 512-B row segments); the rows' vote ballots are spread over lanes
// 0..kVoteRows-1 and stored as contiguous bytes of vote_bits[k][a ..].  Every lane also
// carries the total weight in agent order (core.py:107-120: the same for every column,
// and free beside the stream), so no separate reduction launch is needed.
constexpr int kVoteRows = 16;
// A batch's kVoteRows weights: one vector load (lane q < kVoteRows holds w[a + q]), then a
// readlane pair per row into SGPRs -- instead of kVoteRows scalar loads held across the batch
// (32 SGPRs, which spilled to VGPR lanes: ~7 writelane / readlane per row).
constexpr bool kVoteWLane = true;
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int2 x = *reinterpret_cast<const int2*>(&v);
  int2 y;
  y.x = __builtin_amdgcn_readlane(x.x, l);
  y.y = __builtin_amdgcn_readlane(x.y, l);
  return *reinterpret_cast<const double*>(&y);
}
// v_writelane_b32 (the LLVM intrinsic; clang has no builtin for it): lane l of the result =
// src (wave-uniform), every other lane keeps old -- a row's vote ballot into its agent's lane
// without a (lane == q) mask per row held in SGPRs
__device__ int bce_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ unsigned long long writelane_u64(unsigned long long v, int l, unsigned long long old) {
  const unsigned lo = (unsigned)bce_writelane((int)(unsigned)v, l, (int)(unsigned)old);
  const unsigned hi = (unsigned)bce_writelane((int)(unsigned)(v >> 32), l, (int)(unsigned)(old >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
// kVoteBlock: threads per workgroup -- its waves read neighbouring 512-B pieces of each row:
// 1024 threads 22.74-22.98 ms per C5 iteration, 512 23.60-23.66, 256 23.61-23.79 (profiles/archive/r05zh/,
// archive/r05zi/)
constexpr int kVoteBlock = 1024;
constexpr bool kVoteXcd = true;
__global__ __launch_bounds__(kVoteBlock) void reestimate_consensus_votes_kernel(
    const double* __restrict__ P, int64_t A, int64_t M, int64_t ld, const double* __restrict__ w,
    double* __restrict__ cons, uint8_t* __restrict__ null_out, unsigned long long* __restrict__ vote_bits,
    unsigned long long* __restrict__ cvote_words, unsigned long long* __restrict__ ok_words,
    const int32_t* __restrict__ only_if) {
  // only_if (nullable): run only when *only_if != 0 -- the MFMA entry point launches this
  // kernel behind its own and lets the weight check pick one of the two on the device
  if (only_if && *only_if == 0) return;
  const int lane = lane_id();
  // kVoteXcd: workgroups are dealt round-robin to the 8 XCDs; block b takes column range
  // xcd_block(b) so each XCD streams one contiguous slice of every row
  int64_t blk = blockIdx.x;
  if constexpr (kVoteXcd) {
    const int64_t nb = gridDim.x, per = nb / 8, x = blk & 7, q = blk >> 3;
    if (blk < per * 8) blk = x * per + q;  // the last nb % 8 blocks keep their own ranges
  }
  const int64_t m = blk * (int64_t)blockDim.x + threadIdx.x;
  const int64_t k = m >> 6;
  if ((k << 6) >= M) return;  // whole wave past the last market (wave-uniform)
  const bool in = m < M;
  double ws = 0.0, total = 0.0;
  const double* col = P + (in ? m : 0);  // every lane's column address is valid: loads unconditional
  unsigned long long* vb = vote_bits + k * A;
  int64_t a = 0;
  for (; a + kVoteRows <= A; a += kVoteRows) {
    double v[kVoteRows];
#pragma unroll
    for (int q = 0; q < kVoteRows; ++q) v[q] = col[(a + q) * ld];  // lanes past M: column 0, never stored
    const double wl = kVoteWLane ? w[a + (lane & (kVoteRows - 1))] : 0.0;
    unsigned long long mine = 0;
#pragma unroll
    for (int q = 0; q < kVoteRows; ++q) {
      const double wq = kVoteWLane ? readlane_f64(wl, q) : w[a + q];
      // the signal's avg is 0 + p (core.py:116,136); p * w instead of (0 + p) * w differs only
      // in the sign of a zero product (p = -0.0), and ws -- which starts at +0.0 and so is
      // never -0.0 under round-to-nearest -- is unchanged by adding a zero of either sign
      ws += v[q] * wq;
      total += wq;
      mine = writelane_u64(ballot(in && v[q] >= 0.5), q, mine);  // market.py:298-299
    }
    if (lane < kVoteRows) vb[a + lane] = mine;
  }
  for (; a < A; ++a) {
    const double v = in ? col[a * ld] : 0.0;
    ws += (0.0 + v) * w[a];
    total += w[a];
    const unsigned long long b = ballot(in && v >= 0.5);
    if (lane == 0) vb[a] = b;
  }
  const bool isnull = (total == 0.0);
  const double c = isnull ? 0.0 : ws / total;
  if (in) {
    cons[m] = c;
    null_out[m] = isnull ? 1 : 0;
  }
  const unsigned long long okw = ballot(in && !isnull);
  const unsigned long long cvw = ballot(in && !isnull && c >= 0.5);
  if (lane == 0) {
    ok_words[k] = okw;
    cvote_words[k] = cvw;
  }
}

// Pass 2 from the vote bits: lane per agent, a block's 4 waves = 256 agents, blockIdx.y =
// a slice of the vote words; agree[a] += popc(ok & ~(vote ^ cvote)) per word.  The first
// agent block also counts the resolved markets of its slice.  (Exact, order-free.)
constexpr int kVoteUnroll = 8;
__global__ __launch_bounds__(256) void reestimate_agreement_votes_kernel(
    const unsigned long long* __restrict__ vote_bits, int64_t A, int64_t K,
    const unsigned long long* __restrict__ cvote_words, const unsigned long long* __restrict__ ok_words,
    long long* __restrict__ agree, long long* __restrict__ resolved) {
  const int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t per = (K + gridDim.y - 1) / gridDim.y;
  const int64_t k0 = blockIdx.y * per;
  const int64_t k1 = (K < k0 + per) ? K : k0 + per;
  const bool in = a < A;
  const unsigned long long* col = vote_bits + (in ? a : 0);
  long long acc = 0;
  int64_t k = k0;
  for (; k + kVoteUnroll <= k1; k += kVoteUnroll) {
    unsigned long long x[kVoteUnroll];
#pragma unroll
    for (int q = 0; q < kVoteUnroll; ++q) x[q] = in ? col[(k + q) * A] : 0ull;
#pragma unroll
    for (int q = 0; q < kVoteUnroll; ++q) acc += __popcll(ok_words[k + q] & ~(x[q] ^ cvote_words[k + q]));
  }
  for (; k < k1; ++k) acc += __popcll(ok_words[k] & ~((in ? col[k * A] : 0ull) ^ cvote_words[k]));
  if (in && acc) atomicAdd(reinterpret_cast<unsigned long long*>(&agree[a]), (unsigned long long)acc);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    long long r = 0;
    for (int64_t q = k0; q < k1; ++q) r += __popcll(ok_words[q]);
    if (r) atomicAdd(reinterpret_cast<unsigned long long*>(resolved), (unsigned long long)r);
  }
}

// ---- BCE_MODE_FAST pass 1 on the matrix cores ---------------------------------------
// w^T P as v_mfma_f64_16x16x4_f64, fed by the exact kernel's load schedule: lane = market
// column m0 + lane, one coalesced 512-B row segment per agent, the row's vote ballot IS the
// agent's vote word (no regrouping).  The lane's own cell is the B operand: lane l = n + 16k
// holds B[k][n] = P[a][m0 + 16k + n], and A is the agent's weight on a "diagonal" --
// lane l = i + 16k holds A[i][k] = (i % 4 == k) ? w_a : 0 -- so D[i][n] += w_a * B[i % 4][n]:
// row i of D accumulates market m0 + 16 (i % 4) + n, one MFMA per agent row of 64 markets,
// each market's sum in agent order (the MFMA's own rounding of the product; the three zero
// products are exact).  Accumulator r of lane l then holds D[4 (l >> 4) + r][l & 15], i.e.
// market m0 + 16 r + (l & 15): lane l's own sum is accumulator l >> 4.  One accumulator
// chain (the MFMA's dependent issue is hidden by the other waves), 8 waves per SIMD, as many
// row loads in flight as the exact kernel (kMfmaTwoAcc: even / odd agents on two chains).
// A zero operand times a NaN / inf cell would leak NaN into the other three markets of the
// column, so the B operand carries non-finite cells as 0 and the lane keeps its own
// column's flags: a NaN cell makes the consensus NaN (as in every order), any cell outside
// [0, 1] (inf included) sends the market to reestimate_fixup_kernel's exact redo.
// The sums are within 4*A*2^-53 of the exact consensus; markets within 8*A*2^-53 of 0.5 --
// where the vote could differ -- are redone in exact agent order too, so the votes and
// therefore the agreement counts are identical to the exact path.
// Precondition of the error bound and the null test: every weight finite and >= 0.
// reestimate_total_kernel checks it on the device; if any weight breaks it, the MFMA and
// fixup kernels exit at once and the exact kernel (launched behind them, gated on the same
// word) computes the iteration instead -- same results, exact-mode speed.
// (Rounds 3-4 used A = w broadcast over 16 rows and B = a 4-agent x 16-market block --
// 128-B row pieces and a 16-bit regrouping of four ballots per word, 25.0-26.0 ms against
// the exact kernel's 23.2-23.6; round 5's transposed variant of it took 28.7 ms,
// profiles/archive/r05f/.)
typedef double mfma_d4 __attribute__((ext_vector_type(4)));
// kMfma4x4: v_mfma_f64_4x4x4_4b_f64 instead -- four 4x4x4 blocks; lane l = 16 r + 4 b + c holds
// A[i = c][k = r], B[k = r][j = c] and D[i = r][j = c] of block b (probed on the GPU: an A lane
// one-hot reaches D lanes 16 i + 4 b + j from B lanes 16 k + 4 b + j).  With A on the same
// diagonal as the 16x16x4 form ((l & 3) == (l >> 4): i == k) lane l's D accumulates w_a times
// its OWN cell: one f64 accumulator per lane (2 VGPRs instead of 8), a shorter dependent chain
constexpr bool kMfma4x4 = true;
using mfma_acc = std::conditional_t<kMfma4x4, double, mfma_d4>;
__device__ __forceinline__ double mfma_f64(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ mfma_d4 mfma_f64(double a, double b, mfma_d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// the lane's own market sum: the 4x4x4 accumulator, or accumulator r = lane >> 4 of the 16x16x4
__device__ __forceinline__ double mfma_own(double acc, int) { return acc; }
__device__ __forceinline__ double mfma_own(mfma_d4 acc, int r) {
  return (r == 0) ? acc[0] : (r == 1) ? acc[1] : (r == 2) ? acc[2] : acc[3];
}
constexpr bool kMfmaTwoAcc = false;  // even / odd agent rows on two accumulator chains
// The exact kernel's load schedule: 16 agent rows per batch, no prefetch of the next batch,
// 1024-thread workgroups at 8 waves per SIMD (64 VGPRs, 9 spilled): 24.15-24.23 ms per C5
// iteration against 25.41-25.60 for 8 rows + prefetch on 512-thread workgroups at 6 waves,
// 8 rows / 1024 threads 25.74-25.76, 16 rows / 512 threads 24.30-24.36 (three interleaved reps,
// profiles/r06ab1/; the exact pass 23.59-23.88 on that box)
constexpr int kMfmaRows = 16;        // agent rows per batch (the exact kernel: kVoteRows = 16)
constexpr bool kMfmaPrefetch = false;
constexpr int kMfmaWpe = kMfmaPrefetch ? 6 : 8;  // waves per SIMD the VGPR budget allows
constexpr int kMfmaBlock = 1024;

__global__ __launch_bounds__(256) void reestimate_total_kernel(const double* __restrict__ w, int64_t A,
                                                               double* __restrict__ total_fast,
                                                               int32_t* __restrict__ nflag) {
  __shared__ double part[256];
  __shared__ int badS;
  if (threadIdx.x == 0) badS = 0;
  __syncthreads();
  double s = 0.0;
  bool bad = false;
  for (int64_t a = threadIdx.x; a < A; a += 256) {
    const double x = w[a];
    s += x;  // fixed order: deterministic
    bad = bad || !(x >= 0.0 && x <= __builtin_huge_val());  // negative, NaN or +inf
  }
  if (bad) badS = 1;
  part[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *total_fast = part[0];
    nflag[0] = 0;     // flagged-market count
    nflag[1] = badS;  // 1: a weight breaks the precondition -> the exact kernel runs instead
  }
}

__global__ __launch_bounds__(kMfmaBlock) __attribute__((amdgpu_waves_per_eu(kMfmaWpe, kMfmaWpe))) void reestimate_votes_mfma_kernel(
    const double* __restrict__ P, int64_t A, int64_t M, int64_t ld, const double* __restrict__ w,
    const double* __restrict__ total_fast, double* __restrict__ cons, uint8_t* __restrict__ null_out,
    unsigned long long* __restrict__ vote_bits, unsigned long long* __restrict__ cvote_words,
    unsigned long long* __restrict__ ok_words, int32_t* __restrict__ nflag, int32_t* __restrict__ flags) {
  if (nflag[1]) return;  // weights outside [0, inf): the gated exact kernel does this iteration
  const int lane = lane_id();
  int64_t blk = blockIdx.x;  // one contiguous column slice per XCD, as the exact pass (kVoteXcd)
  if constexpr (kVoteXcd) {
    const int64_t nb = gridDim.x, per = nb / 8, x = blk & 7, q = blk >> 3;
    if (blk < per * 8) blk = x * per + q;
  }
  const int64_t m = blk * (int64_t)blockDim.x + threadIdx.x;
  const int64_t k = m >> 6;
  if ((k << 6) >= M) return;  // whole wave past the last market (wave-uniform)
  const bool in = m < M;
  // A[i][k] with i = lane & 15, k = lane >> 4 (16x16x4) or i = lane & 3, k = lane >> 4 (4x4x4)
  const bool diag = (lane & 3) == (lane >> 4);
  const double* col = P + (in ? m : 0);  // every lane's column address is valid: loads unconditional
  unsigned long long* vb = vote_bits + k * A;
  mfma_acc acc0{}, acc1{};
  bool odd = false, hnan = false;
  const double dsel = diag ? 1.0 : 0.0;  // A = w_a * dsel: w_a or +0 (w finite >= 0)
  // b = the cell clamped to [0, 1], NaN -> 0 (IEEE maxNum): equal to v exactly for a cell in
  // [0, 1] (-0.0 compares equal), so b != v marks every other cell, NaN included; and
  // b >= 0.5 iff v >= 0.5 for every v (the vote)
  auto row = [&](double v, double wq, mfma_acc& acc) {
    const double b = __builtin_fmin(__builtin_fmax(v, 0.0), 1.0);
    odd = odd || (b != v);
    hnan = hnan || (v != v);
    acc = mfma_f64(wq * dsel, b, acc);
  };
  int64_t a = 0;
  // kMfmaPrefetch: the next batch's rows are issued before this batch's MFMA chain (whose
  // dependent issue would otherwise hold back the next loads)
  double v[kMfmaRows];
  if (kMfmaPrefetch && kMfmaRows <= A) {
#pragma unroll
    for (int q = 0; q < kMfmaRows; ++q) v[q] = col[q * ld];
  }
  for (; a + kMfmaRows <= A; a += kMfmaRows) {
    double vn[kMfmaRows];
    if (kMfmaPrefetch) {
      if (a + 2 * kMfmaRows <= A) {  // wave-uniform
#pragma unroll
        for (int q = 0; q < kMfmaRows; ++q) vn[q] = col[(a + kMfmaRows + q) * ld];
      }
    } else {
#pragma unroll
      for (int q = 0; q < kMfmaRows; ++q) v[q] = col[(a + q) * ld];  // lanes past M: column 0 (b clamped)
    }
    const double wl = kVoteWLane ? w[a + (lane & (kMfmaRows - 1))] : 0.0;
    unsigned long long mine = 0;
#pragma unroll
    for (int q = 0; q < kMfmaRows; ++q) {
      row(v[q], kVoteWLane ? readlane_f64(wl, q) : w[a + q], (kMfmaTwoAcc && (q & 1)) ? acc1 : acc0);
      mine = writelane_u64(ballot(in && v[q] >= 0.5), q, mine);  // market.py:298-299
    }
    if (lane < kMfmaRows) vb[a + lane] = mine;
    if (kMfmaPrefetch) {
#pragma unroll
      for (int q = 0; q < kMfmaRows; ++q) v[q] = vn[q];
    }
  }
  for (; a < A; ++a) {
    const double v = in ? col[a * ld] : 0.0;
    row(v, w[a], acc0);
    const unsigned long long bq = ballot(in && v >= 0.5);
    if (lane == 0) vb[a] = bq;
  }
  const int r = lane >> 4;
  const double s0 = mfma_own(acc0, r);
  const double s1 = kMfmaTwoAcc ? mfma_own(acc1, r) : 0.0;
  const double total = *total_fast;
  const bool isnull = (total == 0.0);  // w >= 0: zero in every order iff every weight is zero
  const double c = isnull ? 0.0 : hnan ? __builtin_nan("") : (kMfmaTwoAcc ? s0 + s1 : s0) / total;
  // |fast - exact| <= ~4*A*2^-53 for cells in [0, 1] (both sums of non-negative terms within
  // A*2^-53 relative of the true one, c <= 1); a column holding another value is redone,
  // a column holding a NaN never (NaN in every order)
  const double bound = 8.0 * (double)(A + 2) * 0x1p-53;
  const bool near = in && !isnull && !hnan && (fabs(c - 0.5) <= bound || odd);
  if (in) {
    cons[m] = c;
    null_out[m] = isnull ? 1 : 0;
  }
  if (near) flags[atomicAdd(nflag, 1)] = (int32_t)m;
  const unsigned long long okw = ballot(in && !isnull);
  const unsigned long long cvw = ballot(in && !isnull && c >= 0.5);
  if (lane == 0) {
    ok_words[k] = okw;
    cvote_words[k] = cvw;
  }
}

// Exact redo of the flagged markets (agent-order sums, as reestimate_consensus_votes_kernel):
// lane per flagged market, 64 flags per wave (grid-stride over the flag list, whose length
// only the device knows), agents streamed kVoteRows rows at a time.  Each lane runs its own
// two ordered chains (core.py:116,120,136), so 64 markets advance per instruction; the flag
// list is filled a wave's ballot at a time in column order, so neighbouring lanes mostly
// read neighbouring columns.
__global__ __launch_bounds__(256) void reestimate_fixup_kernel(const double* __restrict__ P, int64_t A, int64_t ld,
                                                               const double* __restrict__ w,
                                                               const int32_t* __restrict__ nflag,
                                                               const int32_t* __restrict__ flags,
                                                               double* __restrict__ cons,
                                                               unsigned long long* __restrict__ cvote_words) {
  const int nf = nflag[0];
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t f0 = wave * 64; f0 < nf; f0 += nwaves * 64) {
    const int64_t f = f0 + lane_id();
    const bool in = f < nf;
    const int64_t m = in ? flags[f] : 0;
    const double* col = P + m;
    double ws = 0.0, total = 0.0;
    int64_t a = 0;
    for (; a + kVoteRows <= A; a += kVoteRows) {
      double v[kVoteRows];
#pragma unroll
      for (int q = 0; q < kVoteRows; ++q) v[q] = in ? col[(a + q) * ld] : 0.0;
#pragma unroll
      for (int q = 0; q < kVoteRows; ++q) {
        const double wq = w[a + q];
        ws += (0.0 + v[q]) * wq;
        total += wq;
      }
    }
    for (; a < A; ++a) {
      const double wq = w[a];
      ws += (0.0 + (in ? col[a * ld] : 0.0)) * wq;
      total += wq;
    }
    if (in) {
      const double c = ws / total;  // total > 0: flagged markets are not null
      cons[m] = c;
      const unsigned long long bit = 1ull << (m & 63);
      if (c >= 0.5) atomicOr(&cvote_words[m >> 6], bit);
      else atomicAnd(&cvote_words[m >> 6], ~bit);
    }
  }
}

__global__ void reestimate_weights_kernel(int64_t A, const long long* agree, const long long* resolved,
                                          double* w) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < A;
       a += (int64_t)gridDim.x * blockDim.x) {
    const long long tot = *resolved;
    w[a] = tot > 0 ? (double)agree[a] / (double)tot : 0.5;  // market.py:310
  }
}

}  // namespace bce

using namespace bce;

extern "C" int bce_agreement_stats(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                                   const double* prob, const int8_t* outcome, int32_t* correct,
                                   int32_t* total, void* stream) {
  BCE_REQUIRE(n_markets >= 0, "agreement: n_markets < 0");
  if (n_markets == 0) return BCE_OK;
  BCE_REQUIRE(offsets && sid && prob && outcome && correct && total, "agreement: NULL argument");
  int64_t blocks = (n_markets + 3) / 4;
  const int64_t cap = (int64_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(agreement_kernel, dim3((int)blocks), dim3(256), 0, as_stream(stream), offsets,
                     n_markets, sid, prob, outcome, correct, total);
  return check_launch("agreement_kernel");
}

extern "C" int bce_reestimate_consensus(const double* P, int64_t A, int64_t M, int64_t ld,
                                        const double* w, double* consensus, uint8_t* null_out,
                                        void* stream) {
  BCE_REQUIRE(A > 0 && M >= 0 && ld >= M, "reestimate: bad shape");
  if (M == 0) return BCE_OK;
  BCE_REQUIRE(P && w && consensus && null_out, "reestimate: NULL argument");
  hipStream_t st = as_stream(stream);
  double* tot = nullptr;
  BCE_HIP(hipMallocAsync((void**)&tot, sizeof(double), st));
  hipLaunchKernelGGL(weight_total_kernel, dim3(1), dim3(64), 0, st, w, A, tot);
  hipLaunchKernelGGL(reestimate_consensus_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st,
                     P, A, M, ld, w, tot, consensus, null_out);
  int rc = check_launch("reestimate_consensus_kernel");
  BCE_HIP(hipFreeAsync(tot, st));
  return rc;
}

extern "C" int bce_reestimate_agreement(const double* P, int64_t A, int64_t M, int64_t ld,
                                        const double* consensus, const uint8_t* null_in,
                                        int64_t* agreement, int64_t* resolved, void* stream) {
  BCE_REQUIRE(A > 0 && M >= 0 && ld >= M, "reestimate_agreement: bad shape");
  if (M == 0) return BCE_OK;
  BCE_REQUIRE(P && consensus && null_in && agreement && resolved, "reestimate_agreement: NULL");
  const int64_t n_mt = (M + 256 * kAgMT - 1) / (256 * kAgMT);
  const int64_t n_at = (A + kAgAT - 1) / kAgAT;
  BCE_REQUIRE(n_mt * n_at < (1ll << 31), "reestimate_agreement: grid too large");
  hipLaunchKernelGGL(reestimate_agreement_kernel, dim3((unsigned)(n_mt * n_at)),
                     dim3(256), 0, as_stream(stream), P, A, M, ld, consensus, null_in,
                     reinterpret_cast<long long*>(agreement), reinterpret_cast<long long*>(resolved));
  return check_launch("reestimate_agreement_kernel");
}

extern "C" int bce_reestimate_weights(int64_t A, const int64_t* agreement, const int64_t* resolved,
                                      double* w, void* stream) {
  BCE_REQUIRE(A > 0 && agreement && resolved && w, "reestimate_weights: bad argument");
  hipLaunchKernelGGL(reestimate_weights_kernel, dim3((unsigned)((A + 255) / 256)), dim3(256), 0,
                     as_stream(stream), A, reinterpret_cast<const long long*>(agreement),
                     reinterpret_cast<const long long*>(resolved), w);
  return check_launch("reestimate_weights_kernel");
}

extern "C" int bce_reestimate_consensus_votes(const double* P, int64_t A, int64_t M, int64_t ld,
                                              const double* w, double* consensus, uint8_t* null_out,
                                              uint64_t* vote_bits, uint64_t* cvote_words,
                                              uint64_t* ok_words, void* stream) {
  BCE_REQUIRE(A > 0 && M >= 0 && ld >= M, "reestimate_votes: bad shape");
  if (M == 0) return BCE_OK;
  BCE_REQUIRE(P && w && consensus && null_out && vote_bits && cvote_words && ok_words,
              "reestimate_votes: NULL argument");
  hipLaunchKernelGGL(reestimate_consensus_votes_kernel, dim3((unsigned)((M + kVoteBlock - 1) / kVoteBlock)), dim3(kVoteBlock), 0,
                     as_stream(stream), P, A, M, ld, w, consensus, null_out,
                     reinterpret_cast<unsigned long long*>(vote_bits), reinterpret_cast<unsigned long long*>(cvote_words),
                     reinterpret_cast<unsigned long long*>(ok_words), (const int32_t*)nullptr);
  return check_launch("reestimate_consensus_votes_kernel");
}

extern "C" int bce_reestimate_agreement_votes(const uint64_t* vote_bits, int64_t A, int64_t M,
                                              const uint64_t* cvote_words, const uint64_t* ok_words,
                                              int64_t* agreement, int64_t* resolved, void* stream) {
  BCE_REQUIRE(A > 0 && M >= 0, "reestimate_agreement_votes: bad shape");
  if (M == 0) return BCE_OK;
  BCE_REQUIRE(vote_bits && cvote_words && ok_words && agreement && resolved, "reestimate_agreement_votes: NULL");
  const int64_t K = (M + 63) / 64;
  const int64_t ab = (A + 255) / 256;
  // enough blocks to fill the chip: slices of the vote words across blockIdx.y
  int64_t ks = (4 * (int64_t)cu_count() * 8 + ab - 1) / ab;
  if (ks > K) ks = K;
  if (ks > 65535) ks = 65535;
  if (ks < 1) ks = 1;
  BCE_REQUIRE(ab < (1ll << 31), "reestimate_agreement_votes: grid too large");
  hipLaunchKernelGGL(reestimate_agreement_votes_kernel, dim3((unsigned)ab, (unsigned)ks), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const unsigned long long*>(vote_bits), A, K,
                     reinterpret_cast<const unsigned long long*>(cvote_words),
                     reinterpret_cast<const unsigned long long*>(ok_words), reinterpret_cast<long long*>(agreement),
                     reinterpret_cast<long long*>(resolved));
  return check_launch("reestimate_agreement_votes_kernel");
}

extern "C" int bce_reestimate_consensus_votes_mfma(const double* P, int64_t A, int64_t M, int64_t ld,
                                                   const double* w, double* consensus, uint8_t* null_out,
                                                   uint64_t* vote_bits, uint64_t* cvote_words, uint64_t* ok_words,
                                                   void* scratch, int64_t scratch_bytes, void* stream) {
  BCE_REQUIRE(A > 0 && M >= 0 && ld >= M, "reestimate_votes_mfma: bad shape");
  if (M == 0) return BCE_OK;
  BCE_REQUIRE(P && w && consensus && null_out && vote_bits && cvote_words && ok_words && scratch,
              "reestimate_votes_mfma: NULL argument");
  BCE_REQUIRE(scratch_bytes >= bce_reestimate_mfma_scratch_bytes(M),
              "reestimate_votes_mfma: scratch too small (%lld < %lld)", (long long)scratch_bytes,
              (long long)bce_reestimate_mfma_scratch_bytes(M));
  BCE_REQUIRE((uintptr_t)scratch % 8 == 0, "reestimate_votes_mfma: scratch must be 8-byte aligned");
  hipStream_t st = as_stream(stream);
  double* total = reinterpret_cast<double*>(scratch);
  int32_t* nflag = reinterpret_cast<int32_t*>(total + 1);
  int32_t* flags = nflag + 2;
  hipLaunchKernelGGL(reestimate_total_kernel, dim3(1), dim3(256), 0, st, w, A, total, nflag);
  int rc = check_launch("reestimate_total_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(reestimate_votes_mfma_kernel, dim3((unsigned)((M + kMfmaBlock - 1) / kMfmaBlock)), dim3(kMfmaBlock), 0, st, P, A, M, ld,
                     w, total, consensus, null_out, reinterpret_cast<unsigned long long*>(vote_bits),
                     reinterpret_cast<unsigned long long*>(cvote_words), reinterpret_cast<unsigned long long*>(ok_words),
                     nflag, flags);
  rc = check_launch("reestimate_votes_mfma_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(reestimate_fixup_kernel, dim3((unsigned)cu_count() * 4), dim3(256), 0, st, P, A, ld, w, nflag,
                     flags, consensus, reinterpret_cast<unsigned long long*>(cvote_words));
  rc = check_launch("reestimate_fixup_kernel");
  if (rc) return rc;
  // precondition fallback (weights negative / NaN / inf): exits at once unless nflag[1] != 0
  hipLaunchKernelGGL(reestimate_consensus_votes_kernel, dim3((unsigned)((M + kVoteBlock - 1) / kVoteBlock)), dim3(kVoteBlock), 0, st, P, A, M,
                     ld, w, consensus, null_out, reinterpret_cast<unsigned long long*>(vote_bits),
                     reinterpret_cast<unsigned long long*>(cvote_words),
                     reinterpret_cast<unsigned long long*>(ok_words), (const int32_t*)(nflag + 1));
  return check_launch("reestimate_consensus_votes_kernel (fallback)");
}

extern "C" int64_t bce_reestimate_mfma_scratch_bytes(int64_t M) { return 16 + 4 * (M > 0 ? M : 1); }
