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
