// aggregate.hip -- cross-market aggregation of consensus outputs
// (CrossMarketAggregator.aggregate_consensus, market.py:340-408) for many groups at once.
//
// A group is an ordered list of market indices (the markets matched by the patterns, in
// list_markets order, duplicates kept: market.py:355-357).  Members without a consensus
// (no result, or consensus None) are skipped (:369-375).  Per group:
//   weighted_average  sum(cons*conf)/sum(conf), or sum(cons)/k when sum(conf) == 0 (:386-393)
//   median            sorted(cons)[k // 2] (:394-397)
//   majority          #(cons >= 0.5) / k (:398-401)
//   confidence        sum(conf) / k (:407)
// Sums run left to right in list order from 0.0 (builtin sum), FP contraction off, so
// every output is bit-identical to the reference.  One 256-thread workgroup per group:
// chunks of 256 members are gathered, compacted into LDS in list order with ballots, and
// three lanes of wave 0 carry the three ordered chains; the median is an exact 8-pass
// MSB radix select over order-preserving 64-bit keys (no sort, no extra memory).
#include "bce_device.hpp"
#include "bce_internal.hpp"

#pragma clang fp contract(off)

namespace bce {

struct AggArgs {
  const int64_t* goff;
  int64_t n_groups;
  const int64_t* members;
  int64_t n_markets;
  const double* cons;
  const double* conf;
  const uint8_t* has;
  double* wavg;
  double* median;
  double* majority;
  double* mean_conf;
  int64_t* n_included;
};

// Order-preserving key of a double (total order; -0.0 is keyed as +0.0 because sorted()
// treats them as equal).
__device__ __forceinline__ uint64_t f64_key(double x) {
  if (x == 0.0) x = 0.0;
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_f64(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

constexpr int kAggT = 256;

__global__ __launch_bounds__(kAggT) void aggregate_kernel(AggArgs a) {
  __shared__ double sV[3][kAggT];  // conf, cons, cons*conf of the chunk's valid members
  __shared__ int sWave[kAggT / 64 + 1];
  __shared__ int sHist[256];
  __shared__ unsigned long long sVotes;
  __shared__ double sTot[3];
  __shared__ uint64_t sPrefix;
  __shared__ int64_t sRank;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    const int64_t b = a.goff[g], e = a.goff[g + 1];
    double chain = 0.0;  // lanes 0..2 of wave 0: sum(conf), sum(cons), sum(cons*conf)
    int64_t k = 0;
    if (t == 0) sVotes = 0;
    for (int64_t c0 = b; c0 < e; c0 += kAggT) {
      const int64_t i = c0 + t;
      bool valid = false;
      double x = 0.0, c = 0.0;
      if (i < e) {
        const int64_t m = a.members[i];
        valid = (m >= 0 && m < a.n_markets) && a.has[m] != 0;
        if (valid) {
          x = a.cons[m];
          c = a.conf[m];
        }
      }
      const unsigned long long msk = ballot(valid);
      if (lane == 0) sWave[w] = __popcll(msk);
      __syncthreads();
      int base = 0, cnt = 0;
#pragma unroll
      for (int q = 0; q < kAggT / 64; ++q) {
        base += (q < w) ? sWave[q] : 0;
        cnt += sWave[q];
      }
      if (valid) {
        const int pos = base + __popcll(msk & lt);
        sV[0][pos] = c;
        sV[1][pos] = x;
        sV[2][pos] = x * c;  // market.py:391
      }
      const unsigned long long vm = ballot(valid && x >= 0.5);  // market.py:400
      if (lane == 0 && vm) atomicAdd(&sVotes, (unsigned long long)__popcll(vm));
      __syncthreads();
      if (t < 3) {
        const double* v = sV[t];
        for (int j = 0; j < cnt; ++j) chain = chain + v[j];
      }
      k += cnt;
      __syncthreads();  // chunk buffer reused
    }
    if (t < 3) sTot[t] = chain;
    __syncthreads();
    if (t == 0) {
      const double tconf = sTot[0], tcons = sTot[1], tprod = sTot[2];
      const double kd = (double)k;
      const bool any = k > 0;
      const double nan = __longlong_as_double(0x7FF8000000000000ll);
      if (a.n_included) a.n_included[g] = k;
      if (a.mean_conf) a.mean_conf[g] = any ? tconf / kd : nan;
      if (a.wavg) a.wavg[g] = !any ? nan : (tconf == 0.0) ? tcons / kd : tprod / tconf;
      if (a.majority) a.majority[g] = any ? (double)sVotes / kd : nan;
    }
    if (a.median) {
      // k-th smallest (k = count // 2) by MSB radix select, 8 bits per pass
      if (t == 0) {
        sPrefix = 0;
        sRank = k / 2;
      }
      for (int pass = 0; pass < 8 && k > 0; ++pass) {
        const int sh = 56 - 8 * pass;
        sHist[t] = 0;
        __syncthreads();
        const uint64_t pre = sPrefix;
        const uint64_t pmask = (pass == 0) ? 0ull : (~0ull << (sh + 8));
        for (int64_t i = b + t; i < e; i += kAggT) {
          const int64_t m = a.members[i];
          if (m >= 0 && m < a.n_markets && a.has[m]) {
            const uint64_t key = f64_key(a.cons[m]);
            if ((key & pmask) == pre) atomicAdd(&sHist[(key >> sh) & 255], 1);
          }
        }
        __syncthreads();
        if (t == 0) {
          int64_t r = sRank, acc = 0;
          int d = 0;
          for (; d < 255; ++d) {
            if (acc + sHist[d] > r) break;
            acc += sHist[d];
          }
          sRank = r - acc;
          sPrefix = pre | ((uint64_t)d << sh);
        }
        __syncthreads();
      }
      if (t == 0) a.median[g] = (k > 0) ? key_f64(sPrefix) : __longlong_as_double(0x7FF8000000000000ll);
    }
    __syncthreads();  // LDS state reused by the next group
  }
}

}  // namespace bce

using namespace bce;

extern "C" int bce_aggregate_groups(const int64_t* group_offsets, int64_t n_groups,
                                    const int64_t* members, int64_t n_markets,
                                    const double* consensus, const double* confidence,
                                    const uint8_t* has_consensus, double* wavg, double* median,
                                    double* majority, double* mean_conf, int64_t* n_included,
                                    void* stream) {
  BCE_REQUIRE(n_groups >= 0 && n_markets >= 0, "aggregate_groups: negative size");
  if (n_groups == 0) return BCE_OK;
  BCE_REQUIRE(group_offsets && members && consensus && confidence && has_consensus,
              "aggregate_groups: NULL input array");
  BCE_REQUIRE(wavg || median || majority || mean_conf || n_included, "aggregate_groups: no output");
  AggArgs a{group_offsets, n_groups, members, n_markets, consensus, confidence, has_consensus,
            wavg, median, majority, mean_conf, n_included};
  int64_t grid = n_groups;
  const int64_t cap = (int64_t)cu_count() * 8;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)grid), dim3(kAggT), 0, as_stream(stream), a);
  return check_launch("aggregate_kernel");
}
