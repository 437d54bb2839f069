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
// chunks of 1024 members are gathered (indices two chunks ahead, values one chunk ahead of
// use), compacted into LDS in list order with ballots, and three lanes of wave 0 carry the
// three ordered chains in 8-term batches; the median is an exact 8-pass
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

// One workgroup per group (no per-CU cap): -15% against 8 looping workgroups per CU.
// kAggWpe: minimum waves per SIMD the VGPR budget must allow.  The compiler's own choice, 90
// VGPRs, holds five groups per CU; 6 (78 VGPRs, 2 spilled) holds six -- as many as the 25.7 KB
// of LDS allows: 0.0860 vs 0.0943 ms (+median 0.173 vs 0.193, profiles/archive/r04w/).  Dropping the
// cons*conf LDS array so more groups fit (the product formed in the chain) ran 2x slower
// (0.19-0.22 ms, profiles/archive/r04v/; code reverted): the chains' loop is the critical path.
// Round 5: the same pipelining in C++ (4-term batches, the next read during the adds) ran 0.117
// vs 0.0858 ms (profiles/archive/r05o/; the compiler waited on every batch, 8- or 16-term batches
// spilled 35 / 71 VGPRs) -- hence the asm chain below.
constexpr int kAggWpe = 6;
// The last chunk's ordered chains (kAggChainAsm): acc += src[0..ce) left to right in asm, four
// 4-term batches in fixed registers v[48:79] (inside the 80-VGPR budget), each reloaded 16 terms
// ahead right after its adds -- the compiler's own loop waits on every batch (it copies the
// loop-carried batch behind an lgkmcnt(0)).  Run after the chunk loop, where the next chunk's
// gather registers are dead; reads may run 16 past ce (inside the kernel's LDS).  f4 line:
// 0.0723 ms against 0.0858 without it, 0.0764 with two batches, 0.0728 with six
// (profiles/archive/r05za/, archive/r05zb/).
constexpr bool kAggChainAsm = true;
__device__ __forceinline__ void agg_chain_asm(double& acc, const double* src, int ce) {
  const int steps = ce / 16;
  const int nfull = steps * 16;
  if (steps) {
    unsigned addr = (unsigned)(uintptr_t)src;
    int st = steps;
    asm volatile(
        "ds_read_b128 v[48:51], %[ad] offset:0\n"
        "ds_read_b128 v[52:55], %[ad] offset:16\n"
        "ds_read_b128 v[56:59], %[ad] offset:32\n"
        "ds_read_b128 v[60:63], %[ad] offset:48\n"
        "ds_read_b128 v[64:67], %[ad] offset:64\n"
        "ds_read_b128 v[68:71], %[ad] offset:80\n"
        "ds_read_b128 v[72:75], %[ad] offset:96\n"
        "ds_read_b128 v[76:79], %[ad] offset:112\n"
        "1:\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[48:49]\n"
        "v_add_f64 %[acc], %[acc], v[50:51]\n"
        "v_add_f64 %[acc], %[acc], v[52:53]\n"
        "v_add_f64 %[acc], %[acc], v[54:55]\n"
        "ds_read_b128 v[48:51], %[ad] offset:128\n"
        "ds_read_b128 v[52:55], %[ad] offset:144\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[56:57]\n"
        "v_add_f64 %[acc], %[acc], v[58:59]\n"
        "v_add_f64 %[acc], %[acc], v[60:61]\n"
        "v_add_f64 %[acc], %[acc], v[62:63]\n"
        "ds_read_b128 v[56:59], %[ad] offset:160\n"
        "ds_read_b128 v[60:63], %[ad] offset:176\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[64:65]\n"
        "v_add_f64 %[acc], %[acc], v[66:67]\n"
        "v_add_f64 %[acc], %[acc], v[68:69]\n"
        "v_add_f64 %[acc], %[acc], v[70:71]\n"
        "ds_read_b128 v[64:67], %[ad] offset:192\n"
        "ds_read_b128 v[68:71], %[ad] offset:208\n"
        "s_waitcnt lgkmcnt(6)\n"
        "v_add_f64 %[acc], %[acc], v[72:73]\n"
        "v_add_f64 %[acc], %[acc], v[74:75]\n"
        "v_add_f64 %[acc], %[acc], v[76:77]\n"
        "v_add_f64 %[acc], %[acc], v[78:79]\n"
        "ds_read_b128 v[72:75], %[ad] offset:224\n"
        "ds_read_b128 v[76:79], %[ad] offset:240\n"
        "v_add_u32 %[ad], 128, %[ad]\n"
        "s_sub_u32 %[st], %[st], 1\n"
        "s_cmp_lg_u32 %[st], 0\n"
        "s_cbranch_scc1 1b\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [ad] "+v"(addr), [st] "+s"(st)
        :
        : "memory", "scc", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79");
  }
  for (int j = nfull; j < ce; ++j) acc = acc + src[j];
}
constexpr int kAggT = 256;
constexpr int kAggPer = 4;                  // members per thread per chunk
constexpr int kAggCh = kAggT * kAggPer;     // chunk = 1024 members, list order r-major


__global__ __launch_bounds__(kAggT) __attribute__((amdgpu_waves_per_eu(kAggWpe, 8))) void aggregate_kernel(AggArgs a) {
  // conf, cons, cons*conf of the chunk's valid members; 16-B aligned rows padded by 16 doubles:
  // agg_chain_asm's ds_read_b128 batches read up to 16 terms past last_cnt (never added)
  __shared__ __attribute__((aligned(16))) double sV[3][kAggCh + 16];
  __shared__ int sWave[kAggPer][kAggT / 64];
  __shared__ int sHist[256];
  __shared__ int sWsum[kAggT / 64];
  __shared__ unsigned long long sVotes;
  __shared__ double sTot[3];
  __shared__ uint64_t sPrefix;
  __shared__ int64_t sRank;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    const int64_t b = a.goff[g], e = a.goff[g + 1];
    // software pipeline: member indices one chunk ahead of the gathers, gathers one chunk
    // ahead of the compaction, so the ordered chains run while the next chunk is in flight
    auto load_idx = [&](int64_t c0, int64_t* id) {
#pragma unroll
      for (int r = 0; r < kAggPer; ++r) {
        const int64_t i = c0 + r * kAggT + t;
        id[r] = (i < e) ? a.members[i] : -1;
      }
    };
    bool v[kAggPer];
    double x[kAggPer], c[kAggPer];
    auto gather = [&](const int64_t* id) {
#pragma unroll
      for (int r = 0; r < kAggPer; ++r) {
        const int64_t m = id[r];
        const bool in = m >= 0 && m < a.n_markets;
        v[r] = in && a.has[m] != 0;
        x[r] = in ? a.cons[m] : 0.0;
        c[r] = in ? a.conf[m] : 0.0;
      }
    };
    int64_t idn[kAggPer];
    load_idx(b, idn);
    gather(idn);
    load_idx(b + kAggCh, idn);
    double chain = 0.0;  // lanes 0..2 of wave 0: sum(conf), sum(cons), sum(cons*conf)
    int64_t k = 0;
    int last_cnt = 0;
    if (t == 0) sVotes = 0;
    for (int64_t c0 = b; c0 < e; c0 += kAggCh) {
      unsigned long long msk[kAggPer];
      unsigned votes = 0;
#pragma unroll
      for (int r = 0; r < kAggPer; ++r) {
        msk[r] = ballot(v[r]);
        if (lane == 0) sWave[r][w] = __popcll(msk[r]);
        votes += __popcll(ballot(v[r] && x[r] >= 0.5));  // market.py:400
      }
      __syncthreads();
      int run = 0;
#pragma unroll
      for (int r = 0; r < kAggPer; ++r) {
        int before = run;
#pragma unroll
        for (int q = 0; q < kAggT / 64; ++q) before += (q < w) ? sWave[r][q] : 0;
        if (v[r]) {
          const int pos = before + __popcll(msk[r] & lt);
          sV[0][pos] = c[r];
          sV[1][pos] = x[r];
          sV[2][pos] = x[r] * c[r];  // market.py:391
        }
#pragma unroll
        for (int q = 0; q < kAggT / 64; ++q) run += sWave[r][q];
      }
      const int cnt = run;
      if (lane == 0 && votes) atomicAdd(&sVotes, (unsigned long long)votes);
      __syncthreads();
      if (kAggChainAsm && c0 + kAggCh >= e) {  // the last chunk: its chains after the loop
        k += cnt;
        last_cnt = cnt;
        break;
      }
      gather(idn);                     // next chunk in flight during the chains
      load_idx(c0 + 2 * kAggCh, idn);
      if (t < 3) {
        const double* vv = sV[t];
        int j = 0;
        for (; j + 8 <= cnt; j += 8) {
          double q8[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) q8[q] = vv[j + q];
#pragma unroll
          for (int q = 0; q < 8; ++q) chain = chain + q8[q];
        }
        for (; j < cnt; ++j) chain = chain + vv[j];
      }
      k += cnt;
      __syncthreads();  // chunk buffer reused
    }
    if (kAggChainAsm && t < 3 && last_cnt > 0) agg_chain_asm(chain, sV[t], last_cnt);
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
      // a group that fit in one chunk still has its valid consensus values in sV[1]
      const bool in_lds = (e - b) <= kAggCh;
      for (int pass = 0; pass < 8 && k > 0; ++pass) {
        const int sh = 56 - 8 * pass;
        sHist[t] = 0;
        __syncthreads();
        const uint64_t pre = sPrefix;
        const uint64_t pmask = (pass == 0) ? 0ull : (~0ull << (sh + 8));
        if (in_lds) {
          for (int j = t; j < (int)k; j += kAggT) {
            const uint64_t key = f64_key(sV[1][j]);
            if ((key & pmask) == pre) atomicAdd(&sHist[(key >> sh) & 255], 1);
          }
        } else {
          for (int64_t i = b + t; i < e; i += kAggT) {
            const int64_t m = a.members[i];
            if (m >= 0 && m < a.n_markets && a.has[m]) {
              const uint64_t key = f64_key(a.cons[m]);
              if ((key & pmask) == pre) atomicAdd(&sHist[(key >> sh) & 255], 1);
            }
          }
        }
        __syncthreads();
        // bin holding rank r: block-wide inclusive scan of the 256 bin counts
        const int hv = sHist[t];
        int inc = hv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(inc, o);
          if (lane >= o) inc += y;
        }
        if (lane == 63) sWsum[w] = inc;
        const int64_t r = sRank;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kAggT / 64; ++q) inc += (q < w) ? sWsum[q] : 0;
        const int exc = inc - hv;
        if ((int64_t)exc <= r && r < (int64_t)inc) {  // exactly one bin
          sRank = r - exc;
          sPrefix = pre | ((uint64_t)t << sh);
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
  const int64_t cap = (int64_t)1 << 30;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)grid), dim3(kAggT), 0, as_stream(stream), a);
  return check_launch("aggregate_kernel");
}
