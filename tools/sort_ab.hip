// Sort A/B for the C3 wide kernel (verdict r04 item 1), not product code: 4096-key blocks
// (one workgroup of 8 waves per block, R = 8 keys per thread) sorted by
//   bitonic  the shipped register network, consensus_wide.hip wide_sort<8, 8, 8> (keys
//            sid << 12 | i, striped input i = c*NT + t, blocked output q = t*R + r), and
//   radix    a stable LSD radix sort of the same keys on the sid bits only (the index bits
//            ride along), 4-bit digits, per-thread packed 16-bit digit counters in LDS
//            (ds_add_rtn on the thread's own column: ranks in input order without atomics
//            contention), a raking exclusive scan over [digit][thread], scatter, blocked
//            read-back -- ceil(sid_bits / 4) passes.
// Keys: sids Zipf(1.1) over S (a random permutation of ranks, as make_c3), i = position.
// Both outputs are compared word for word; prints ms per 100M keys for each.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics \
//         -I bayesian-consensus-engine_amd/csrc -c tools/sort_ab.hip -o /tmp/sort_ab.o
//   hipcc --offload-arch=gfx950 /tmp/sort_ab.o bayesian-consensus-engine_amd/lib/obj/capi.o -o tools/bin/sort_ab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "consensus_wide.hip"

using namespace bce;

constexpr int NW = 8, R = 8, NT = 64 * NW, P = NT * R, IB = 12;

__global__ __launch_bounds__(NT) void bitonic_bench(const unsigned* in, unsigned* out, int nblocks) {
  __shared__ __attribute__((aligned(16))) unsigned sX[2 * NT * R];
  const int t = threadIdx.x, lane = lane_id();
  for (int b = blockIdx.x; b < nblocks; b += gridDim.x) {
    unsigned key[R];
#pragma unroll
    for (int c = 0; c < R; ++c) key[c] = in[(size_t)b * P + c * NT + t];  // striped, as wide_load
    wide_sort<NW, NW, R>(key, sX, t, lane);
#pragma unroll
    for (int r = 0; r < R; r += 4)
      *reinterpret_cast<uint4*>(out + (size_t)b * P + t * R + r) = make_uint4(key[r], key[r + 1], key[r + 2], key[r + 3]);
    __syncthreads();
  }
}

template <int PASSES>
__global__ __launch_bounds__(NT) void radix_bench(const unsigned* in, unsigned* out, int nblocks) {
  __shared__ __attribute__((aligned(16))) unsigned cnt[8 * NT];  // [w][t]: digits w (lo half), w + 8 (hi half)
  __shared__ __attribute__((aligned(16))) unsigned sK[P];
  __shared__ unsigned wsum[NW];
  const int t = threadIdx.x, lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  for (int b = blockIdx.x; b < nblocks; b += gridDim.x) {
    unsigned key[R];
    // blocked order i = t*R + r is the stable order; the striped input is transposed through LDS
    // (the product would load blocked directly)
#pragma unroll
    for (int c = 0; c < R; ++c) sK[c * NT + t] = in[(size_t)b * P + c * NT + t];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(sK + t * R + r);
      key[r] = v.x; key[r + 1] = v.y; key[r + 2] = v.z; key[r + 3] = v.w;
    }
#pragma unroll
    for (int pass = 0; pass < PASSES; ++pass) {
      const int sh = IB + 4 * pass;
#pragma unroll
      for (int w = 0; w < 8; ++w) cnt[w * NT + t] = 0;  // own column
      unsigned rk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const unsigned d = (key[r] >> sh) & 15u;
        const unsigned hs = (d >> 3) * 16u;
        const unsigned old = atomicAdd(&cnt[(d & 7u) * NT + t], 1u << hs);
        rk[r] = (old >> hs) & 0xffffu;
      }
      __syncthreads();
      // raking exclusive scan over memory order (w, t): thread t owns words 8t .. 8t+7
      uint4 v0 = *reinterpret_cast<const uint4*>(cnt + 8 * t), v1 = *reinterpret_cast<const uint4*>(cnt + 8 * t + 4);
      unsigned x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      unsigned s = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned y = x[k];
        x[k] = s;
        s += y;
      }
      const unsigned incl = (unsigned)wave_incl_scan((int)s);
      if (lane == 63) wsum[wv] = incl;
      __syncthreads();
      unsigned pre = incl - s, tot = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const unsigned ws = wsum[w];
        pre += (w < wv) ? ws : 0u;
        tot += ws;
      }
      *reinterpret_cast<uint4*>(cnt + 8 * t) = make_uint4(x[0] + pre, x[1] + pre, x[2] + pre, x[3] + pre);
      *reinterpret_cast<uint4*>(cnt + 8 * t + 4) = make_uint4(x[4] + pre, x[5] + pre, x[6] + pre, x[7] + pre);
      __syncthreads();
      const unsigned tlo = tot & 0xffffu;  // keys with a digit 0..7
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const unsigned d = (key[r] >> sh) & 15u;
        const unsigned wd = cnt[(d & 7u) * NT + t];
        const unsigned base = (d < 8u) ? (wd & 0xffffu) : ((wd >> 16) + tlo);
        sK[base + rk[r]] = key[r];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; r += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(sK + t * R + r);
        key[r] = v.x; key[r + 1] = v.y; key[r + 2] = v.z; key[r + 3] = v.w;
      }
      __syncthreads();  // sK and cnt are rewritten by the next pass / block
    }
#pragma unroll
    for (int r = 0; r < R; r += 4)
      *reinterpret_cast<uint4*>(out + (size_t)b * P + t * R + r) = make_uint4(key[r], key[r + 1], key[r + 2], key[r + 3]);
  }
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                       \
    }                                                                 \
  } while (0)

template <class K>
static float time_kernel(K launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int nblocks = argc > 1 ? atoi(argv[1]) : 24414;  // ~100M keys
  const int S = argc > 2 ? atoi(argv[2]) : 1000000;
  const size_t N = (size_t)nblocks * P;
  std::mt19937_64 rng(3);
  std::vector<unsigned> perm(S);
  for (int i = 0; i < S; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  // Zipf(1.1) over S by inverse CDF on a table
  std::vector<double> cdf(S);
  double acc = 0;
  for (int k = 0; k < S; ++k) cdf[k] = (acc += std::pow(k + 1.0, -1.1));
  std::uniform_real_distribution<double> U(0.0, acc);
  std::vector<unsigned> h(N);
  for (size_t j = 0; j < N; ++j) {
    const int k = (int)(std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin());
    const unsigned sid = perm[std::min(k, S - 1)];
    const unsigned i = (unsigned)(j % P);
    h[j] = (sid << IB) | i;
  }
  int sid_bits = 0;
  while ((1 << sid_bits) < S) ++sid_bits;
  const int passes = (sid_bits + 3) / 4;
  unsigned *din, *d1, *d2;
  CK(hipMalloc(&din, N * 4));
  CK(hipMalloc(&d1, N * 4));
  CK(hipMalloc(&d2, N * 4));
  CK(hipMemcpy(din, h.data(), N * 4, hipMemcpyHostToDevice));
  int dev = 0, cus = 0, bpc_b = 0, bpc_r = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc_b, bitonic_bench, NT, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc_r, radix_bench<5>, NT, 0));
  const int gb = std::min(nblocks, cus * bpc_b), gr = std::min(nblocks, cus * bpc_r);
  auto lb = [&]() { hipLaunchKernelGGL(bitonic_bench, dim3(gb), dim3(NT), 0, 0, din, d1, nblocks); };
  auto lr = [&]() {
    if (passes <= 5) hipLaunchKernelGGL(radix_bench<5>, dim3(gr), dim3(NT), 0, 0, din, d2, nblocks);
    else hipLaunchKernelGGL(radix_bench<6>, dim3(gr), dim3(NT), 0, 0, din, d2, nblocks);
  };
  const float tb = time_kernel(lb, 20), tr = time_kernel(lr, 20);
  CK(hipDeviceSynchronize());
  std::vector<unsigned> o1(N), o2(N);
  CK(hipMemcpy(o1.data(), d1, N * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o2.data(), d2, N * 4, hipMemcpyDeviceToHost));
  size_t diff = 0;
  for (size_t j = 0; j < N; ++j) diff += o1[j] != o2[j];
  bool sorted = true;
  for (size_t b = 0; b < (size_t)nblocks && sorted; ++b)
    sorted = std::is_sorted(o1.begin() + b * P, o1.begin() + (b + 1) * P);
  const double scale = 1e8 / (double)N;
  printf("{\"keys\": %zu, \"sources\": %d, \"sid_bits\": %d, \"radix_passes\": %d, \"blocks_per_cu\": [%d, %d], "
         "\"bitonic_ms_per_1e8\": %.4f, \"radix_ms_per_1e8\": %.4f, \"outputs_differ\": %zu, \"bitonic_sorted\": %s}\n",
         N, S, sid_bits, passes <= 5 ? 5 : 6, bpc_b, bpc_r, tb * scale, tr * scale, diff, sorted ? "true" : "false");
  return diff == 0 && sorted ? 0 : 2;
}
