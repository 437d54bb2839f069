// gather_probe.hip -- what the per-signal relconf gather costs next to the C2 stream
// (experiment tooling, not product code).
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/bin/gather_probe
//
// Each thread owns 4 consecutive signals of the 1M x 32 workload: reads sid (16 B) and
// prob (32 B), optionally gathers the 4 table rows {rel, conf} (16 B each, random over
// S = 10k sources), writes usid (16 B), weight and nweight (32 B each).  Variants:
//   mix          stream only (the C2 byte mix without per-market outputs)
//   mix_g        + one 16-B gather per signal from the 160 KB table in global memory
//   mix_g8       + one 8-B gather per signal (rel only, 80 KB table)
//   mix_lds      + one 16-B gather per signal from the table staged in LDS (160 KB)
//   g_only       gathers only (sid stream in, one 8-B sum per thread out)
//   g_lds_only   LDS gathers only
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int S = 10000;

template <int MODE>  // 0 stream, 1 global16, 2 global8, 3 lds16
__global__ __launch_bounds__(1024) void mix(const int4* __restrict__ sid, const double4* __restrict__ prob,
                                             const double2* __restrict__ tab, int4* __restrict__ usid,
                                             double4* __restrict__ w, double4* __restrict__ nw, int64_t n4) {
  extern __shared__ double2 sT[];
  if (MODE == 3) {
    for (int i = threadIdx.x; i < S; i += blockDim.x) sT[i] = tab[i];
    __syncthreads();
  }
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = g; i < n4; i += st) {
    const int4 s = sid[i];
    const double4 p = prob[i];
    double4 a = p, b = p;
    if (MODE == 1 || MODE == 3) {
      double2 t0, t1, t2, t3;
      if (MODE == 1) { t0 = tab[s.x]; t1 = tab[s.y]; t2 = tab[s.z]; t3 = tab[s.w]; }
      else { t0 = sT[s.x]; t1 = sT[s.y]; t2 = sT[s.z]; t3 = sT[s.w]; }
      a = make_double4(t0.x * p.x, t1.x * p.y, t2.x * p.z, t3.x * p.w);
      b = make_double4(t0.y, t1.y, t2.y, t3.y);
    } else if (MODE == 2) {
      const double* t = reinterpret_cast<const double*>(tab);
      a = make_double4(t[s.x] * p.x, t[s.y] * p.y, t[s.z] * p.z, t[s.w] * p.w);
    }
    usid[i] = s;
    w[i] = a;
    nw[i] = b;
  }
}

template <int MODE>  // 1 global16, 3 lds16
__global__ __launch_bounds__(1024) void gonly(const int4* __restrict__ sid, const double2* __restrict__ tab,
                                               double* __restrict__ out, int64_t n4) {
  extern __shared__ double2 sT[];
  if (MODE == 3) {
    for (int i = threadIdx.x; i < S; i += blockDim.x) sT[i] = tab[i];
    __syncthreads();
  }
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  double acc = 0;
  for (int64_t i = g; i < n4; i += st) {
    const int4 s = sid[i];
    double2 t0, t1, t2, t3;
    if (MODE == 1) { t0 = tab[s.x]; t1 = tab[s.y]; t2 = tab[s.z]; t3 = tab[s.w]; }
    else { t0 = sT[s.x]; t1 = sT[s.y]; t2 = sT[s.z]; t3 = sT[s.w]; }
    acc += t0.x * t0.y + t1.x * t1.y + t2.x * t2.y + t3.x * t3.y;
  }
  if (acc == 1234.5) out[0] = acc;
}

int main() {
  const int64_t M = 1000000, L = 32, N = M * L, n4 = N / 4;
  std::vector<int> hs(N);
  srand(2);
  for (auto& x : hs) x = rand() % S;
  std::vector<double> ht(2 * S);
  for (auto& x : ht) x = (double)rand() / RAND_MAX;
  int4* sid; double4* prob; double2* tab; int4* usid; double4 *w, *nw; double* out;
  CK(hipMalloc(&sid, N * 4)); CK(hipMalloc(&prob, N * 8)); CK(hipMalloc(&tab, S * 16));
  CK(hipMalloc(&usid, N * 4)); CK(hipMalloc(&w, N * 8)); CK(hipMalloc(&nw, N * 8)); CK(hipMalloc(&out, 64));
  CK(hipMemcpy(sid, hs.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemset(prob, 0, N * 8));
  CK(hipMemcpy(tab, ht.data(), S * 16, hipMemcpyHostToDevice));
  const size_t lds = S * 16;
  CK(hipFuncSetAttribute((const void*)mix<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)gonly<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 32.0 * N;  // 12 in + 20 out per signal
  auto timeit = [&](const char* name, double b, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const int K = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < K; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= K;
    printf("{\"kernel\": \"%s\", \"ms\": %.5f, \"GBps\": %.1f}\n", name, ms, b / ms / 1e6);
    fflush(stdout);
  };
  for (int nt : {256, 512, 1024}) {
    char nm[96];
    const int per = (nt == 1024) ? 2 : (nt == 512) ? 4 : 8;
    const int grid = 256 * per;
    snprintf(nm, 96, "mix nt%d", nt); timeit(nm, bytes, [&] { mix<0><<<grid, nt>>>(sid, prob, tab, usid, w, nw, n4); });
    snprintf(nm, 96, "mix_g nt%d", nt); timeit(nm, bytes, [&] { mix<1><<<grid, nt>>>(sid, prob, tab, usid, w, nw, n4); });
    snprintf(nm, 96, "mix_g8 nt%d", nt); timeit(nm, bytes, [&] { mix<2><<<grid, nt>>>(sid, prob, tab, usid, w, nw, n4); });
    snprintf(nm, 96, "g_only nt%d", nt); timeit(nm, 4.0 * N, [&] { gonly<1><<<grid, nt>>>(sid, tab, out, n4); });
    // LDS table: one workgroup per CU
    snprintf(nm, 96, "mix_lds nt%d", nt); timeit(nm, bytes, [&] { mix<3><<<256, nt, lds>>>(sid, prob, tab, usid, w, nw, n4); });
    snprintf(nm, 96, "g_lds_only nt%d", nt); timeit(nm, 4.0 * N, [&] { gonly<3><<<256, nt, lds>>>(sid, tab, out, n4); });
  }
  return 0;
}
