// sol_c2.hip -- speed-of-light for the config-2 traffic mix (experiment tooling, not
// product code).  Streams exactly the bytes one consensus launch must move at 1M x 32
// (SURVEY d2): reads sid int32[N] + prob fp64[N] + offsets int64[M+1], writes usid
// int32[N] + weight/nweight fp64[N] + 3 fp64 + 2 int32 per market, with trivial compute,
// so its time is the achievable floor for that read/write mix on this box.
//   hipcc --offload-arch=gfx950 -O3 tools/sol_c2.hip -o tools/bin/sol_c2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct Bufs {
  const int4* sid; const int4* prob; const int4* off;
  int4* usid; int4* w; int4* nw; int4* cons; int4* conf; int4* tw; int4* nu; int4* err;
  int64_t n16_sid, n16_prob, n16_off, n16_m8, n16_m4;
};

typedef int v4i __attribute__((ext_vector_type(4)));
__device__ inline void nts(int4 v, int4* d) {
  v4i x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, (v4i*)d);
}

template <int NT, bool NTS>
__global__ __launch_bounds__(NT) void sol_mix(Bufs b) {
  // one grid-stride loop per array: each 16-B chunk of sid feeds usid, each of prob feeds
  // both weight and nweight (same byte ratio as the kernel: 12 B in, 20 B out per signal).
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x, st = (int64_t)gridDim.x * NT;
  for (int64_t i = g; i < b.n16_prob; i += st) {
    int4 p = b.prob[i];
    if (NTS) { nts(p, &b.w[i]); nts(p, &b.nw[i]); }
    else { b.w[i] = p; b.nw[i] = p; }
    if ((i & 1) == 0) {
      int4 s = b.sid[i >> 1];
      if (NTS) nts(s, &b.usid[i >> 1]); else b.usid[i >> 1] = s;
    }
  }
  for (int64_t i = g; i < b.n16_m8; i += st) {
    int4 o = b.off[i];
    b.cons[i] = o; b.conf[i] = o; b.tw[i] = o;
    if ((i & 1) == 0) { b.nu[i >> 1] = o; b.err[i >> 1] = o; }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void rd_only(Bufs b, int* sink) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x, st = (int64_t)gridDim.x * NT;
  int acc = 0;
  for (int64_t i = g; i < b.n16_prob; i += st) {
    int4 p = b.prob[i]; acc ^= p.x ^ p.w;
    if ((i & 1) == 0) { int4 s = b.sid[i >> 1]; acc ^= s.y; }
  }
  if (acc == 0x12345678) sink[0] = acc;
}

template <int NT>
__global__ __launch_bounds__(NT) void wr_only(Bufs b) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x, st = (int64_t)gridDim.x * NT;
  int4 z = make_int4(g, 1, 2, 3);
  for (int64_t i = g; i < b.n16_prob; i += st) {
    b.w[i] = z; b.nw[i] = z;
    if ((i & 1) == 0) b.usid[i >> 1] = z;
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void copy_k(const int4* a, int4* c, int64_t n16) {
  const int64_t g = (int64_t)blockIdx.x * NT + threadIdx.x, st = (int64_t)gridDim.x * NT;
  for (int64_t i = g; i < n16; i += st) c[i] = a[i];
}

int main(int argc, char** argv) {
  const int64_t M = 1000000, L = 32, N = M * L;
  Bufs b;
  void* p;
  auto alloc = [&](size_t bytes) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0, bytes)); return p; };
  b.sid = (const int4*)alloc(N * 4); b.prob = (const int4*)alloc(N * 8); b.off = (const int4*)alloc((M + 8) * 8);
  b.usid = (int4*)alloc(N * 4); b.w = (int4*)alloc(N * 8); b.nw = (int4*)alloc(N * 8);
  b.cons = (int4*)alloc(M * 8); b.conf = (int4*)alloc(M * 8); b.tw = (int4*)alloc(M * 8);
  b.nu = (int4*)alloc(M * 4); b.err = (int4*)alloc(M * 4);
  int* sink = (int*)alloc(64);
  b.n16_sid = N * 4 / 16; b.n16_prob = N * 8 / 16; b.n16_off = (M + 1) * 8 / 16;
  b.n16_m8 = M * 8 / 16; b.n16_m4 = M * 4 / 16;
  const double bytes_mix = 12.0 * N + 8.0 * (M + 1) + 32.0 * M + 20.0 * N;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    CK(hipDeviceSynchronize());
    const int K = 100;
    CK(hipEventRecord(e0));
    for (int i = 0; i < K; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= K;
    printf("{\"kernel\": \"%s\", \"ms\": %.5f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
  };
  for (int gpc : {4, 8, 16}) {
    int grid = 256 * gpc;
    char nm[64];
    snprintf(nm, 64, "mix_256x%d", gpc);
    timeit(nm, bytes_mix, [&] { sol_mix<256, false><<<grid, 256>>>(b); });
    snprintf(nm, 64, "mix_nt_256x%d", gpc);
    timeit(nm, bytes_mix, [&] { sol_mix<256, true><<<grid, 256>>>(b); });
    snprintf(nm, 64, "rd_256x%d", gpc);
    timeit(nm, 12.0 * N, [&] { rd_only<256><<<grid, 256>>>(b, sink); });
    snprintf(nm, 64, "wr_256x%d", gpc);
    timeit(nm, 20.0 * N, [&] { wr_only<256><<<grid, 256>>>(b); });
    snprintf(nm, 64, "copy_256x%d", gpc);
    timeit(nm, 16.0 * N, [&] { copy_k<256><<<grid, 256>>>(b.prob, b.w, b.n16_prob); });
  }
  return 0;
}
