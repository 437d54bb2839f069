// microbench.hip -- access-pattern rates that decide the consensus kernel's layout
// (experiment tooling, not product code).  hipcc --offload-arch=gfx950 -O3 tools/microbench.hip
//
//  gather16   lane-random 16-B loads from a 160 KB table (the relconf gather)
//  gather8    lane-random 8-B loads from the same table
//  coalx4     streaming 16-B loads, lanes contiguous (1 KiB per wave-instruction)
//  transx4    streaming 16-B loads, lane = row (rows of ROW bytes), chunk c per instruction
//  transdma   as transx4 but LDS-DMA (global_load_lds_dwordx4)
//  coaldma    as coalx4 but LDS-DMA
//  st_trans8  8-B stores, lane = row (row stride 256 B), slot j per instruction
//  st_coal8   8-B stores, lanes contiguous
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ __launch_bounds__(64) void gather16(const double2* tab, const int* idx, int64_t n_tiles, double* out) {
  const int lane = threadIdx.x;
  double acc = 0;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int* ip = idx + (t & 1023) * 2048 + lane * 32;
    int ids[32];
#pragma unroll
    for (int k = 0; k < 32; k += 4) { int4 v = *(const int4*)(ip + k); ids[k] = v.x; ids[k+1] = v.y; ids[k+2] = v.z; ids[k+3] = v.w; }
#pragma unroll
    for (int k = 0; k < 32; ++k) { double2 v = tab[ids[k]]; acc += v.x * v.y; }
  }
  if (acc == 12345.0) out[0] = acc;
}

template <int AUX>
__global__ __launch_bounds__(64) void gather16_aux(const double2* tab, const int* idx, int64_t n_tiles, double* out) {
  const int lane = threadIdx.x;
  double acc = 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)tab, 0, 10000 * 16, 0x00020000);
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int* ip = idx + (t & 1023) * 2048 + lane * 32;
    int ids[32];
#pragma unroll
    for (int k = 0; k < 32; k += 4) { int4 v = *(const int4*)(ip + k); ids[k] = v.x; ids[k+1] = v.y; ids[k+2] = v.z; ids[k+3] = v.w; }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, ids[k] * 16, 0, AUX);
      double2 d = *reinterpret_cast<double2*>(&v);
      acc += d.x * d.y;
    }
  }
  if (acc == 12345.0) out[0] = acc;
}

__global__ __launch_bounds__(64) void gather16_ntl(const double2* tab, const int* idx, int64_t n_tiles, double* out) {
  const int lane = threadIdx.x;
  double acc = 0;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int* ip = idx + (t & 1023) * 2048 + lane * 32;
    int ids[32];
#pragma unroll
    for (int k = 0; k < 32; k += 4) { int4 v = *(const int4*)(ip + k); ids[k] = v.x; ids[k+1] = v.y; ids[k+2] = v.z; ids[k+3] = v.w; }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const double x = __builtin_nontemporal_load(&tab[ids[k]].x);
      const double y = __builtin_nontemporal_load(&tab[ids[k]].y);
      acc += x * y;
    }
  }
  if (acc == 12345.0) out[0] = acc;
}

__global__ __launch_bounds__(64) void gather8(const double* tab, const int* idx, int64_t n_tiles, double* out) {
  const int lane = threadIdx.x;
  double acc = 0;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int* ip = idx + (t & 1023) * 2048 + lane * 32;
    int ids[32];
#pragma unroll
    for (int k = 0; k < 32; k += 4) { int4 v = *(const int4*)(ip + k); ids[k] = v.x; ids[k+1] = v.y; ids[k+2] = v.z; ids[k+3] = v.w; }
#pragma unroll
    for (int k = 0; k < 32; ++k) { acc += tab[ids[k]]; }
  }
  if (acc == 12345.0) out[0] = acc;
}

// tile = 64 rows of ROW bytes (contiguous 64*ROW bytes)
template <int ROW>
__global__ __launch_bounds__(64) void coalx4(const int4* src, int64_t n_tiles, int* out) {
  const int lane = threadIdx.x;
  int acc = 0;
  constexpr int NI = ROW * 64 / 1024;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int4* p = src + t * (ROW * 64 / 16);
    int4 v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = p[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < NI; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  if (acc == 0x12345) out[0] = acc;
}

template <int ROW>
__global__ __launch_bounds__(64) void transx4(const int4* src, int64_t n_tiles, int* out) {
  const int lane = threadIdx.x;
  int acc = 0;
  constexpr int NI = ROW / 16;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int4* p = src + t * (ROW * 64 / 16) + lane * (ROW / 16);
    int4 v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = p[i];
#pragma unroll
    for (int i = 0; i < NI; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  if (acc == 0x12345) out[0] = acc;
}

template <int ROW, bool TRANS>
__global__ __launch_bounds__(64) void dmax4(const int4* src, int64_t n_tiles, int* out) {
  __shared__ int4 buf[ROW * 64 / 16];
  const int lane = threadIdx.x;
  int acc = 0;
  constexpr int NI = ROW * 64 / 1024;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int4* p = src + t * (ROW * 64 / 16);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int4* g = TRANS ? p + lane * (ROW / 16) + i : p + i * 64 + lane;
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(buf + i * 64), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int4 v = buf[lane * 3 % (ROW * 4)];
    acc ^= v.x;
    __builtin_amdgcn_s_barrier();
  }
  if (acc == 0x12345) out[0] = acc;
}

template <bool TRANS>
__global__ __launch_bounds__(64) void st8(double* dst, int64_t n_tiles) {
  const int lane = threadIdx.x;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    double* p = dst + t * 2048;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (TRANS) p[lane * 32 + j] = (double)j;
      else p[j * 64 + lane] = (double)j;
    }
  }
}

int main() {
  int dev = 0;
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, dev));
  const int cus = pr.multiProcessorCount;
  const int64_t S = 10000;
  double2* tab;
  int* idx;
  CK(hipMalloc(&tab, S * 16));
  CK(hipMemset(tab, 0, S * 16));
  std::vector<int> hidx(1024 * 2048);
  srand(1);
  for (auto& x : hidx) x = rand() % S;
  CK(hipMalloc(&idx, hidx.size() * 4));
  CK(hipMemcpy(idx, hidx.data(), hidx.size() * 4, hipMemcpyHostToDevice));
  const int64_t big = 1ll << 30;  // 1 GiB
  void *src, *dst;
  CK(hipMalloc(&src, big));
  CK(hipMalloc(&dst, big));
  CK(hipMemset(src, 1, big));
  double* dout;
  CK(hipMalloc(&dout, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double bytes, double instrs) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 10;
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double s = ms / 1e3 / R;
    const double cyc = s * 2.4e9;
    printf("%-28s %8.3f ms  %8.1f GB/s  %7.2f cyc/wave-instr/CU\n", name, s * 1e3, bytes / s / 1e9,
           cyc * cus / instrs);
  };
  for (int occ : {8}) {
    const int grid = cus * occ;
    const int64_t tiles = 200000;
    char nm[64];
    snprintf(nm, 64, "gather16 occ%d", occ);
    timeit(nm, [&] { gather16<<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 32.0);
    snprintf(nm, 64, "gather16_buf aux0 occ%d", occ);
    timeit(nm, [&] { gather16_aux<0><<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 32.0);
    snprintf(nm, 64, "gather16_buf aux1(glc) occ%d", occ);
    timeit(nm, [&] { gather16_aux<1><<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 32.0);
    snprintf(nm, 64, "gather16_buf aux2(slc) occ%d", occ);
    timeit(nm, [&] { gather16_aux<2><<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 32.0);
    snprintf(nm, 64, "gather16_buf aux3 occ%d", occ);
    timeit(nm, [&] { gather16_aux<3><<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 32.0);
    snprintf(nm, 64, "gather16_nt occ%d", occ);
    timeit(nm, [&] { gather16_ntl<<<grid, 64>>>(tab, idx, tiles, dout); }, tiles * 2048.0 * 16, tiles * 64.0);
    snprintf(nm, 64, "gather8 occ%d", occ);
    timeit(nm, [&] { gather8<<<grid, 64>>>((const double*)tab, idx, tiles, dout); }, tiles * 2048.0 * 8, tiles * 32.0);
  }
  return 0;
}
