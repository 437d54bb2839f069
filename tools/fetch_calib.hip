// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE on gfx950 for the access shapes the
// consensus kernels use (experiment tooling, not product code).
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/bin/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/bin/fetch_calib
//
// MI355X_MICROARCH.md documents FETCH_SIZE = 1/2 of the bytes of a wide coalesced
// streaming read; random 16-B gathers are "uncalibrated".  Each kernel here moves a known
// number of requests so FETCH_SIZE per request can be read off the counter file:
//   calib_stream      1 GiB read, 16 B per lane, coalesced              (known: 2^30 B)
//   calib_gather_big  2^24 random 16-B gathers from a 4 GiB table      (1 line each, no reuse)
//   calib_gather_mall 2^24 random 16-B gathers from a 16 MiB table     (C3's relconf table)
//   calib_gather_l2   2^24 random 16-B gathers from a 160 KB table     (C2's relconf table)
// Every kernel writes one double per thread (grid-sized, small) so nothing is optimised out.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void calib_stream(const double2* __restrict__ a, int64_t n2, double* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  double s = 0.0;
  for (int64_t i = g; i < n2; i += st) { const double2 v = a[i]; s += v.x + v.y; }
  out[g] = s;
}

template <int TAG>
__global__ __launch_bounds__(256) void calib_gather(const double2* __restrict__ tab, uint32_t rows, int64_t gathers,
                                                    double* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  double s = 0.0;
  for (int64_t i = g; i < gathers; i += st) {
    const uint32_t r = mix32((uint32_t)i * 2654435761U + TAG) % rows;
    const double2 v = tab[r];
    s += v.x + v.y;
  }
  out[g] = s;
}

int main() {
  const int64_t big = (int64_t)1 << 32;  // 4 GiB
  double2* tab;
  double* out;
  CK(hipMalloc(&tab, big));
  CK(hipMemset(tab, 0, big));
  const int grid = 256 * 8, block = 256;
  CK(hipMalloc(&out, (size_t)grid * block * sizeof(double)));
  const int64_t gathers = (int64_t)1 << 24;
  for (int rep = 0; rep < 3; ++rep) {
    calib_stream<<<grid, block>>>(tab, ((int64_t)1 << 30) / 16, out);
    calib_gather<1><<<grid, block>>>(tab, (uint32_t)(big / 16), gathers, out);
    calib_gather<2><<<grid, block>>>(tab, (16u << 20) / 16, gathers, out);
    calib_gather<3><<<grid, block>>>(tab, 10000, gathers, out);
  }
  CK(hipDeviceSynchronize());
  printf("fetch_calib: stream 2^30 B; gathers 2^24 x 16 B (big / 16 MiB / 160 KB tables), 3 reps\n");
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
