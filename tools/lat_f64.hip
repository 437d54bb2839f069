// lat_f64.hip -- dependent-chain latency of v_add_f64 on one wave (experiment tooling).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void chain(double* out, double y, int iters, long long* cyc) {
  double x = threadIdx.x;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x = x + y;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void chain3(double* out, double y, int iters, long long* cyc) {  // 3 independent chains per lane
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) { x0 = x0 + y; x1 = x1 + y; x2 = x2 + y; }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = x0 + x1 + x2;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* o; long long* c; hipMalloc(&o, 64 * 8); hipMalloc(&c, 8);
  long long h;
  const int it = 10000;
  chain<<<1, 64>>>(o, 1e-9, it, c); hipDeviceSynchronize();
  chain<<<1, 64>>>(o, 1e-9, it, c); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("v_add_f64 dependent: %.2f cyc/add\n", (double)h / (it * 16.0));
  chain3<<<1, 64>>>(o, 1e-9, it, c); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("3 chains/lane:       %.2f cyc/element (3 adds)\n", (double)h / (it * 16.0));
  return 0;
}
