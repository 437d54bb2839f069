// c5_probe.hip -- config-5 pass-1 access-shape probe (experiment tooling, not product code).
// Times the single-read re-estimation pass (agent-major P [A][M] fp64, lane per market
// column, agent-order sums + one vote bit per cell) in several shapes on a 16k x 1M P:
//   CPL   market columns per lane (1: 8-B loads, 512 B per wave-instruction; 2: 16-B loads,
//         1 KB, vote words split into even/odd columns of a 128-column group)
//   ROWS  agent rows loaded per step (loads in flight per wave)
//   NT    nontemporal loads of P
// Every variant's consensus must be bit-identical (same agent order per column).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/c5_probe.hip -o tools/bin/c5_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#pragma clang fp contract(off)

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

__global__ void fill(double* P, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    P[i] = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  }
}

template <int CPL, int ROWS, bool NT, bool SYNC = false, int MAP = 0, bool BLK = false>
__global__ __launch_bounds__(256) void votes_k(const double* __restrict__ P, int64_t A, int64_t M, int64_t ld,
                                               const double* __restrict__ w, double* __restrict__ cons,
                                               unsigned long long* __restrict__ vbits) {
  const int lane = threadIdx.x & 63;
  // wave group of 64*CPL columns; MAP 1: wave-major (group = wave * grid + block), MAP 2:
  // consecutive groups on one XCD (blockIdx % 8), MAP 0: block-major
  const int64_t G = gridDim.x;
  const int64_t g = MAP == 1 ? (int64_t)(threadIdx.x >> 6) * G + blockIdx.x
                  : MAP == 2 ? (int64_t)(((blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3)) * 4 + (threadIdx.x >> 6))
                             : (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t c0 = g * 64 * CPL;
  if (!SYNC && c0 >= M) return;
  const int64_t m = c0 + lane * CPL;
  const bool in = m + CPL - 1 < M;
  // BLK: column-blocked layout, block g of 64*CPL columns is one contiguous [A][64*CPL]
  // slab, so a wave's rows are adjacent (8 KB per 16 rows) instead of ld*8 bytes apart
  const double* col = BLK ? P + (in ? g * A * 64 * CPL + lane * CPL : 0) : P + (in ? m : 0);
  const int64_t rs = BLK ? 64 * CPL : ld;
  unsigned long long* vb = vbits + g * CPL * A;
  double ws[CPL], total = 0.0;
#pragma unroll
  for (int e = 0; e < CPL; ++e) ws[e] = 0.0;
  for (int64_t a = 0; a + ROWS <= A; a += ROWS) {
    double v[ROWS][CPL];
#pragma unroll
    for (int q = 0; q < ROWS; ++q) {
      const double* src = col + (a + q) * rs;
      if constexpr (CPL == 2 || CPL == 4) {
#pragma unroll
        for (int h = 0; h < CPL / 2; ++h) {
          d2v x = NT ? __builtin_nontemporal_load(reinterpret_cast<const d2v*>(src) + h) : reinterpret_cast<const d2v*>(src)[h];
          v[q][2 * h] = x.x; v[q][2 * h + 1] = x.y;
        }
      } else {
        v[q][0] = NT ? __builtin_nontemporal_load(src) : *src;
      }
    }
    unsigned long long mine[CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) mine[e] = 0;
#pragma unroll
    for (int q = 0; q < ROWS; ++q) {
      const double wq = w[a + q];
      total += wq;
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        ws[e] += (0.0 + v[q][e]) * wq;
        const unsigned long long b = __ballot(in && v[q][e] >= 0.5);
        mine[e] = (lane == q) ? b : mine[e];
      }
    }
    if (lane < ROWS && c0 < M) {
#pragma unroll
      for (int e = 0; e < CPL; ++e) vb[e * A + a + lane] = mine[e];
    }
    if (SYNC) __syncthreads();
  }
  if (in) {
#pragma unroll
    for (int e = 0; e < CPL; ++e) cons[m + e] = total == 0.0 ? 0.0 : ws[e] / total;
  }
}

// Row-band sweep: one launch per band of B agent rows, every wave of the chip in the same
// band, each column's running sum carried in HBM between bands (ws[M] read + written per
// band) -- the chip-wide access front stays B rows deep instead of drifting apart.
template <int ROWS>
__global__ __launch_bounds__(256) void band_k(const double* __restrict__ P, int64_t A, int64_t M, int64_t ld,
                                              const double* __restrict__ w, double* __restrict__ wsb,
                                              unsigned long long* __restrict__ vbits, int64_t a0, int64_t B) {
  const int lane = threadIdx.x & 63;
  const int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t g = m >> 6;
  if ((g << 6) >= M) return;
  const bool in = m < M;
  const double* col = P + (in ? m : 0);
  unsigned long long* vb = vbits + g * A;
  double ws = (a0 == 0 || !in) ? 0.0 : wsb[m];
  for (int64_t a = a0; a < a0 + B; a += ROWS) {
    double v[ROWS];
#pragma unroll
    for (int q = 0; q < ROWS; ++q) v[q] = in ? col[(a + q) * ld] : 0.0;
    unsigned long long mine = 0;
#pragma unroll
    for (int q = 0; q < ROWS; ++q) {
      ws += (0.0 + v[q]) * w[a + q];
      const unsigned long long b = __ballot(in && v[q] >= 0.5);
      mine = (lane == q) ? b : mine;
    }
    if (lane < ROWS) vb[a + lane] = mine;
  }
  if (in) wsb[m] = ws;
}

int main(int argc, char** argv) {
  const int64_t A = 16384, M = 1000000, ld = M;
  double *P, *w, *cons, *ref;
  unsigned long long* vb;
  CK(hipMalloc(&P, (A * M + A * 128) * 8));  // + one 128-column slab: the blocked layout's last partial block
  CK(hipMalloc(&w, A * 8));
  CK(hipMalloc(&cons, M * 8));
  CK(hipMalloc(&ref, M * 8));
  CK(hipMalloc(&vb, ((M + 127) / 128) * 2 * A * 8));
  fill<<<4096, 256>>>(P, A * M + A * 128);
  double* hw = (double*)malloc(A * 8);
  for (int64_t i = 0; i < A; ++i) hw[i] = (i % 7 == 0) ? 0.25 : 0.5;
  CK(hipMemcpy(w, hw, A * 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 8.0 * A * M;
  bool have_ref = false;
  double* h1 = (double*)malloc(M * 8);
  double* h2 = (double*)malloc(M * 8);
  auto run = [&](const char* name, int cpl, auto launch) {
    const int reps = 4;
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best; sum += ms;
    }
    bool same = true;
    if (!have_ref) { CK(hipMemcpy(ref, cons, M * 8, hipMemcpyDeviceToDevice)); have_ref = true; }
    else {
      CK(hipMemcpy(h1, ref, M * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2, cons, M * 8, hipMemcpyDeviceToHost));
      same = memcmp(h1, h2, M * 8) == 0;
    }
    printf("{\"variant\": \"%s\", \"best_ms\": %.3f, \"mean_ms\": %.3f, \"TBps\": %.3f, \"frac\": %.3f, \"same_cons\": %s}\n",
           name, best, sum / reps, bytes / best / 1e9, bytes / best / 1e9 / 8.0, same ? "true" : "false");
    fflush(stdout);
    (void)cpl;
  };
#define V(C, R, N, S, MP, B)                                                                            \
  run("cpl" #C "_rows" #R "_nt" #N "_map" #MP "_blk" #B, C, [&] {                                      \
    const int64_t groups = (M + 64 * C - 1) / (64 * C);                                                 \
    votes_k<C, R, N, S, MP, B><<<(unsigned)(((groups + 3) / 4 + 7) & ~7), 256>>>(P, A, M, ld, w, cons, vb); \
  })
  double* wsb;
  CK(hipMalloc(&wsb, M * 8));
  for (int64_t B : {64, 256, 1024}) {
    for (int round = 0; round < 2; ++round) {
      const int reps = 3;
      float best = 1e30f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        for (int64_t a0 = 0; a0 < A; a0 += B)
          band_k<16><<<(unsigned)((M + 255) / 256), 256>>>(P, A, M, ld, w, wsb, vb, a0, B);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      printf("{\"variant\": \"band%lld_rows16\", \"best_ms\": %.3f, \"TBps\": %.3f, \"frac\": %.3f}\n", (long long)B, best,
             bytes / best / 1e9, bytes / best / 1e9 / 8.0);
      fflush(stdout);
    }
  }
  for (int round = 0; round < 2; ++round) {
    V(1, 16, 0, 0, 0, false);
    V(1, 16, 0, 0, 0, true);
  }
  return 0;
}
