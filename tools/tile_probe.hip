// tile_probe.hip -- the config-2 traffic of consensus_tab32_kernel with its occupancy and
// access shapes but trivial compute (experiment tooling, not product code).
//   hipcc --offload-arch=gfx950 -O3 tools/tile_probe.hip -o tools/bin/tile_probe
//
// One persistent workgroup of W waves per CU (the real kernel: W = 4, the LDS table takes
// the CU), a wave owns a tile of 64 consecutive markets x 32 signals and moves exactly its
// bytes: sid (4 B) + prob (8 B) in, usid (4 B) + weight + nweight (8 + 8 B) out per
// signal, 3 fp64 + 2 int32 per market.  Shapes:
//   piece64   the kernel's: four consecutive lanes cover one contiguous 64-B piece of a
//             market's row, 16 markets per instruction
//   row128    eight lanes cover a whole 128-B sid row / 256-B prob row piece
//   linear    lane-linear: an instruction covers 1 KiB contiguous (ignores market rows)
// and optionally the next tile's loads issued before this tile's stores (PREF).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct Args {
  const uint32_t* sid; const double* prob;
  uint32_t* usid; double* w; double* nw;
  double* cons; double* conf; double* tw; int* nu; int* err;
  int64_t M;
};

// SHAPE: 0 piece64, 1 row128, 2 linear, 3 half-row 128-B pieces for probs too
typedef unsigned u4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint32_t* p) {
  if (NT) { const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p)); return make_uint4(v.x, v.y, v.z, v.w); }
  return *reinterpret_cast<const uint4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16(uint32_t* p, uint4 v) {
  if (NT) { const u4v x = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(x, reinterpret_cast<u4v*>(p)); }
  else *reinterpret_cast<uint4*>(p) = v;
}
template <int SHAPE, bool NT = false>
__device__ __forceinline__ void tile_load(const Args& a, int64_t B, int lane_in, uint4 (&s)[8], uint4 (&p)[16]) {
  // SHAPE 4 = SHAPE 3's addresses, lanes permuted (bits 0-2 <-> 3-5): a 128-B piece is
  // read by lanes m, m+8, ..., m+56 instead of 8 consecutive lanes
  const int lane = (SHAPE == 4) ? (((lane_in & 7) << 3) | (lane_in >> 3)) : lane_in;
  constexpr int SH = (SHAPE == 4) ? 3 : SHAPE;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int64_t e;  // element (u32) offset of this lane's 16-B chunk
    if (SH == 0) e = 32 * (16 * (k & 3) + (lane >> 2)) + 16 * (k >> 2) + 4 * (lane & 3);
    else if (SH == 1 || SH == 3) e = 32 * (8 * k + (lane >> 3)) + 4 * (lane & 7);
    else e = 256 * k + 4 * lane;
    s[k] = ld16<NT>(a.sid + B + e);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int64_t e;  // element (u32 of the prob array viewed as u32) offset
    if (SH == 0) e = 64 * (16 * (k & 3) + (lane >> 2)) + 16 * (k >> 2) + 4 * (lane & 3);
    else if (SH == 1) e = 64 * (4 * k + (lane >> 4)) + 4 * (lane & 15);
    else if (SH == 3) e = 64 * (8 * (k & 7) + (lane >> 3)) + 32 * (k >> 3) + 4 * (lane & 7);
    else e = 256 * k + 4 * lane;
    p[k] = ld16<NT>(reinterpret_cast<const uint32_t*>(a.prob + B) + e);
  }
}

template <int W, int SHAPE, bool PF = false, bool NT = false, int MAP = 0>
__global__ __launch_bounds__(64 * W) void tile_mix(Args a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t n_tiles = a.M / 64;
  const int64_t stride = (int64_t)gridDim.x * W;
  uint4 sn[8], pn[16];
  // MAP 0: a workgroup's waves take consecutive tiles (the kernel's); 1: wave-major, so
  // consecutive tiles land on consecutive workgroups (and XCDs); 2: consecutive tiles on
  // the same XCD's workgroups (blockIdx % 8 = XCD)
  const int64_t G = gridDim.x;
  int64_t tile;
  if (MAP == 0) tile = (int64_t)blockIdx.x * W + wv;
  else if (MAP == 1) tile = (int64_t)wv * G + blockIdx.x;
  else if (MAP == 2) tile = (int64_t)(((blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3)) * W + wv);
  else {  // wave-major with chunks of C = MAP - 1 consecutive tiles on one XCD
    constexpr int C = MAP - 1;
    const int64_t x = blockIdx.x & 7, sl = blockIdx.x >> 3;
    tile = (int64_t)wv * G + ((sl / C) * 8 + x) * C + (sl % C);
  }
  if (PF && tile < n_tiles) tile_load<SHAPE, NT>(a, tile * 64 * 32, lane, sn, pn);
  for (; tile < n_tiles; tile += stride) {
    const int64_t B = tile * 64 * 32;  // first signal of the tile
    uint4 s[8];
    uint4 p[16];
    if (PF) {
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] = sn[k];
#pragma unroll
      for (int k = 0; k < 16; ++k) p[k] = pn[k];
      if (tile + stride < n_tiles) tile_load<SHAPE, NT>(a, (tile + stride) * 64 * 32, lane, sn, pn);
    } else {
      tile_load<SHAPE, NT>(a, B, lane, s, p);
    }
    // trivial compute: fold so nothing is dead
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= s[k].x ^ s[k].w;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += p[k].y;
    // per-market outputs (lane = market)
    const int64_t mk = tile * 64 + lane;
    a.cons[mk] = (double)acc;
    a.conf[mk] = (double)lane;
    a.tw[mk] = 1.0;
    a.nu[mk] = 32;
    a.err[mk] = -1;
    // per-unique outputs: usid 8 KiB, weight 16 KiB, nweight 16 KiB per tile
    const int lane_o = lane;
    const int lane_s = (SHAPE == 4) ? (((lane_o & 7) << 3) | (lane_o >> 3)) : lane_o;
    constexpr int SS = (SHAPE == 4) ? 3 : SHAPE;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int64_t e;
      if (SS == 0) e = 32 * (16 * (k & 3) + (lane_s >> 2)) + 16 * (k >> 2) + 4 * (lane_s & 3);
      else if (SS == 1 || SS == 3) e = 32 * (8 * k + (lane_s >> 3)) + 4 * (lane_s & 7);
      else e = 256 * k + 4 * lane_s;
      st16<NT>(a.usid + B + e, s[k]);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      int64_t e;
      if (SS == 0) e = 64 * (16 * (k & 3) + (lane_s >> 2)) + 16 * (k >> 2) + 4 * (lane_s & 3);
      else if (SS == 1) e = 64 * (4 * k + (lane_s >> 4)) + 4 * (lane_s & 15);
      else if (SS == 3) e = 64 * (8 * (k & 7) + (lane_s >> 3)) + 32 * (k >> 3) + 4 * (lane_s & 7);
      else e = 256 * k + 4 * lane_s;
      st16<NT>(reinterpret_cast<uint32_t*>(a.w + B) + e, p[k]);
      st16<NT>(reinterpret_cast<uint32_t*>(a.nw + B) + e, p[k]);
    }
  }
}

int main() {
  const int64_t M = 1000000, N = M * 32;
  Args a;
  a.M = M;
  CK(hipMalloc((void**)&a.sid, N * 4)); CK(hipMalloc((void**)&a.prob, N * 8));
  CK(hipMalloc((void**)&a.usid, N * 4)); CK(hipMalloc((void**)&a.w, N * 8)); CK(hipMalloc((void**)&a.nw, N * 8));
  CK(hipMalloc((void**)&a.cons, M * 8)); CK(hipMalloc((void**)&a.conf, M * 8)); CK(hipMalloc((void**)&a.tw, M * 8));
  CK(hipMalloc((void**)&a.nu, M * 4)); CK(hipMalloc((void**)&a.err, M * 4));
  CK(hipMemset((void*)a.sid, 1, N * 4)); CK(hipMemset((void*)a.prob, 0, N * 8));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 32.0 * N + 32.0 * M;
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 50; ++i) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const int K = 100;
    CK(hipEventRecord(e0));
    for (int i = 0; i < K; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= K;
    printf("{\"probe\": \"%s\", \"ms\": %.5f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  // lane-permuted pieces (for VALU-only permlane transposes) vs the kernel's shape
  for (int r = 0; r < 3; ++r) {
    timeit("half128 w8 1wg/cu nt map1", [&] { tile_mix<8, 3, false, true, 1><<<cus, 512>>>(a); });
    timeit("half128-lanes-permuted w8 1wg/cu nt map1", [&] { tile_mix<8, 4, false, true, 1><<<cus, 512>>>(a); });
  }
  return 0;
}
